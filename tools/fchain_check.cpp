// fchain_check.cpp -- CPU check of the exact parallel fp32 chain
// (path_planning_2d_amd/csrc/pp2_fchain.h) against the plain sequential
// chain, on adversarial inputs.  It restates the device algorithm's structure
// (chunk tables from an approximate running sum, a driver that applies 64
// chunk entries per step by a prefix scan and adds failing chunks term by
// term) so that the logic is exercised without a GPU.  Built and run by
// tests/test_fchain_cpu.py:
//   g++ -O2 -std=c++17 -ffp-contract=off -I path_planning_2d_amd/csrc tools/fchain_check.cpp
// Exit status 0 = every case bit-exact.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <cmath>
#include <random>
#include <vector>

#include "pp2_fchain.h"

using namespace pp2::fchain;

static float seq_sum(const std::vector<float>& t) {
  float s = 0.0f;
  for (float v : t) s = s + v;
  return s;
}

static long g_exact_fail = 0;

struct Stats {
  long chunks = 0, fallback = 0, planned = 0;
};

static long g_plan_fail = 0;

// k_fc_tables' crossing plan of the terms [x0, x1) from the approximate sum
// before them (sp), followed from the state (E, k) as k_fc_walk does: true
// with the state after the chunk when every check passes.
static bool follow_plan(const std::vector<float>& t, int x0, int x1, float sp, int* pE, int* pk) {
  const int E0 = domain_of(sp);
  float a = sp;
  int prev = E0, nc = 0, D[4] = {E0, 0, 0, 0};
  float ts[4] = {0, 0, 0, 0}, d[4] = {0, 0, 0, 0};
  for (int x = x0; x < x1; ++x) {
    a += fabsf(t[x]);
    const int Dx = domain_of(a);
    if (Dx > prev) {  // a crossing term
      if (++nc > 3) return false;
      D[nc] = Dx;
      ts[nc] = fabsf(t[x]);
    } else {
      bool tie;
      d[nc] += units_of(fabsf(t[x]), Dx, &tie);
      if (tie) return false;
    }
    prev = Dx;
  }
  if (nc < 1) return false;
  for (int sg = 0; sg <= nc; ++sg)
    if (!(d[sg] < (float)kK24) || (sg > 0 && (D[sg] - E0 < 1 || D[sg] - E0 > 15))) return false;
  if (*pE != E0) return false;
  int Ep = *pE, kp = *pk + (int)d[0];
  if (kp > kK24) return false;
  for (int sg = 1; sg <= nc; ++sg) {
    const float sv = value_of(Ep, kp) + ts[sg];
    state_of(sv, &Ep, &kp);
    kp += (int)d[sg];
    if (Ep != D[sg] || kp > kK24) return false;
  }
  *pE = Ep;
  *pk = kp;
  return true;
}

// The device algorithm, chunk = `chunk` terms.
static float fchain_sum(const std::vector<float>& t, int chunk, Stats* st) {
  const int n = (int)t.size();
  if (n == 0) return 0.0f;
  bool pos = false, neg = false, bad = false;
  for (float v : t) {
    if (!std::isfinite(v)) bad = true;
    else if (v > 0.0f) pos = true;
    else if (v < 0.0f) neg = true;
  }
  if (bad || (pos && neg)) return seq_sum(t);
  const int nch = (n + chunk - 1) / chunk;
  // pass 1: approximate chunk sums of |t|, exclusive prefix
  std::vector<float> P(nch);
  float run = 0.0f;
  for (int j = 0; j < nch; ++j) {
    P[j] = run;
    float a = 0.0f;
    for (int x = j * chunk; x < n && x < (j + 1) * chunk; ++x) a += fabsf(t[x]);
    run += a;
  }
  // pass 2: tables (the increment sum in any order: here reversed)
  std::vector<uint32_t> tab(nch);
  for (int j = 0; j < nch; ++j) {
    const int E = domain_of(P[j]);
    float d = 0.0f, mx = 0.0f;
    bool tie = false;
    const int x1 = std::min(n, (j + 1) * chunk);
    for (int x = x1 - 1; x >= j * chunk; --x) {
      bool tx;
      d += units_of(fabsf(t[x]), E, &tx);
      tie |= tx;
      mx = std::max(mx, fabsf(t[x]));
    }
    // a chunk adding nothing: tabled for the lowest domain where it adds
    // nothing (k_fc_tables' zero_domain)
    int Ez = E;
    if (d == 0.0f) {
      const uint32_t b = bits_of(mx);
      const int et = (int)(b >> 23);
      Ez = b == 0u ? kEMin : std::max((et == 0 ? -127 : et - 127) + 25, kEMin);
    }
    tab[j] = make_entry(std::min(E, Ez), d, tie);
  }
  // driver: 64 chunks per step
  int E = kEMin, k = 0;
  int j = 0;
  while (j < nch) {
    int incl[64];
    bool ok[64];
    int acc = 0;
    for (int l = 0; l < 64; ++l) {
      const int jj = j + l;
      const uint32_t e = jj < nch ? tab[jj] : kNoEntry;
      const bool valid = entry_applies(e, E);
      acc += valid ? entry_units(e) : 0;
      incl[l] = acc;
      ok[l] = valid && k + acc <= kK24;
    }
    int f = 0;
    while (f < 64 && ok[f]) ++f;
    if (f > 0) {
      k += incl[f - 1];
      normalise(&E, &k);
    }
    st->chunks += f;
    j += f;
    if (j < nch && f < 64) {
      // the chunk's crossing plan (k_fc_tables' chunk_plan, followed as
      // k_fc_walk does): where its checks pass, its state must be the
      // term-by-term one below
      const int x1p = std::min(n, (j + 1) * chunk);
      int Ep = E, kp = k;
      const bool planned = follow_plan(t, j * chunk, x1p, P[j], &Ep, &kp);
      // the failing chunk term by term, each increment applied exactly
      // (add_exact: the device's per-element scan) -- and checked against
      // the plain fp32 adds
      float s = value_of(E, k);
      const int x1 = std::min(n, (j + 1) * chunk);
      int E2 = E, k2 = k;
      for (int x = j * chunk; x < x1; ++x) {
        s = s + fabsf(t[x]);
        add_exact(&E2, &k2, fabsf(t[x]));
        if (bits_of(value_of(E2, k2)) != bits_of(s)) ++g_exact_fail;
      }
      state_of(s, &E, &k);
      if (planned) {
        ++st->planned;
        normalise(&Ep, &kp);
        int En = E, kn = k;
        normalise(&En, &kn);
        if (Ep != En || kp != kn) ++g_plan_fail;
      }
      ++st->chunks;
      ++st->fallback;
      ++j;
    }
  }
  const float r = value_of(E, k);
  if (neg) return r == 0.0f ? 0.0f : -r;
  return r;
}

static int fails = 0;

// The running sums (cdf) of a non-negative chain, every one of them from
// add_exact from the chain start, against the plain fp32 running sums.
static void check_cdf(const std::vector<float>& t) {
  for (float v : t)
    if (!(v >= 0.0f) || !std::isfinite(v)) return;
  float s = 0.0f;
  int E = kEMin, k = 0;
  for (float v : t) {
    s = s + v;
    add_exact(&E, &k, v);
    if (bits_of(value_of(E, k)) != bits_of(s)) {
      ++g_exact_fail;
      return;
    }
  }
}

static void check(const char* what, const std::vector<float>& t, int chunk, Stats* st) {
  const float a = seq_sum(t), b = fchain_sum(t, chunk, st);
  check_cdf(t);
  if (bits_of(a) != bits_of(b) && !(std::isnan(a) && std::isnan(b))) {
    if (fails < 20)
      printf("MISMATCH %s n=%zu chunk=%d: seq %.9g (0x%08x) fchain %.9g (0x%08x)\n", what,
             t.size(), chunk, a, bits_of(a), b, bits_of(b));
    ++fails;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<float> U(0.0f, 1.0f);
  Stats st;
  const int chunks[] = {1, 4, 64, 256, 1000};
  for (int rep = 0; rep < reps; ++rep) {
    const int n = (int)(rng() % 70000);
    const int chunk = chunks[rng() % 5];
    std::vector<float> t(n);
    const int kind = rep % 10;
    for (int x = 0; x < n; ++x) {
      float v = 0.0f;
      switch (kind) {
        case 0: v = U(rng); break;                                       // uniform
        case 1: v = ldexpf(U(rng), -(int)(rng() % 60)); break;           // wide range
        case 2: v = 1.0f / 52429.0f; break;                              // constant
        case 3: v = (rng() % 7 == 0) ? U(rng) * 1e-5f : 0.0f; break;     // sparse
        case 4: v = -U(rng) * 37.0f; break;                              // non-positive
        case 5: v = ldexpf((float)(rng() % 8), -20); break;              // few bits: ties
        case 6: v = ldexpf(U(rng), -140); break;                         // subnormal range
        case 7: v = (rng() % 2 ? 1.0f : -1.0f) * U(rng); break;          // mixed sign
        case 8: v = (x % 3 == 0) ? -0.0f : -ldexpf(U(rng), -10); break;  // -0 and negatives
        case 9: v = x == n / 2 ? 1e30f : U(rng) * 1e-3f; break;          // one huge term
      }
      t[x] = v;
    }
    check("random", t, chunk, &st);
  }
  // ties by construction: s = 1 (k = 2^23 at E = 0), terms of half an ulp
  {
    std::vector<float> t(1, 1.0f);
    for (int i = 0; i < 5000; ++i) t.push_back(ldexpf(1.0f, -24));
    for (int c : chunks) check("half-ulp ties", t, c, &st);
    t.assign(1, 1.0f + ldexpf(1.0f, -23));
    for (int i = 0; i < 5000; ++i) t.push_back(ldexpf(1.0f, -24) * (i % 3 == 0 ? 3.0f : 1.0f));
    for (int c : chunks) check("tie parity", t, c, &st);
  }
  // crossing exactly onto a power of two, then tiny terms
  {
    std::vector<float> t = {0.5f, 0.25f, 0.25f};
    for (int i = 0; i < 3000; ++i) t.push_back(ldexpf(1.0f, -25));
    for (int c : chunks) check("onto 2^k", t, c, &st);
  }
  // a concentrated, normalised belief: the exact sum ends at or next to 1.0,
  // the approximate one on the other side, then a long tail far below half an
  // ulp (entries of d = 0 tabled for the binade below: entry_applies)
  for (int rep = 0; rep < 40; ++rep) {
    const int m = 50 + (int)(rng() % 3000);
    std::vector<float> t;
    float s = 0.0f;
    for (int i = 0; i < m; ++i) t.push_back(U(rng)), s = s + t.back();
    for (float& v : t) v = v / s;
    for (int i = 0; i < 60000; ++i)
      t.push_back(rep % 2 ? ldexpf(U(rng), -40) : (i % 7 ? 0.0f : ldexpf(1.0f, -26)));
    for (int c : chunks) check("concentrated + tail", t, c, &st);
  }
  // ties one by one: a term of (m + 1/2) ulps on a random state -- the
  // increment by k's parity (tie_increment) against the fp32 add
  for (int rep = 0; rep < 2000000; ++rep) {
    const int E = -126 + (int)(rng() % 250);
    const int k = (E == kEMin ? 0 : (1 << 23)) + (int)(rng() % (1u << 23));
    const int m = (int)(rng() % 5 == 0 ? rng() % 4 : rng() % (1u << (rng() % 23)));
    const float t = ldexpf((float)m + 0.5f, E - 23);
    if (!std::isfinite(t) || t == 0.0f) continue;
    int E2 = E, k2 = k;
    add_exact(&E2, &k2, t);
    const float want = value_of(E, k) + t;
    if (bits_of(value_of(E2, k2)) != bits_of(want)) {
      if (g_exact_fail < 5) printf("TIE E=%d k=%d m=%d\n", E, k, m);
      ++g_exact_fail;
    }
  }
  // all zeros, -0, empty, single
  {
    std::vector<float> z(1000, 0.0f), mz(1000, -0.0f), e, one(1, -3.5f);
    for (int c : chunks) {
      check("zeros", z, c, &st);
      check("-zeros", mz, c, &st);
      check("empty", e, c, &st);
      check("single", one, c, &st);
    }
  }
  // a belief-like sum: uniform over 65536 cells, and products with alphas
  {
    std::vector<float> b(65536), d(65536);
    for (int i = 0; i < 65536; ++i) b[i] = 1.0f / 52429.0f * (i % 5 ? 1.0f : 0.0f);
    for (int i = 0; i < 65536; ++i) d[i] = b[i] * -(20.0f + 20.0f * U(rng));
    check("belief", b, 256, &st);
    check("belief dot", d, 256, &st);
  }
  printf("fchain_check: %d mismatches; %ld chunks, %ld term-by-term (%.2f %%), %ld of them "
         "planned; %ld add_exact mismatches, %ld plan mismatches\n", fails, st.chunks,
         st.fallback, st.chunks ? 100.0 * st.fallback / st.chunks : 0.0, st.planned, g_exact_fail,
         g_plan_fail);
  return fails || g_exact_fail || g_plan_fail ? 1 : 0;
}
