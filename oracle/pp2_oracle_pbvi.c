/*
 * pp2_oracle_pbvi.c -- CPU restatement of the reference's PBVI lower bound
 * (src/pomdp/point_based_value_iteration_cuda.cu).  TEST INFRASTRUCTURE ONLY
 * (see pp2_oracle.h): the product never links or calls this file.
 *
 * Arithmetic follows where each step runs in the reference:
 *   device (nvcc --use_fast_math: FTZ, contracted fma) -- cudaBayesBeliefUpdate
 *     (:88-133, orc_belief_update with ftz) and cudaComputeGammaOA (:297-341);
 *   host x86 (IEEE, no FMA) -- normalizeProbDensity (:135-145),
 *     sampleFromProbDensity (:147-163), the L1 distances (:238-246),
 *     inner_product (:610-622);
 *   cuBLAS (CUDA 8) -- Sgemm (:505-513) and Sgeam (:542-550).  cuBLAS's
 *     summation order is not published: the Sgemm dot product is pinned here
 *     as the x-ordered fmaf chain acc = fma(G[k][x], b[i][x], acc) from 0
 *     (PARITY UNPINNED against cuBLAS itself); Sgeam with alpha = beta = 1 is
 *     fl(x + y).
 * libstdc++'s heap algorithms (bits/stl_heap.h, unchanged since GCC 4.x) are
 * restated for the partial_sort call of :264-269 (see select_top below).
 */
#include "pp2_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static inline float ftz(float x) { return fabsf(x) < FLT_MIN ? copysignf(0.0f, x) : x; }

/* sampleFromProbDensity (:147-163): fp32 partial_sum, first index with
 * cdf >= r.  The reference returns n (past the end) when rounding leaves
 * cdf[n-1] < r and then reads out of bounds; here the last index whose
 * partial sum grew is taken instead (the same rule as the QV-tree sampler). */
static size_t sample_density(const float* d, size_t n, size_t stride, float r) {
  float acc = 0.0f, prev = 0.0f;
  size_t last = 0;
  for (size_t i = 0; i < n; ++i) {
    prev = acc;
    acc = acc + d[i * stride];
    if (acc >= r) return i;
    if (acc != prev) last = i;
  }
  return last;
}

static float rand_unit(orc_rand_state* rs) {
  return (float)orc_rand_next(rs) / ((float)2147483647 + 1.0f);  /* rand()/(RAND_MAX+1.0f) */
}

/* libstdc++ std::__adjust_heap / __push_heap / make_heap / sort_heap with
 * comp(i, j) = key[i] > key[j] (the lambda of :266-268). */
static int heap_comp(const float* key, size_t i, size_t j) { return key[i] > key[j]; }

static void push_heap_(size_t* f, long hole, long top, size_t v, const float* key) {
  long parent = (hole - 1) / 2;
  while (hole > top && heap_comp(key, f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}

static void adjust_heap_(size_t* f, long hole, long len, size_t v, const float* key) {
  const long top = hole;
  long child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (heap_comp(key, f[child], f[child - 1])) child--;
    f[hole] = f[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    f[hole] = f[child - 1];
    hole = child - 1;
  }
  push_heap_(f, hole, top, v, key);
}

/* partial_sort(idx.begin(), idx.end(), idx.begin()+100, comp) (:264-269) has
 * its middle and last arguments swapped: libstdc++ then runs
 * __heap_select(first, end, begin+100) -- make_heap over the whole range, an
 * empty selection loop -- and sort_heap(first, end): a full heap sort. */
void orc_heap_sort_desc(size_t n, const float* key, size_t* idx) {
  for (size_t i = 0; i < n; ++i) idx[i] = i;
  const long len = (long)n;
  if (len >= 2) {
    for (long parent = (len - 2) / 2;; --parent) {
      adjust_heap_(idx, parent, len, idx[parent], key);
      if (parent == 0) break;
    }
  }
  for (long last = len; last > 1;) {
    --last;
    size_t v = idx[last];
    idx[last] = idx[0];
    adjust_heap_(idx, 0, last, v, key);
  }
}

int orc_pbvi_belief_set(int H, int W, const float* T, const float* L, const float* b0,
                        int S, orc_rand_state* rs, float* b_set) {
  const size_t n = (size_t)H * W;
  if (S < 1) return -1;
  memcpy(b_set, b0, n * sizeof(float));
  int set_size = 1;
  float* cand = (float*)malloc(9 * n * sizeof(float));
  float* new_bs = (float*)malloc((size_t)S * n * sizeof(float));
  float* new_l1 = (float*)malloc((size_t)S * sizeof(float));
  size_t* order = (size_t*)malloc((size_t)S * sizeof(size_t));
  while (set_size < S) {
    for (int i = 0; i < set_size; ++i) {
      const float* bi = b_set + (size_t)i * n;
      float l1a[9];
      for (int a = 0; a < 9; ++a) {
        /* :212-222 -- three rand() calls per action, in this order */
        const float r1 = rand_unit(rs), r2 = rand_unit(rs), r3 = rand_unit(rs);
        const size_t s = sample_density(bi, n, 1, r1);
        const size_t nl = sample_density(T + 81 * s + 9 * a, 9, 1, r2);
        long ny = (long)(s / W) + (long)(nl / 3) - 1, nx = (long)(s % W) + (long)(nl % 3) - 1;
        /* out of the grid only when rand() == 0 picks a zero-probability
         * entry (the reference then indexes out of bounds): stay at s */
        if (ny < 0 || ny >= H || nx < 0 || nx >= W) ny = (long)(s / W), nx = (long)(s % W);
        const size_t ns = (size_t)ny * W + (size_t)nx;
        const int z = (int)sample_density(L + 16 * ns, 16, 1, r3);
        float* nb = cand + (size_t)a * n;
        orc_belief_update(H, W, T, L, bi, a, z, nb, 1);
        orc_normalize_seq(n, nb); /* :232-235 */
        float best = FLT_MAX;      /* :238-246 */
        for (int j = 0; j < set_size; ++j) {
          const float* bj = b_set + (size_t)j * n;
          float l1 = 0.0f;
          for (size_t k = 0; k < n; ++k) l1 += fabsf(nb[k] - bj[k]);
          if (l1 < best) best = l1;
        }
        l1a[a] = best;
      }
      int ba = 0; /* max_element: first maximum (:251-252) */
      for (int a = 1; a < 9; ++a)
        if (l1a[ba] < l1a[a]) ba = a;
      memcpy(new_bs + (size_t)i * n, cand + (size_t)ba * n, n * sizeof(float));
      new_l1[i] = l1a[ba];
    }
    if (set_size < 100) { /* :257-262 */
      const int m = set_size;
      for (int i = 0; i < m && set_size < S; ++i)
        memcpy(b_set + (size_t)(set_size++) * n, new_bs + (size_t)i * n, n * sizeof(float));
    } else { /* :263-276 */
      orc_heap_sort_desc((size_t)set_size, new_l1, order);
      for (int i = 0; i < 100 && set_size < S; ++i)
        memcpy(b_set + (size_t)(set_size++) * n, new_bs + order[i] * n, n * sizeof(float));
    }
  }
  free(cand);
  free(new_bs);
  free(new_l1);
  free(order);
  return 0;
}

int orc_pbvi_iterations(float gamma) {
  /* :440-441, evaluated in float as std::log(float) / std::ceil(float) do */
  return (int)(uint32_t)ceilf(logf(1.0e-3f / 5.0f) / logf(gamma));
}

/* cudaComputeGammaOA (:297-341) for one (a, o): out[k][x] for every alpha k */
static void gamma_ao(int H, int W, float gamma, const float* T, const float* L, int a, int o,
                     int S, const float* alphas, float* out) {
  const size_t n = (size_t)H * W;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const size_t idx = (size_t)y * W + x;
      float tm[9];
      int ok[9];
      for (int s = 0; s < 9; ++s) {
        const int sx = x + s % 3 - 1, sy = y + s / 3 - 1;
        tm[s] = T[81 * idx + 9 * a + s];
        ok[s] = !(sx < 0 || sx >= W || sy < 0 || sy >= H);
        if (ok[s]) tm[s] = ftz(tm[s] * L[16 * ((size_t)sy * W + sx) + o]);
      }
      for (int k = 0; k < S; ++k) {
        const float* al = alphas + (size_t)k * n;
        float acc = 0.0f;
        for (int s = 0; s < 9; ++s) {
          if (!ok[s]) continue;
          const size_t sidx = (size_t)(y + s / 3 - 1) * W + (x + s % 3 - 1);
          acc = ftz(fmaf(tm[s], ftz(al[sidx]), acc));
        }
        out[(size_t)k * n + idx] = ftz(gamma * acc);
      }
    }
}

int orc_pbvi_backup(int H, int W, float gamma, const float* T, const float* L, const float* R,
                    int S, const float* b_set, float* alphas, uint8_t* actions, int iterations) {
  const size_t n = (size_t)H * W;
  if (iterations <= 0) iterations = orc_pbvi_iterations(gamma);
  float* gao = (float*)malloc((size_t)S * n * sizeof(float));
  float* ga = (float*)malloc((size_t)9 * S * n * sizeof(float));
  int* kstar = (int*)malloc((size_t)S * sizeof(int));
  if (!gao || !ga || !kstar) return -1;
  for (int it = 0; it < iterations; ++it) {
    for (int a = 0; a < 9; ++a) {
      float* gaa = ga + (size_t)a * S * n;
      for (int i = 0; i < S; ++i) /* Gamma_a[a][i] = R[:, a] (:459-467) */
        for (size_t x = 0; x < n; ++x) gaa[(size_t)i * n + x] = R[9 * x + a];
      for (int o = 0; o < 16; ++o) {
        gamma_ao(H, W, gamma, T, L, a, o, S, alphas, gao);
        /* Sgemm (:505-513) + max_element per belief (:531-537) */
        for (int i = 0; i < S; ++i) {
          const float* bi = b_set + (size_t)i * n;
          int best = 0;
          float bv = 0.0f;
          for (int k = 0; k < S; ++k) {
            const float* g = gao + (size_t)k * n;
            float acc = 0.0f;
            for (size_t x = 0; x < n; ++x) acc = fmaf(g[x], bi[x], acc);
            if (k == 0 || bv < acc) { bv = acc; best = k; }
          }
          kstar[i] = best;
        }
        /* Sgeam: Gamma_a += alphas_ao_max (:542-550) */
        for (int i = 0; i < S; ++i) {
          const float* g = gao + (size_t)kstar[i] * n;
          float* d = gaa + (size_t)i * n;
          for (size_t x = 0; x < n; ++x) d[x] = d[x] + g[x];
        }
      }
    }
    /* action selection (:610-626) */
    for (int i = 0; i < S; ++i) {
      const float* bi = b_set + (size_t)i * n;
      float opt = -FLT_MAX;
      int oa = 0;
      for (int a = 0; a < 9; ++a) {
        const float* g = ga + ((size_t)a * S + i) * n;
        float v = 0.0f;
        for (size_t x = 0; x < n; ++x) v = v + bi[x] * g[x];
        if (v > opt) { opt = v; oa = a; }
      }
      memcpy(alphas + (size_t)i * n, ga + ((size_t)oa * S + i) * n, n * sizeof(float));
      actions[i] = (uint8_t)oa;
    }
  }
  free(gao);
  free(ga);
  free(kstar);
  return iterations;
}
