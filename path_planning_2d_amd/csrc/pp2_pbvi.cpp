// pp2_pbvi.cpp -- PBVI lower bound (C ABI pp2_pbvi_*, include/pp2.h).
//
// Restates src/pomdp/point_based_value_iteration_cuda.cu with every per-cell
// loop on the device and the model, belief set and alpha vectors resident in
// HBM.  The reference's per-(a,o) round trips -- Gamma_ao to the host
// (:406-427), back for the Sgemm (:497-503), the max-alpha gather on the host
// (:531-540) and back again -- become six launches per iteration, each over
// all 144 (a, o) pairs at once while their Gamma_ao fits the budget below:
//
//   Gamma_ao   k_pbvi_gamma_ao    G[a,o][k] for every alpha k           (HBM-bound)
//   Sgemm      k_gemm_nt          C[a,o][i][k] = <b_i, G[a,o][k]>       (MFMA f32)
//   max        k_argmax_rows      k*[a,o][i] = first argmax_k C[a,o][i][k]
//   Sgeam      k_pbvi_gamma_a     Gamma_a[i] = R_a + sum_o G[a,o][k*[a,o][i]]
//   values     k_rows_chain       V[a][i] = inner_product(b_i, Gamma_a[i])
//   select     k_pbvi_select      alpha_i = Gamma_a*[i], a* = first argmax_a V[a][i]
// The belief-set expansion (:165-295) keeps the reference's glibc rand()
// stream and arithmetic: the samples, the candidates' update and
// normalisation, and every L1 distance are batched over all (belief, action)
// pairs of a round.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "pp2_ctx.h"
#include "pp2_pbvi_internal.h"
#include "pp2_rand.h"

namespace pp2rt {

struct PbviState {
  int S = 0, Sp = 0, ld = 0, hw = 0;
  float* bset = nullptr;      // [Sp][ld] belief set
  float* alpha[2] = {nullptr, nullptr};  // [Sp][ld] alpha vectors (ping-pong)
  int acur = 0;
  uint8_t* actions = nullptr;  // [Sp]
  bool has_set = false;
  // backup scratch
  float* G = nullptr;    // [group*16][Sp][ld]  Gamma_ao of the actions in flight
  float* Ga = nullptr;   // [9][Sp][ld]         Gamma_a
  float* Cm = nullptr;   // [group*16][Sp][Sp]  <b_i, Gamma_ao_k>
  int* kstar = nullptr;  // [group*16][Sp]
  float* V = nullptr;    // [9][Sp]
};

namespace {

template <typename T>
int dalloc(T** p, size_t count, hipStream_t st) {
  if (*p) return PP2_OK;
  if (hipMalloc(p, count * sizeof(T)) != hipSuccess) {
    *p = nullptr;
    return set_err(PP2_ENOMEM, "hipMalloc %zu B (PBVI)", count * sizeof(T));
  }
  HIPCHK(hipMemsetAsync(*p, 0, count * sizeof(T), st));
  return PP2_OK;
}

template <typename T>
void dfree(T** p) {
  if (*p) (void)hipFree(*p);
  *p = nullptr;
}

int round_up(int v, int m) { return (v + m - 1) / m * m; }

constexpr int kMaxBeliefs = 4096;

int check_pbvi_ctx(pp2_ctx* c) {
  CHECK(check_model(c));
  if (c->nranks > 1 || c->group || c->g.rows != c->g.grows)
    return set_err(PP2_EINVAL, "PBVI runs on an unsharded context");
  return PP2_OK;
}

void free_scratch(PbviState* p) {
  dfree(&p->G);
  dfree(&p->Ga);
  dfree(&p->Cm);
  dfree(&p->kstar);
  dfree(&p->V);
}

// (Re)size the state for S beliefs; alphas and actions are zeroed.
int ensure_state(pp2_ctx* c, int S) {
  if (S < 1) return set_err(PP2_EINVAL, "belief set size must be >= 1");
  // the expansion's 9 n candidates index grid.y of the update / division
  // launches (< 65536); the reference node uses 500
  if (S > kMaxBeliefs) return set_err(PP2_EINVAL, "belief set size %d > %d", S, kMaxBeliefs);
  PbviState*& p = c->pbvi;
  if (!p) p = new PbviState();
  const int hw = c->g.rows * c->g.width;
  const int Sp = round_up(S, pp2::kGemmTile), ld = round_up(hw, pp2::kPbviChunk);
  if (p->Sp != Sp || p->ld != ld) {
    dfree(&p->bset);
    dfree(&p->alpha[0]);
    dfree(&p->alpha[1]);
    dfree(&p->actions);
    free_scratch(p);
  }
  p->S = S;
  p->Sp = Sp;
  p->ld = ld;
  p->hw = hw;
  const size_t rows = (size_t)Sp * ld;
  CHECK(dalloc(&p->bset, rows, c->stream));
  CHECK(dalloc(&p->alpha[0], rows, c->stream));
  CHECK(dalloc(&p->alpha[1], rows, c->stream));
  CHECK(dalloc(&p->actions, (size_t)Sp, c->stream));
  HIPCHK(hipMemsetAsync(p->alpha[0], 0, rows * sizeof(float), c->stream));
  HIPCHK(hipMemsetAsync(p->alpha[1], 0, rows * sizeof(float), c->stream));
  HIPCHK(hipMemsetAsync(p->actions, 0, (size_t)Sp, c->stream));
  p->acur = 0;
  ++c->pbvi_version;
  return PP2_OK;
}

// dst rows of ld floats <- host rows of hw floats (pad cells stay 0)
int upload_rows(pp2_ctx* c, float* dst, int ld, const float* src, int hw, int rows) {
  HIPCHK(hipMemcpy2DAsync(dst, (size_t)ld * sizeof(float), src, (size_t)hw * sizeof(float),
                          (size_t)hw * sizeof(float), rows, hipMemcpyHostToDevice, c->stream));
  return PP2_OK;
}

int download_rows(pp2_ctx* c, float* dst, const float* src, int ld, int hw, int rows) {
  HIPCHK(hipMemcpy2DAsync(dst, (size_t)hw * sizeof(float), src, (size_t)ld * sizeof(float),
                          (size_t)hw * sizeof(float), rows, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return PP2_OK;
}

struct SetScratch {
  float *cdf = nullptr, *cand = nullptr, *l1 = nullptr, *rnd = nullptr, *sums = nullptr,
        *best_l1 = nullptr;
  int *srow = nullptr, *best_a = nullptr;
  uint8_t *us = nullptr, *zs = nullptr;
  ~SetScratch() {
    dfree(&cdf);
    dfree(&cand);
    dfree(&l1);
    dfree(&rnd);
    dfree(&sums);
    dfree(&best_l1);
    dfree(&srow);
    dfree(&best_a);
    dfree(&us);
    dfree(&zs);
  }
};

// generateBeliefSet (:165-295).
int belief_set_impl(pp2_ctx* c, const float* b0, int S, uint32_t seed, uint64_t* rand_calls) {
  CHECK(ensure_state(c, S));
  PbviState* p = c->pbvi;
  p->has_set = false;
  const int hw = p->hw, ld = p->ld;
  const int maxc = 9 * S;  // candidates of the largest round (< 9 S)
  SetScratch w;
  CHECK(dalloc(&w.cdf, (size_t)p->Sp * ld, c->stream));
  CHECK(dalloc(&w.cand, (size_t)maxc * ld, c->stream));
  CHECK(dalloc(&w.l1, (size_t)maxc * S, c->stream));
  CHECK(dalloc(&w.rnd, (size_t)3 * maxc, c->stream));
  CHECK(dalloc(&w.sums, (size_t)maxc, c->stream));
  CHECK(dalloc(&w.best_l1, (size_t)S, c->stream));
  CHECK(dalloc(&w.srow, (size_t)maxc, c->stream));
  CHECK(dalloc(&w.best_a, (size_t)S, c->stream));
  CHECK(dalloc(&w.us, (size_t)maxc, c->stream));
  CHECK(dalloc(&w.zs, (size_t)maxc, c->stream));
  {
    std::vector<int> srow(maxc);
    std::vector<uint8_t> us(maxc);
    for (int k = 0; k < maxc; ++k) {
      srow[k] = k / 9;
      us[k] = (uint8_t)(k % 9);
    }
    HIPCHK(hipMemcpyAsync(w.srow, srow.data(), maxc * sizeof(int), hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(hipMemcpyAsync(w.us, us.data(), maxc, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  CHECK(upload_rows(c, p->bset, ld, b0, hw, 1));
  HIPCHK(pp2::launch_rows_seq(c->stream, pp2::ROW_CDF, p->bset, ld, 1, hw, nullptr, w.cdf));

  GlibcRand rng;
  rng.seed(seed);
  std::vector<float> rnd;
  std::vector<float> best_l1(S);
  std::vector<int> best_a(S);
  int set_size = 1;
  while (set_size < S) {
    const int n = set_size, nc = 9 * n;
    rnd.resize((size_t)3 * nc);
    for (float& r : rnd) r = rng.unit();  // (i, a, {state, next state, observation})
    HIPCHK(hipMemcpyAsync(w.rnd, rnd.data(), rnd.size() * sizeof(float), hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(pp2::launch_pbvi_sample(c->stream, c->g, c->T.v, c->L.v, w.cdf, ld, n, w.rnd, w.zs,
                                   nullptr));
    HIPCHK(pp2::launch_pbvi_update(c->stream, c->g, c->T.v, c->L.v, p->bset, ld, w.srow, w.us,
                                   w.zs, nc, w.cand));
    HIPCHK(pp2::launch_rows_seq(c->stream, pp2::ROW_SUM, w.cand, ld, nc, hw, w.sums, nullptr));
    HIPCHK(pp2::launch_rows_div(c->stream, w.cand, ld, nc, hw, w.sums));
    HIPCHK(pp2::launch_pair_chain(c->stream, pp2::PAIR_L1, w.cand, nc, p->bset, n, ld, hw, w.l1,
                                  S));
    HIPCHK(pp2::launch_pbvi_pick(c->stream, w.l1, S, n, n, w.best_l1, w.best_a));
    HIPCHK(hipMemcpyAsync(best_l1.data(), w.best_l1, n * sizeof(float), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipMemcpyAsync(best_a.data(), w.best_a, n * sizeof(int), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));

    std::vector<size_t> order(n);
    std::iota(order.begin(), order.end(), 0);
    int take = n;
    if (n >= 100) {
      // partial_sort(idx.begin(), idx.end(), idx.begin() + 100, comp) (:264-269)
      // has its middle and last swapped; libstdc++ then heap-sorts the whole
      // range: make_heap + sort_heap with the same comparator.
      auto comp = [&](size_t a, size_t b) { return best_l1[a] > best_l1[b]; };
      std::make_heap(order.begin(), order.end(), comp);
      std::sort_heap(order.begin(), order.end(), comp);
      take = 100;
    }
    const int first_new = set_size;
    for (int k = 0; k < take && set_size < S; ++k) {
      const size_t i = order[k];
      HIPCHK(hipMemcpyAsync(p->bset + (size_t)set_size * ld,
                            w.cand + (size_t)(9 * i + best_a[i]) * ld, (size_t)ld * sizeof(float),
                            hipMemcpyDeviceToDevice, c->stream));
      ++set_size;
    }
    HIPCHK(pp2::launch_rows_seq(c->stream, pp2::ROW_CDF, p->bset + (size_t)first_new * ld, ld,
                                set_size - first_new, hw, nullptr,
                                w.cdf + (size_t)first_new * ld));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  p->has_set = true;
  if (rand_calls) *rand_calls = rng.calls;
  return PP2_OK;
}

// Actions whose Gamma_ao slices are resident at once: all 9 (one GEMM
// launch of 144 batches) when they fit kGaoBudget bytes, else fewer.
constexpr size_t kGaoBudget = size_t(48) << 30;

int backup_impl(pp2_ctx* c, int iterations) {
  PbviState* p = c->pbvi;
  if (!p || !p->has_set) return set_err(PP2_ESTATE, "no PBVI belief set");
  if (iterations <= 0)  // :440-441, in float like std::log(float) / std::ceil(float)
    iterations = (int)(uint32_t)std::ceil(std::log(1.0e-3f / 5.0f) / std::log(c->gamma));
  const int S = p->S, Sp = p->Sp, ld = p->ld, hw = p->hw;
  const long long gstride = (long long)Sp * ld;
  const size_t per_action = (size_t)16 * gstride * sizeof(float);
  const int group = (int)std::max<size_t>(1, std::min<size_t>(9, kGaoBudget / per_action));
  CHECK(dalloc(&p->G, (size_t)16 * group * gstride, c->stream));
  CHECK(dalloc(&p->Ga, (size_t)9 * gstride, c->stream));
  CHECK(dalloc(&p->Cm, (size_t)16 * group * Sp * Sp, c->stream));
  CHECK(dalloc(&p->kstar, (size_t)16 * group * Sp, c->stream));
  CHECK(dalloc(&p->V, (size_t)9 * Sp, c->stream));
  for (int it = 0; it < iterations; ++it) {
    const float* al = p->alpha[p->acur];
    for (int a0 = 0; a0 < 9; a0 += group) {
      const int a1 = std::min(9, a0 + group), nb = 16 * (a1 - a0);
      HIPCHK(pp2::launch_pbvi_gamma_ao(c->stream, c->g, c->gamma, c->T.v, c->L.v, al, ld, S, a0,
                                       a1, p->G, gstride));
      HIPCHK(pp2::launch_gemm_nt(c->stream, p->bset, p->G, p->Cm, Sp, Sp, ld, nb, gstride,
                                 (long long)Sp * Sp, 1, 0));
      HIPCHK(pp2::launch_argmax_rows(c->stream, p->Cm, nb * Sp, S, Sp, p->kstar, nullptr));
      HIPCHK(pp2::launch_pbvi_gamma_a(c->stream, c->g, c->R.v, p->G, gstride, ld, S, a0, a1,
                                      p->kstar, Sp, p->Ga));
    }
    HIPCHK(pp2::launch_rows_dot(c->stream, p->bset, Sp, p->Ga, ld, 9 * Sp, hw, p->V));
    HIPCHK(pp2::launch_pbvi_select(c->stream, p->V, p->Ga, Sp, S, ld, p->alpha[p->acur ^ 1],
                                   p->actions));
    p->acur ^= 1;
    ++c->pbvi_version;
  }
  return PP2_OK;
}

}  // namespace

void pbvi_free(pp2_ctx* c) {
  PbviState* p = c->pbvi;
  if (!p) return;
  dfree(&p->bset);
  dfree(&p->alpha[0]);
  dfree(&p->alpha[1]);
  dfree(&p->actions);
  free_scratch(p);
  delete p;
  c->pbvi = nullptr;
}

int pbvi_alphas(pp2_ctx* c, const float** alpha, int* S, int* Sp, int* ld) {
  PbviState* p = c->pbvi;
  if (!p || p->S <= 0) return set_err(PP2_ESTATE, "no PBVI alpha vectors");
  *alpha = p->alpha[p->acur];
  *S = p->S;
  *Sp = p->Sp;
  *ld = p->ld;
  return PP2_OK;
}

int pbvi_eval_device(pp2_ctx* c, int n, const float* d_beliefs, int ld, float* d_dots) {
  PbviState* p = c->pbvi;
  HIPCHK(pp2::launch_pair_chain(c->stream, pp2::PAIR_DOT, d_beliefs, n, p->alpha[p->acur], p->S,
                                ld, p->hw, d_dots, p->S));
  return PP2_OK;
}

}  // namespace pp2rt

using namespace pp2rt;

int pp2_pbvi_belief_set(pp2_ctx* c, const float* b0, uint32_t set_size, uint32_t rand_seed,
                        uint64_t* rand_calls) {
  CHECK(check_pbvi_ctx(c));
  if (!b0) return set_err(PP2_EINVAL, "null initial belief");
  DeviceGuard dg(c->device);
  return belief_set_impl(c, b0, (int)set_size, rand_seed, rand_calls);
}

int pp2_pbvi_set_beliefs(pp2_ctx* c, uint32_t set_size, const float* beliefs) {
  CHECK(check_pbvi_ctx(c));
  if (!beliefs) return set_err(PP2_EINVAL, "null beliefs");
  DeviceGuard dg(c->device);
  CHECK(ensure_state(c, (int)set_size));
  PbviState* p = c->pbvi;
  CHECK(upload_rows(c, p->bset, p->ld, beliefs, p->hw, p->S));
  HIPCHK(hipStreamSynchronize(c->stream));
  p->has_set = true;
  return PP2_OK;
}

int pp2_pbvi_get_beliefs(pp2_ctx* c, float* beliefs) {
  CHECK(check_ctx(c));
  PbviState* p = c->pbvi;
  if (!p || !p->has_set) return set_err(PP2_ESTATE, "no PBVI belief set");
  DeviceGuard dg(c->device);
  return download_rows(c, beliefs, p->bset, p->ld, p->hw, p->S);
}

int pp2_pbvi_backup(pp2_ctx* c, int iterations) {
  CHECK(check_pbvi_ctx(c));
  DeviceGuard dg(c->device);
  return backup_impl(c, iterations);
}

int pp2_pbvi_solve(pp2_ctx* c, const float* b0, uint32_t set_size, uint32_t rand_seed,
                   uint64_t* rand_calls) {
  CHECK(pp2_pbvi_belief_set(c, b0, set_size, rand_seed, rand_calls));
  DeviceGuard dg(c->device);
  CHECK(backup_impl(c, 0));
  HIPCHK(hipStreamSynchronize(c->stream));
  return PP2_OK;
}

int pp2_pbvi_info(pp2_ctx* c, uint32_t* set_size, int* has_beliefs) {
  CHECK(check_ctx(c));
  PbviState* p = c->pbvi;
  if (set_size) *set_size = p ? (uint32_t)p->S : 0;
  if (has_beliefs) *has_beliefs = p && p->has_set;
  return PP2_OK;
}

int pp2_pbvi_get(pp2_ctx* c, float* alphas, uint8_t* actions) {
  CHECK(check_ctx(c));
  PbviState* p = c->pbvi;
  if (!p) return set_err(PP2_ESTATE, "no PBVI state");
  DeviceGuard dg(c->device);
  if (alphas) CHECK(download_rows(c, alphas, p->alpha[p->acur], p->ld, p->hw, p->S));
  if (actions) {
    HIPCHK(hipMemcpyAsync(actions, p->actions, p->S, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  return PP2_OK;
}

int pp2_pbvi_set(pp2_ctx* c, uint32_t set_size, const float* alphas, const uint8_t* actions) {
  CHECK(check_pbvi_ctx(c));
  if (!alphas || !actions) return set_err(PP2_EINVAL, "null alphas / actions");
  for (uint32_t i = 0; i < set_size; ++i)
    if (actions[i] > 8) return set_err(PP2_EINVAL, "action %u of alpha %u out of range", actions[i], i);
  DeviceGuard dg(c->device);
  const bool keep_set = c->pbvi && c->pbvi->has_set && c->pbvi->S == (int)set_size;
  CHECK(ensure_state(c, (int)set_size));
  PbviState* p = c->pbvi;
  p->has_set = keep_set;
  CHECK(upload_rows(c, p->alpha[p->acur], p->ld, alphas, p->hw, p->S));
  ++c->pbvi_version;
  HIPCHK(hipMemcpyAsync(p->actions, actions, set_size, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return PP2_OK;
}

int pp2_pbvi_evaluate(pp2_ctx* c, int n, const float* beliefs, float* values, uint8_t* actions) {
  CHECK(check_ctx(c));
  PbviState* p = c->pbvi;
  if (!p) return set_err(PP2_ESTATE, "no PBVI alpha vectors");
  if (n < 0 || (n > 0 && !beliefs)) return set_err(PP2_EINVAL, "bad belief batch");
  if (n == 0) return PP2_OK;
  DeviceGuard dg(c->device);
  const int ld = p->ld;
  float *d_b = nullptr, *d_dots = nullptr, *d_v = nullptr;
  int* d_i = nullptr;
  struct Free {
    float **a, **b, **c;
    int** d;
    ~Free() {
      dfree(a);
      dfree(b);
      dfree(c);
      dfree(d);
    }
  } fr{&d_b, &d_dots, &d_v, &d_i};
  CHECK(dalloc(&d_b, (size_t)n * ld, c->stream));
  CHECK(dalloc(&d_dots, (size_t)n * p->S, c->stream));
  CHECK(dalloc(&d_v, (size_t)n, c->stream));
  CHECK(dalloc(&d_i, (size_t)n, c->stream));
  CHECK(upload_rows(c, d_b, ld, beliefs, p->hw, n));
  CHECK(pbvi_eval_device(c, n, d_b, ld, d_dots));
  HIPCHK(pp2::launch_argmax_rows(c->stream, d_dots, n, p->S, p->S, d_i, d_v));
  std::vector<int> idx(n);
  std::vector<uint8_t> act(p->S);
  HIPCHK(hipMemcpyAsync(idx.data(), d_i, n * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(act.data(), p->actions, p->S, hipMemcpyDeviceToHost, c->stream));
  if (values)
    HIPCHK(hipMemcpyAsync(values, d_v, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (actions)
    for (int i = 0; i < n; ++i) actions[i] = act[idx[i]];
  return PP2_OK;
}

// savePbviDataToFile / loadPbviDataFromFile (:737-797): one alpha vector per
// line ("%15.8f" per cell) in dir/pbvi_alphas, one "%10u" action per line in
// dir/pbvi_actions.  The loader reads each action as an unsigned int and
// stores it as uint8 (the reference scans "%u" straight into uint8_t storage).
int pp2_pbvi_save(pp2_ctx* c, const char* dir) {
  CHECK(check_ctx(c));
  PbviState* p = c->pbvi;
  if (!p) return set_err(PP2_ESTATE, "no PBVI alpha vectors");
  std::vector<float> al((size_t)p->S * p->hw);
  std::vector<uint8_t> act(p->S);
  CHECK(pp2_pbvi_get(c, al.data(), act.data()));
  CHECK(write_text(join(dir, "pbvi_alphas"), al, p->hw));
  const std::string path = join(dir, "pbvi_actions");
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return set_err(PP2_EIO, "cannot open %s for writing", path.c_str());
  for (uint8_t a : act) fprintf(f, "%10u\n", (unsigned)a);
  if (fclose(f) != 0) return set_err(PP2_EIO, "write %s failed", path.c_str());
  return PP2_OK;
}

int pp2_pbvi_load(pp2_ctx* c, const char* dir, uint32_t set_size) {
  CHECK(check_pbvi_ctx(c));
  if (set_size < 1) return set_err(PP2_EINVAL, "belief set size must be >= 1");
  const size_t hw = owned_cells(c);
  std::vector<float> al((size_t)set_size * hw);
  CHECK(read_text(join(dir, "pbvi_alphas"), al));
  std::vector<uint8_t> act(set_size);
  CHECK(read_actions(join(dir, "pbvi_actions"), act));
  return pp2_pbvi_set(c, set_size, al.data(), act.data());
}
