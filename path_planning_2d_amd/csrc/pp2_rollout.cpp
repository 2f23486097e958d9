// pp2_rollout.cpp -- batched fp16 QV-tree rollouts (C ABI pp2_rollout_*).
//
// Host driver of k_rollout_band (pp2_rollout_dev.hip) and the leaf pass
// (k_rollout_leaf_mfma there, or k_rollout_leaf in pp2_kernels.hip for rows
// that are not 16-B aligned): groups the copies of every step by action (chunks of
// rollout_chunk() copies sharing u, so a wave gathers its T_u stencil terms
// once for all of them), chains the depth steps
// on the context's stream, and turns the per-copy {stored sum, stored max,
// reward dot} statistics into rewards, observation likelihoods and values.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "pp2_ctx.h"

using namespace pp2rt;

namespace {
constexpr int kMaxChunk = 64;  // bound on rollout_chunk() (chunk padding room)
constexpr int kRollStats = 3;
constexpr int kLeafStats = 10;
}  // namespace

struct pp2_rollout {
  pp2_ctx* ctx = nullptr;
  int copies = 0, depth = 0;
  long long cstride = 0;           // halfs per copy plane (rows+2 rows)
  void* alloc[2] = {nullptr, nullptr};  // allocations (64-B guard in front)
  void* buf[2] = {nullptr, nullptr};    // copy 0's plane (row -1) in each
  float* d_stats = nullptr;        // [depth+1][copies][3]
  float* d_leaf = nullptr;         // [copies][10]
  float* d_partials = nullptr;     // [copies][waves][10]
  void* d_leafmm = nullptr;        // the MFMA leaf pass's scratch (null: the fmaf pass)
  unsigned leaf_fib_version = 0;   // the context's fib_version packed into it (0: none)
  int leaf_fcur = -1;              // ... and the FIB buffer it came from
  int* d_chunks = nullptr;         // per step: u[], first[], n[] (maxchunks each), copies[]
  uint8_t* d_zs = nullptr;         // [depth][copies]
  int maxchunks = 0;
  std::vector<int> nchunks;        // per step
  bool ran = false;
  _Float16* d_root = nullptr;      // one fp16 plane image
};

extern "C" {

int pp2_rollout_destroy(pp2_rollout* r) {
  if (!r) return PP2_OK;
  DeviceGuard dg(r->ctx->device);
  (void)hipStreamSynchronize(r->ctx->stream);
  for (void* p : {r->alloc[0], r->alloc[1], (void*)r->d_stats, (void*)r->d_leaf,
                  (void*)r->d_partials, (void*)r->d_chunks, (void*)r->d_zs, (void*)r->d_root,
                  r->d_leafmm})
    if (p) (void)hipFree(p);
  delete r;
  return PP2_OK;
}

int pp2_rollout_create(pp2_rollout** out, pp2_ctx* c, int copies, int depth) {
  if (!out) return set_err(PP2_EINVAL, "out is null");
  *out = nullptr;
  CHECK(check_model(c));
  if (copies < 1 || depth < 1) return set_err(PP2_EINVAL, "copies and depth must be >= 1");
  // chunks of >= 4 copies index grid.y of the step launch (< 65536)
  if (copies > 131072) return set_err(PP2_EINVAL, "copies %d > 131072", copies);
  if (c->nranks > 1 || c->group || c->g.rows != c->g.grows)
    return set_err(PP2_EINVAL, "rollouts need an unsharded context");
  DeviceGuard dg(c->device);
  pp2_rollout* r = new pp2_rollout();
  r->ctx = c;
  r->copies = copies;
  r->depth = depth;
  r->cstride = (long long)(c->g.rows + 2) * c->g.wp + 16;  // + guard, keeps copies 32-B aligned
  r->maxchunks = copies / pp2::rollout_min_chunk() + 9 + 1;
  const size_t bbytes = (size_t)r->cstride * copies * sizeof(_Float16) + 128;
  const int nw = pp2::rollout_waves(c->g);
  auto fail = [&](int s) {
    pp2_rollout_destroy(r);
    return s;
  };
  if (hipMalloc(&r->alloc[0], bbytes) != hipSuccess || hipMalloc(&r->alloc[1], bbytes) != hipSuccess)
    return fail(set_err(PP2_ENOMEM, "rollout beliefs: 2 x %zu bytes", bbytes));
  for (int i = 0; i < 2; ++i) r->buf[i] = (char*)r->alloc[i] + 64;
  if (hipMemsetAsync(r->alloc[0], 0, bbytes, c->stream) != hipSuccess ||
      hipMemsetAsync(r->alloc[1], 0, bbytes, c->stream) != hipSuccess ||
      hipMalloc(&r->d_stats, (size_t)(depth + 1) * copies * kRollStats * sizeof(float)) != hipSuccess ||
      hipMalloc(&r->d_leaf, (size_t)copies * kLeafStats * sizeof(float)) != hipSuccess ||
      hipMalloc(&r->d_partials, (size_t)copies * nw * kLeafStats * sizeof(float)) != hipSuccess ||
      hipMalloc(&r->d_chunks, (size_t)depth * (3 * r->maxchunks + copies + 9 * kMaxChunk) * sizeof(int)) != hipSuccess ||
      hipMalloc(&r->d_zs, (size_t)depth * copies) != hipSuccess ||
      hipMalloc(&r->d_root, (size_t)r->cstride * sizeof(_Float16)) != hipSuccess)
    return fail(set_err(PP2_ENOMEM, "rollout scratch"));
  if (pp2::rollout_leaf_mfma_ok(c->g, r->cstride) &&
      hipMalloc(&r->d_leafmm, pp2::rollout_leaf_scratch_bytes(c->g, copies)) != hipSuccess)
    return fail(set_err(PP2_ENOMEM, "rollout leaf scratch"));
  *out = r;
  return PP2_OK;
}

int pp2_rollout_set_root(pp2_rollout* r, const float* belief) {
  if (!r || !belief) return set_err(PP2_EINVAL, "null argument");
  pp2_ctx* c = r->ctx;
  DeviceGuard dg(c->device);
  const int H = c->g.rows, W = c->g.width, wp = c->g.wp;
  float mx = 0.0f;
  for (size_t i = 0; i < (size_t)H * W; ++i) mx = std::max(mx, belief[i]);
  if (!(mx > 0.0f)) return set_err(PP2_EINVAL, "root belief has no positive mass");
  // fp16 image of b/max (row -1 and row H are the zero halo rows)
  std::vector<_Float16> img((size_t)r->cstride, (_Float16)0.0f);
  double s = 0.0;
  float m = 0.0f;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const _Float16 h = (_Float16)(belief[(size_t)y * W + x] / mx);
      img[(size_t)(y + 1) * wp + x] = h;
      s += (double)(float)h;
      m = std::max(m, (float)h);
    }
  // no per-copy broadcast: the first step of every run reads this one image
  // for all copies (an L2-resident input), then the copies diverge
  HIPCHK(hipMemcpyAsync(r->d_root, img.data(), img.size() * sizeof(_Float16),
                        hipMemcpyHostToDevice, c->stream));
  std::vector<float> st((size_t)r->copies * kRollStats);
  for (int i = 0; i < r->copies; ++i) {
    st[i * kRollStats + 0] = (float)s;
    st[i * kRollStats + 1] = m;
    st[i * kRollStats + 2] = 0.0f;
  }
  HIPCHK(hipMemcpyAsync(r->d_stats, st.data(), st.size() * sizeof(float),
                        hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  r->ran = false;
  return PP2_OK;
}

int pp2_rollout_run(pp2_rollout* r, const uint8_t* us, const uint8_t* zs) {
  if (!r || !us || !zs) return set_err(PP2_EINVAL, "null argument");
  pp2_ctx* c = r->ctx;
  DeviceGuard dg(c->device);
  const int C = r->copies, D = r->depth, M = r->maxchunks;
  const int kChunk = pp2::rollout_chunk();
  if (kChunk > kMaxChunk) return set_err(PP2_ESTATE, "rollout chunk too large");
  const long long stride = 3LL * M + C + 9LL * kChunk;
  std::vector<int> host((size_t)D * stride, 0);
  r->nchunks.assign(D, 0);
  for (int k = 0; k < D; ++k) {
    int* cu = host.data() + k * stride;
    int* cf = cu + M;
    int* cn = cf + M;
    int* cp = cn + M;
    // copies grouped by action, chunks of exactly kChunk entries: a partial
    // chunk repeats its last copy (the kernel has no per-copy bounds checks)
    int pos = 0, nc = 0;
    for (int u = 0; u < 9; ++u) {
      int in_chunk = 0, last = -1;
      for (int i = 0; i < C; ++i) {
        const uint8_t a = us[(size_t)k * C + i];
        if (a > 8 || zs[(size_t)k * C + i] > 15)
          return set_err(PP2_EINVAL, "step %d copy %d: action/observation out of range", k, i);
        if (a != u) continue;
        if (in_chunk == 0) {
          cu[nc] = u;
          cf[nc] = pos;
          cn[nc] = 0;
          ++nc;
        }
        cp[pos++] = last = i;
        ++cn[nc - 1];
        if (++in_chunk == kChunk) in_chunk = 0;
      }
      for (; in_chunk != 0 && in_chunk < kChunk; ++in_chunk) cp[pos++] = last;
    }
    r->nchunks[k] = nc;
  }
  HIPCHK(hipMemcpyAsync(r->d_chunks, host.data(), host.size() * sizeof(int),
                        hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(r->d_zs, zs, (size_t)D * C, hipMemcpyHostToDevice, c->stream));
  for (int k = 0; k < D; ++k) {
    const int* base = r->d_chunks + k * stride;
    const bool coded = coded_active(c);
    const int E = coded ? c->dict_n : 0;
    const int tw = pp2::tu_width(c->dict_sparse);
    HIPCHK(pp2::launch_rollout_step(c->stream, c->g, c->T.v, c->L.v, c->R.v, c->d_code,
                                    c->d_tu, ((long long)E * tw + 3) & ~3LL, tw, c->d_dl,
                                    (E + 3) & ~3, E, c->dict_sparse,
                                    k == 0 ? (const void*)r->d_root : r->buf[k & 1],
                                    r->buf[(k + 1) & 1], r->cstride, k == 0 ? 0LL : r->cstride,
                                    r->nchunks[k], base,
                                    base + M, base + 3 * M, r->d_zs + (size_t)k * C,
                                    r->d_stats + (size_t)k * C * kRollStats, r->d_partials,
                                    r->d_stats + (size_t)(k + 1) * C * kRollStats, C));
  }
  if (r->d_leafmm) {
    const bool pack = r->leaf_fib_version != c->fib_version || r->leaf_fcur != c->fcur;
    HIPCHK(pp2::launch_rollout_leaf_mfma(c->stream, c->g, c->fib[c->fcur].v, r->buf[D & 1],
                                         r->cstride, C, r->d_leafmm, r->d_leaf, pack));
    r->leaf_fib_version = c->fib_version;
    r->leaf_fcur = c->fcur;
  } else {
    HIPCHK(pp2::launch_rollout_leaf(c->stream, c->g, c->fib[c->fcur].v, r->buf[D & 1],
                                    r->cstride, C, r->d_partials, r->d_leaf));
  }
  r->ran = true;
  return PP2_OK;
}

int pp2_rollout_results(pp2_rollout* r, float* rewards, float* obs_prob, float* leaf_upper,
                        float* value) {
  if (!r) return set_err(PP2_EINVAL, "null rollout");
  if (!r->ran) return set_err(PP2_ESTATE, "rollout has not run");
  pp2_ctx* c = r->ctx;
  DeviceGuard dg(c->device);
  const int C = r->copies, D = r->depth;
  std::vector<float> st((size_t)(D + 1) * C * kRollStats), lf((size_t)C * kLeafStats);
  HIPCHK(hipMemcpyAsync(st.data(), r->d_stats, st.size() * sizeof(float), hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipMemcpyAsync(lf.data(), r->d_leaf, lf.size() * sizeof(float), hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  const float g = c->gamma;
  for (int i = 0; i < C; ++i) {
    double v = 0.0, gk = 1.0;
    for (int k = 0; k < D; ++k) {
      const float* a = &st[((size_t)k * C + i) * kRollStats];        // input of step k
      const float* b = &st[((size_t)(k + 1) * C + i) * kRollStats];  // output of step k
      const float rk = b[2] / a[0];                 // <b_k, R_u> with b_k = B_k / S_k
      const float pk = b[0] * a[1] / a[0];          // sum(L T^T b_k)
      if (rewards) rewards[(size_t)k * C + i] = rk;
      if (obs_prob) obs_prob[(size_t)k * C + i] = pk;
      v += gk * rk;
      gk *= g;
    }
    const float* l = &lf[(size_t)i * kLeafStats];
    float ub = l[1] / l[0];
    for (int q = 2; q < kLeafStats; ++q) ub = std::max(ub, l[q] / l[0]);
    if (leaf_upper) leaf_upper[i] = ub;
    if (value) value[i] = (float)(v + gk * ub);
  }
  return PP2_OK;
}

int pp2_rollout_get_belief(pp2_rollout* r, int copy, float* belief) {
  if (!r || !belief || copy < 0 || copy >= r->copies) return set_err(PP2_EINVAL, "bad arguments");
  pp2_ctx* c = r->ctx;
  DeviceGuard dg(c->device);
  std::vector<_Float16> img((size_t)r->cstride);
  // before a run every copy is the root image
  const _Float16* src = r->ran ? (const _Float16*)r->buf[r->depth & 1] + (size_t)copy * r->cstride
                               : r->d_root;
  HIPCHK(hipMemcpyAsync(img.data(), src, img.size() * sizeof(_Float16), hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int H = c->g.rows, W = c->g.width, wp = c->g.wp;
  double s = 0.0;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) s += (double)(float)img[(size_t)(y + 1) * wp + x];
  if (!(s > 0.0)) return set_err(PP2_ESTATE, "copy %d has no mass", copy);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x)
      belief[(size_t)y * W + x] = (float)((double)(float)img[(size_t)(y + 1) * wp + x] / s);
  return PP2_OK;
}

}  // extern "C"
