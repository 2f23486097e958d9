// pp2_pbvi_dev.hip -- PBVI kernels that restate the reference's DEVICE code
// (built like the other kernel files: FTZ, every fused multiply-add an
// explicit fmaf, as nvcc --use_fast_math contracts it).
//
//   k_pbvi_update    cudaBayesBeliefUpdate (point_based_value_iteration_cuda.cu:88-133)
//                    over a batch of (source row, action, observation) candidates
//   k_pbvi_gamma_ao  cudaComputeGammaOA (:297-341) for one action, all 16
//                    observations and every alpha vector
#include <hip/hip_runtime.h>

#include "pp2_pbvi_internal.h"

namespace pp2 {
namespace {

constexpr int kThreads = 256;
constexpr int kGaoRows = 16;  // alpha vectors per thread in k_pbvi_gamma_ao

__global__ __launch_bounds__(kThreads) void k_pbvi_update(
    Geom g, PlaneSet T, PlaneSet L, const float* __restrict__ src, int ld,
    const int* __restrict__ src_row, const uint8_t* __restrict__ us,
    const uint8_t* __restrict__ zs, float* __restrict__ out) {
  const int c = blockIdx.y;
  const int W = g.width, H = g.rows;
  const int idx = blockIdx.x * kThreads + threadIdx.x;
  if (idx >= H * W) return;
  const int y = idx / W, x = idx - y * W;
  const int u = us[c], z = zs[c];
  const float* __restrict__ b = src + (long long)src_row[c] * ld;
  // p = sum_s T[sidx][u][8-s] * b[sidx] over in-grid neighbours, s ascending
  float p = 0.0f;
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const int sy = y + s / 3 - 1, sx = x + s % 3 - 1;
    if (sy < 0 || sy >= H || sx < 0 || sx >= W) continue;
    const float t = T.p[(long long)sy * T.rs + (long long)(9 * u + 8 - s) * T.ps + sx];
    p = fmaf(t, b[sy * W + sx], p);
  }
  out[(long long)c * ld + idx] = p * L.p[(long long)y * L.rs + (long long)z * L.ps + x];
}

// The QV-tree expansion's 9 predictions of one dense belief row (the child
// of (u, z) is pred[u] * L[z], formed by the IEEE sums of pp2_fchain.hip):
// thread (cell, action u = blockIdx.y).  SPARSE (a coded model whose T rows
// the host verified to be +0 off the base-kernel support): only the
// action's <= 4 support taps -- the others are fmaf(+0, b, p) == p for the
// finite b >= 0 and p != -0 of the chain -- in the same ascending-s order.
template <bool SPARSE>
__global__ __launch_bounds__(kThreads) void k_tree_pred(Geom g, PlaneSet T,
                                                        const float* __restrict__ b, int ld,
                                                        float* __restrict__ pred) {
  const int W = g.width, H = g.rows;
  const int idx = blockIdx.x * kThreads + threadIdx.x, u = blockIdx.y;
  if (idx >= H * W) return;
  const int y = idx / W, x = idx - y * W;
  float p = 0.0f;
  auto tap = [&](int s) {
    const int sy = y + s / 3 - 1, sx = x + s % 3 - 1;
    if (sy < 0 || sy >= H || sx < 0 || sx >= W) return;
    const float t = T.p[(long long)sy * T.rs + (long long)(9 * u + 8 - s) * T.ps + sx];
    p = fmaf(t, b[sy * W + sx], p);
  };
  if constexpr (SPARSE) {
    for (int j = kSupN[u] - 1; j >= 0; --j) tap(8 - kSup[u][j]);  // s ascending
  } else {
#pragma unroll
    for (int s = 0; s < 9; ++s) tap(s);
  }
  pred[(long long)u * ld + idx] = p;
}

// One thread = one cell x, kGaoRows alpha vectors and 8 of the 16
// observations: the 8x9 products T[x][a][s] * L[nbr_s(x)][o] stay in
// registers across the alpha rows (blockIdx.z = 2 * action + half).
// Off-grid neighbours enter as 0 * 0 terms, which leave the chain unchanged
// (it never holds -0), exactly as the reference's skipped terms.  The slices
// are written once and read back by the GEMM after more than the Infinity
// Cache has streamed by: non-temporal stores.
__global__ __launch_bounds__(kThreads) void k_pbvi_gamma_ao(
    Geom g, float gamma, PlaneSet T, PlaneSet L, const float* __restrict__ alpha, int ld, int S,
    int a0, float* __restrict__ G, long long ostride) {
  const int W = g.width, H = g.rows;
  const int a = a0 + (blockIdx.z >> 1), o0 = (blockIdx.z & 1) * 8;
  G += ((long long)(blockIdx.z >> 1) * 16 + o0) * ostride;
  const int idx = blockIdx.x * kThreads + threadIdx.x;
  if (idx >= H * W) return;
  const int y = idx / W, x = idx - y * W;
  int off[9];
  bool ok[9];
  float tm[8][9];
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const int sy = y + s / 3 - 1, sx = x + s % 3 - 1;
    ok[s] = !(sy < 0 || sy >= H || sx < 0 || sx >= W);
    off[s] = ok[s] ? sy * W + sx : idx;
    const float t = T.p[(long long)y * T.rs + (long long)(9 * a + s) * T.ps + x];
#pragma unroll
    for (int o = 0; o < 8; ++o)
      tm[o][s] = ok[s] ? t * L.p[(long long)(ok[s] ? sy : y) * L.rs + (long long)(o0 + o) * L.ps +
                                 (ok[s] ? sx : x)]
                       : 0.0f;
  }
  const int k1 = min(S, (int)(blockIdx.y + 1) * kGaoRows);
  for (int k = blockIdx.y * kGaoRows; k < k1; ++k) {
    const float* __restrict__ al = alpha + (long long)k * ld;
    float av[9];
#pragma unroll
    for (int s = 0; s < 9; ++s) av[s] = ok[s] ? al[off[s]] : 0.0f;
#pragma unroll
    for (int o = 0; o < 8; ++o) {
      float acc = 0.0f;
#pragma unroll
      for (int s = 0; s < 9; ++s) acc = fmaf(tm[o][s], av[s], acc);
      __builtin_nontemporal_store(gamma * acc, G + o * ostride + (long long)k * ld + idx);
    }
  }
}

}  // namespace

hipError_t launch_pbvi_update(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet L,
                              const float* src, int ld, const int* src_row, const uint8_t* us,
                              const uint8_t* zs, int n, float* out) {
  if (n <= 0) return hipSuccess;
  const int hw = g.rows * g.width;
  dim3 grid((hw + kThreads - 1) / kThreads, n);
  hipLaunchKernelGGL(k_pbvi_update, grid, dim3(kThreads), 0, st, g, T, L, src, ld, src_row, us,
                     zs, out);
  return hipGetLastError();
}

hipError_t launch_tree_pred(hipStream_t st, const Geom& g, PlaneSet T, const float* b, int ld,
                            float* pred, bool sparse) {
  const int hw = g.rows * g.width;
  if (hw <= 0) return hipSuccess;
  if (ld < hw) return hipErrorInvalidValue;
  const dim3 grid((hw + kThreads - 1) / kThreads, 9);
  if (sparse)
    hipLaunchKernelGGL(k_tree_pred<true>, grid, dim3(kThreads), 0, st, g, T, b, ld, pred);
  else
    hipLaunchKernelGGL(k_tree_pred<false>, grid, dim3(kThreads), 0, st, g, T, b, ld, pred);
  return hipGetLastError();
}

hipError_t launch_pbvi_gamma_ao(hipStream_t st, const Geom& g, float gamma, PlaneSet T,
                                PlaneSet L, const float* alpha, int ld, int S, int a0, int a1,
                                float* G, long long ostride) {
  if (S <= 0 || a1 <= a0) return hipSuccess;
  const int hw = g.rows * g.width;
  dim3 grid((hw + kThreads - 1) / kThreads, (S + kGaoRows - 1) / kGaoRows, 2 * (a1 - a0));
  hipLaunchKernelGGL(k_pbvi_gamma_ao, grid, dim3(kThreads), 0, st, g, gamma, T, L, alpha, ld, S,
                     a0, G, ostride);
  return hipGetLastError();
}

}  // namespace pp2
