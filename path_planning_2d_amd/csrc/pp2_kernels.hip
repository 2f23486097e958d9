// pp2_kernels.hip -- gfx950 (MI355X) kernels for the path_planning_2d hot path.
//
// Every kernel is HBM-streaming over SoA planes (pp2_internal.h): lane l of a
// 256-thread workgroup owns CPT consecutive cells of one row and reads each
// plane with one CPT-wide vector load, so a wave moves 64*CPT*4 contiguous
// bytes per instruction.  Stencil neighbours at x+-1 are unaligned vector
// loads of the same plane (L1/L2 hits; HBM bytes unchanged); neighbours at
// y+-1 come from the halo rows, which hold zeros at the grid boundary -- the
// reference's "out-of-range contributes 0" rule -- or a neighbour shard's
// rows when the grid is row-sharded across GPUs.
//
// Arithmetic follows the reference kernels term by term (nvcc contracts
// a*b+c to fma; every such fma is spelled out with __builtin_fmaf).  The
// library is built with -fgpu-flush-denormals-to-zero (the reference is built
// with --use_fast_math, CMakeLists.txt:36) and -ffp-contract=off.
#include <float.h>
#include <stdlib.h>

#include "pp2_device.h"

namespace pp2 {

int cells_grid(const Geom& g, int cpt) {
  const long long threads = (long long)g.rows * (g.wp / cpt);
  return (int)((threads + kBlock - 1) / kBlock);
}

// ============================================================================
// (a1) model generation -- cudaGenerateModelData, POMDP
// (src/pomdp/model_generation_cuda.cu:161-347) and MDP
// (src/mdp/path_planning_2d_cuda.cu:76-213).  T is identical for both models,
// so one T serves the Bellman sweep and the belief update; R is the POMDP
// stage reward, C the MDP stage cost.  Pad cells and rows outside the global
// grid are written as zeros.
// ============================================================================
__device__ __forceinline__ void base_kernel(int u, float tp[9]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) tp[i] = 0.0f;
  switch (u) {
    case 0: tp[0] = 0.7f; tp[1] = 0.1f; tp[3] = 0.1f; tp[4] = 0.1f; break;
    case 1: tp[0] = 0.1f; tp[1] = 0.7f; tp[2] = 0.1f; tp[4] = 0.1f; break;
    case 2: tp[1] = 0.1f; tp[2] = 0.7f; tp[4] = 0.1f; tp[5] = 0.1f; break;
    case 3: tp[0] = 0.1f; tp[3] = 0.7f; tp[4] = 0.1f; tp[6] = 0.1f; break;
    case 4: tp[4] = 1.0f; break;
    case 5: tp[2] = 0.1f; tp[4] = 0.1f; tp[5] = 0.7f; tp[8] = 0.1f; break;
    case 6: tp[3] = 0.1f; tp[4] = 0.1f; tp[6] = 0.7f; tp[7] = 0.1f; break;
    case 7: tp[4] = 0.1f; tp[6] = 0.1f; tp[7] = 0.7f; tp[8] = 0.1f; break;
    default: tp[4] = 0.1f; tp[5] = 0.1f; tp[7] = 0.1f; tp[8] = 0.7f; break;
  }
}

__global__ __launch_bounds__(kBlock) void k_model_gen(
    Geom g, const uint8_t* __restrict__ map, int gx, int gy, PlaneSet T,
    PlaneSet L, PlaneSet R, PlaneSet C) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int x = (int)(t % g.wp);
  const int y = (int)(t / g.wp) - g.halo;  // local row in [-halo, rows + halo)
  if (y >= g.rows + g.halo) return;
  const int ry = g.row0 + y;          // global row
  const bool valid = x < g.width && ry >= 0 && ry < g.grows;

  uint8_t lm[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int nx = x + i % 3 - 1, ny = ry + i / 3 - 1;
    lm[i] = (!valid || nx < 0 || nx >= g.width || ny < 0 || ny >= g.grows)
                ? 1 : map[(long long)ny * g.width + nx];
  }
  const bool at_goal = (unsigned)x == (unsigned)gx && (unsigned)ry == (unsigned)gy;
  float mr[9], mc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    mr[i] = lm[i] == 1 ? -2.0f : -1.0f;
    mc[i] = lm[i] == 1 ? 2.0f : 1.0f;
  }
  for (int u = 0; u < 9; ++u) {
    float tp[9], nv[9];
    base_kernel(u, tp);
    // POMDP naive = base kernel (copied before the shift, :213-214)
#pragma unroll
    for (int i = 0; i < 9; ++i) nv[i] = tp[i];
    // MDP naive = base kernel after the trap override (:131-137)
    float nm[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) nm[i] = (lm[4] == 1) ? (i == 4 ? 1.0f : 0.0f) : tp[i];
    // occupied neighbour -> mass stays (:219-224), in index order
#pragma unroll
    for (int i = 0; i < 9; ++i)
      if (lm[i] == 1 && i != 4) { tp[4] += tp[i]; tp[i] = 0.0f; }
    if (lm[4] == 1) {  // trapped (:230-233)
#pragma unroll
      for (int i = 0; i < 9; ++i) tp[i] = 0.0f;
      tp[4] = 1.0f;
    }
    float r = 0.0f, c = 0.0f;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      r = __builtin_fmaf(mr[i], nv[i], r);  // cudaStageReward :288-291
      c = __builtin_fmaf(mc[i], nm[i], c);  // cudaStageCost   :166-169
    }
    if (u == 4) {
      r = at_goal ? 0.0f : -2.0f;  // :293
      c = at_goal ? 0.0f : 2.0f;   // mdp :171
    }
    const long long rowT = (long long)y * T.rs + x;
#pragma unroll
    for (int i = 0; i < 9; ++i) T.p[rowT + (9 * u + i) * T.ps] = valid ? tp[i] : 0.0f;
    R.p[(long long)y * R.rs + u * R.ps + x] = valid ? r : 0.0f;
    C.p[(long long)y * C.rs + u * C.ps + x] = valid ? c : 0.0f;
  }
  // cudaMeasurementLikelihood (:238-264): m = {up, left, right, down}
  const uint8_t m0 = lm[1], m1 = lm[3], m2 = lm[5], m3 = lm[7];
  for (int i = 0; i < 16; ++i) {
    const float l0 = (((i >> 0) & 1) == m0) ? (float)0.98 : (float)0.02;
    const float l1 = (((i >> 1) & 1) == m1) ? (float)0.98 : (float)0.02;
    const float l2 = (((i >> 2) & 1) == m2) ? (float)0.98 : (float)0.02;
    const float l3 = (((i >> 3) & 1) == m3) ? (float)0.98 : (float)0.02;
    const float l = ((l0 * l1) * l2) * l3;
    L.p[(long long)y * L.rs + i * L.ps + x] = valid ? l : 0.0f;
  }
}

hipError_t launch_model_gen(hipStream_t st, const Geom& g, const uint8_t* map,
                            int gx, int gy, PlaneSet T, PlaneSet L, PlaneSet R,
                            PlaneSet C) {
  const long long n = (long long)(g.rows + 2 * g.halo) * g.wp;
  const int grid = (int)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_model_gen, dim3(grid), dim3(kBlock), 0, st, g, map, gx,
                     gy, T, L, R, C);
  return hipGetLastError();
}

// ============================================================================
// (a2) belief update -- cudaBayesBeliefUpdate
// (src/pomdp/point_based_value_iteration_cuda.cu:88-133), gather form:
//   p(x) = L[x][z] * sum_{s=0..8} T[x+off_s][u][8-s] * b(x+off_s)
// as an fma chain in s order, plus the deferred renormalisation of the
// previous step (a3): the stored input is unnormalised with total mass
// *in_sum, so the output is scaled by 1/(*in_sum).  Each workgroup writes
// its partial sum of the output (fixed order) for the next normalisation.
// ============================================================================
template <int CPT>
__global__ __launch_bounds__(kBlock) void k_belief_update(
    Geom g, PlaneSet T, PlaneSet L, const float* __restrict__ b_in,
    float* __restrict__ b_out, int u, int z, const float* __restrict__ in_sum,
    float* __restrict__ partials) {
    const int tpr = g.wp / CPT;
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int y = (int)(t / tpr);
  const int x0 = (int)(t % tpr) * CPT;
  float local = 0.0f;
  if (y < g.rows) {
    const bool le = x0 == 0, re = x0 + CPT == g.wp;
    float p[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) p[k] = 0.0f;
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const int oy = s / 3 - 1, ox = s % 3 - 1;
      const float* tp = T.p + (long long)(y + oy) * T.rs +
                        (long long)(9 * u + 8 - s) * T.ps + x0 + ox;
      const float* bp = b_in + (long long)(y + oy) * g.wp + x0 + ox;
      float tv[CPT], bv[CPT];
      if (ox == 0) {
        ldv<CPT, true>(tp, tv);
        ldv<CPT, true>(bp, bv);
      } else {
        ldv<CPT, false>(tp, tv);
        ldv<CPT, false>(bp, bv);
      }
      if (ox < 0 && le) { tv[0] = 0.0f; bv[0] = 0.0f; }
      if (ox > 0 && re) { tv[CPT - 1] = 0.0f; bv[CPT - 1] = 0.0f; }
#pragma unroll
      for (int k = 0; k < CPT; ++k) p[k] = __builtin_fmaf(tv[k], bv[k], p[k]);
    }
    float lv[CPT];
    ldv<CPT, true>(L.p + (long long)y * L.rs + (long long)z * L.ps + x0, lv);
    const float inv = in_sum ? 1.0f / *in_sum : 1.0f;
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      p[k] = p[k] * lv[k];
      p[k] = p[k] * inv;
      local += p[k];
    }
    stv<CPT>(b_out + (long long)y * g.wp + x0, p);
  }
  write_wave_partial(local, partials, blockIdx.x);
}

hipError_t launch_belief_update(hipStream_t st, const Geom& g, int cpt,
                                PlaneSet T, PlaneSet L, const float* b_in,
                                float* b_out, int u, int z,
                                const float* in_sum, float* partials) {
  const int grid = cells_grid(g, cpt);
  switch (cpt) {
    case 4: hipLaunchKernelGGL(k_belief_update<4>, dim3(grid), dim3(kBlock), 0, st, g, T, L, b_in, b_out, u, z, in_sum, partials); break;
    case 2: hipLaunchKernelGGL(k_belief_update<2>, dim3(grid), dim3(kBlock), 0, st, g, T, L, b_in, b_out, u, z, in_sum, partials); break;
    default: hipLaunchKernelGGL(k_belief_update<1>, dim3(grid), dim3(kBlock), 0, st, g, T, L, b_in, b_out, u, z, in_sum, partials); break;
  }
  return hipGetLastError();
}

__global__ __launch_bounds__(64) void k_sum_finalize(const float* __restrict__ partials,
                                                     int n, float* __restrict__ out) {
  const float s = wave_reduce_partials(partials, n);
  if (threadIdx.x == 0) *out = s;
}

// Plain sum of n values in index order (the shard masses of a shard group).
__global__ void k_sum_ordered(const float* __restrict__ v, int n, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  float s = 0.0f;
  for (int i = 0; i < n; ++i) s += v[i];
  *out = s;
}

hipError_t launch_sum_ordered(hipStream_t st, const float* v, int n, float* out) {
  hipLaunchKernelGGL(k_sum_ordered, dim3(1), dim3(64), 0, st, v, n, out);
  return hipGetLastError();
}

hipError_t launch_sum_finalize(hipStream_t st, const float* partials, int n,
                               float* out) {
  hipLaunchKernelGGL(k_sum_finalize, dim3(1), dim3(64), 0, st, partials, n, out);
  return hipGetLastError();
}

// ============================================================================
// (a4) MDP Bellman backup -- cudaOneStepValueIteration
// (src/mdp/path_planning_2d_cuda.cu:215-264):
//   J'(x) = min_u C[x][u] + sum_i (gamma*T[x][u][i]) * J(x+off_i),
//   A(x)  = first u attaining the min (strict <).
// ============================================================================
template <int CPT, bool NT>
__global__ __launch_bounds__(kBlock) void k_mdp_sweep(
    Geom g, float gamma, PlaneSet T, PlaneSet C, const float* __restrict__ J_in,
    float* __restrict__ J_out, uint8_t* __restrict__ A) {
  const int tpr = g.wp / CPT;
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int y = (int)(t / tpr);
  const int x0 = (int)(t % tpr) * CPT;
  if (y < g.rows) {
    const bool le = x0 == 0, re = x0 + CPT == g.wp;
    float jn[9][CPT];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int oy = i / 3 - 1, ox = i % 3 - 1;
      const float* jp = J_in + (long long)(y + oy) * g.wp + x0 + ox;
      if (ox == 0) ldv<CPT, true>(jp, jn[i]);
      else ldv<CPT, false>(jp, jn[i]);
      if (ox < 0 && le) jn[i][0] = 0.0f;
      if (ox > 0 && re) jn[i][CPT - 1] = 0.0f;
    }
    float best[CPT];
    uint32_t arg[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) { best[k] = FLT_MAX; arg[k] = 0; }
    const float* trow = T.p + (long long)y * T.rs + x0;
    const float* crow = C.p + (long long)y * C.rs + x0;
    // Register double-buffering over actions: the 10 vector loads of action
    // u+1 (C and 9 T planes) are issued before action u is reduced, so each
    // wave keeps 10-20 dwordx4 loads in flight instead of one.
    float cb[2][CPT], tb[2][9][CPT];
    ldv_stream<CPT, NT>(crow, cb[0]);
#pragma unroll
    for (int i = 0; i < 9; ++i) ldv_stream<CPT, NT>(trow + (long long)i * T.ps, tb[0][i]);
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int cur = u & 1, nxt = cur ^ 1;
      if (u < 8) {
        ldv_stream<CPT, NT>(crow + (long long)(u + 1) * C.ps, cb[nxt]);
#pragma unroll
        for (int i = 0; i < 9; ++i)
          ldv_stream<CPT, NT>(trow + (long long)(9 * (u + 1) + i) * T.ps, tb[nxt][i]);
      }
      float cost[CPT];
#pragma unroll
      for (int k = 0; k < CPT; ++k) cost[k] = cb[cur][k];
#pragma unroll
      for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int k = 0; k < CPT; ++k)
          cost[k] = __builtin_fmaf(gamma * tb[cur][i][k], jn[i][k], cost[k]);
#pragma unroll
      for (int k = 0; k < CPT; ++k)
        if (cost[k] < best[k]) { best[k] = cost[k]; arg[k] = (uint32_t)u; }
    }
    stv<CPT>(J_out + (long long)y * g.wp + x0, best);
    uint8_t* ap = A + (long long)y * g.wp + x0;
    if constexpr (CPT == 4) {
      *reinterpret_cast<uint32_t*>(ap) = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    } else if constexpr (CPT == 2) {
      *reinterpret_cast<uint16_t*>(ap) = (uint16_t)(arg[0] | (arg[1] << 8));
    } else {
      *ap = (uint8_t)arg[0];
    }
  }
}

hipError_t launch_mdp_sweep(hipStream_t st, const Geom& g, int cpt,
                            float gamma, PlaneSet T, PlaneSet C,
                            const float* J_in, float* J_out, uint8_t* A, bool nt) {
  const int grid = cells_grid(g, cpt);
  switch (cpt) {
    case 4:
      if (nt) hipLaunchKernelGGL((k_mdp_sweep<4, true>), dim3(grid), dim3(kBlock), 0, st, g, gamma, T, C, J_in, J_out, A);
      else hipLaunchKernelGGL((k_mdp_sweep<4, false>), dim3(grid), dim3(kBlock), 0, st, g, gamma, T, C, J_in, J_out, A);
      break;
    case 2: hipLaunchKernelGGL((k_mdp_sweep<2, false>), dim3(grid), dim3(kBlock), 0, st, g, gamma, T, C, J_in, J_out, A); break;
    default: hipLaunchKernelGGL((k_mdp_sweep<1, false>), dim3(grid), dim3(kBlock), 0, st, g, gamma, T, C, J_in, J_out, A); break;
  }
  return hipGetLastError();
}

// ============================================================================
// North-star loop step, fused: one launch = one belief update (a2, with the
// previous step's renormalisation a3) + one Bellman sweep (a4) over the same
// rows.  Compared with the two kernels back to back this removes a launch
// boundary and the belief kernel's ramp/tail, and the belief's T_u rows are
// the rows the sweep of this and the neighbouring rows stream anyway, so they
// mostly hit L2 / the Infinity Cache instead of HBM.
//  * block -> row mapping is XCD-aware: the blocks dispatched to one XCD
//    (same blockIdx % 8) take consecutive rows, so rows y-1, y, y+1 share an
//    L2 (a speed choice only; any dispatch order is correct);
//  * every wave re-reduces the previous step's per-block belief partials in
//    a fixed order (bit-identical in all blocks), so the 1/sum of the input
//    is known without a separate finalize launch;
//  * arithmetic per cell is exactly k_belief_update's and k_mdp_sweep's.
// ============================================================================

template <int CPT, bool NT>
__global__ __launch_bounds__(kBlock) void k_loop_step(
    Geom g, float gamma, PlaneSet T, PlaneSet L, PlaneSet C,
    const float* __restrict__ b_in, float* __restrict__ b_out, int u, int z,
    const float* __restrict__ in_partials, int in_n, const float* __restrict__ in_sum,
    float* __restrict__ in_sum_out, float* __restrict__ out_partials,
    const float* __restrict__ J_in, float* __restrict__ J_out, uint8_t* __restrict__ A,
    int own0, int own1, float scale) {
  // rows [own0, own1) are this shard's own: only they add to the belief mass
  // and store actions (an extended-domain launch also recomputes halo rows)
  const int tpr = g.wp / CPT;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const long long t = (long long)blk * kBlock + threadIdx.x;
  const int y = (int)(t / tpr);
  const int x0 = (int)(t % tpr) * CPT;
  float local = 0.0f;
  // the previous step's mass (identical bits in every wave of every block)
  float S = 1.0f;
  if (in_partials) S = wave_reduce_partials(in_partials, in_n);
  else if (in_sum) S = *in_sum;
  if (in_sum_out && blockIdx.x == 0 && threadIdx.x == 0) *in_sum_out = S;
  const bool own = y >= own0 && y < own1;
  if (y < g.rows) {
    const bool le = x0 == 0, re = x0 + CPT == g.wp;
    // ---- belief update (k_belief_update)
    float p[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) p[k] = 0.0f;
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const int oy = s / 3 - 1, ox = s % 3 - 1;
      const float* tp = T.p + (long long)(y + oy) * T.rs +
                        (long long)(9 * u + 8 - s) * T.ps + x0 + ox;
      const float* bp = b_in + (long long)(y + oy) * g.wp + x0 + ox;
      float tv[CPT], bv[CPT];
      if (ox == 0) {
        ldv<CPT, true>(tp, tv);
        ldv<CPT, true>(bp, bv);
      } else {
        ldv<CPT, false>(tp, tv);
        ldv<CPT, false>(bp, bv);
      }
      if (ox < 0 && le) { tv[0] = 0.0f; bv[0] = 0.0f; }
      if (ox > 0 && re) { tv[CPT - 1] = 0.0f; bv[CPT - 1] = 0.0f; }
#pragma unroll
      for (int k = 0; k < CPT; ++k) p[k] = __builtin_fmaf(tv[k], bv[k], p[k]);
    }
    float lv[CPT];
    ldv<CPT, true>(L.p + (long long)y * L.rs + (long long)z * L.ps + x0, lv);
    const float inv = (1.0f / S) * scale;  // scale: a power of two (1 unsharded)
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      p[k] = p[k] * lv[k];
      p[k] = p[k] * inv;
      if (own) local += p[k];
    }
    stv<CPT>(b_out + (long long)y * g.wp + x0, p);

    // ---- Bellman sweep (k_mdp_sweep)
    float jn[9][CPT];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int oy = i / 3 - 1, ox = i % 3 - 1;
      const float* jp = J_in + (long long)(y + oy) * g.wp + x0 + ox;
      if (ox == 0) ldv<CPT, true>(jp, jn[i]);
      else ldv<CPT, false>(jp, jn[i]);
      if (ox < 0 && le) jn[i][0] = 0.0f;
      if (ox > 0 && re) jn[i][CPT - 1] = 0.0f;
    }
    float best[CPT];
    uint32_t arg[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k) { best[k] = FLT_MAX; arg[k] = 0; }
    const float* trow = T.p + (long long)y * T.rs + x0;
    const float* crow = C.p + (long long)y * C.rs + x0;
    float cb[2][CPT], tb[2][9][CPT];
    ldv_stream<CPT, NT>(crow, cb[0]);
#pragma unroll
    for (int i = 0; i < 9; ++i) ldv_stream<CPT, NT>(trow + (long long)i * T.ps, tb[0][i]);
#pragma unroll
    for (int a = 0; a < 9; ++a) {
      const int cur = a & 1, nxt = cur ^ 1;
      if (a < 8) {
        ldv_stream<CPT, NT>(crow + (long long)(a + 1) * C.ps, cb[nxt]);
#pragma unroll
        for (int i = 0; i < 9; ++i)
          ldv_stream<CPT, NT>(trow + (long long)(9 * (a + 1) + i) * T.ps, tb[nxt][i]);
      }
      float cost[CPT];
#pragma unroll
      for (int k = 0; k < CPT; ++k) cost[k] = cb[cur][k];
#pragma unroll
      for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int k = 0; k < CPT; ++k)
          cost[k] = __builtin_fmaf(gamma * tb[cur][i][k], jn[i][k], cost[k]);
#pragma unroll
      for (int k = 0; k < CPT; ++k)
        if (cost[k] < best[k]) { best[k] = cost[k]; arg[k] = (uint32_t)a; }
    }
    stv<CPT>(J_out + (long long)y * g.wp + x0, best);
    if (own) {
      uint8_t* ap = A + (long long)y * g.wp + x0;
      if constexpr (CPT == 4) {
        *reinterpret_cast<uint32_t*>(ap) = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
      } else if constexpr (CPT == 2) {
        *reinterpret_cast<uint16_t*>(ap) = (uint16_t)(arg[0] | (arg[1] << 8));
      } else {
        *ap = (uint8_t)arg[0];
      }
    }
  }
  write_wave_partial(local, out_partials, blk);
}

hipError_t launch_loop_step(hipStream_t st, const Geom& g, int cpt, float gamma,
                            PlaneSet T, PlaneSet L, PlaneSet C, const float* b_in,
                            float* b_out, int u, int z, const float* in_partials,
                            int in_n, const float* in_sum, float* in_sum_out,
                            float* out_partials, const float* J_in, float* J_out,
                            uint8_t* A, bool nt, int own0, int own1, float scale) {
  const int grid = cells_grid(g, cpt);
#define PP2_LOOP_ARGS g, gamma, T, L, C, b_in, b_out, u, z, in_partials, in_n, in_sum, \
                      in_sum_out, out_partials, J_in, J_out, A, own0, own1, scale
  switch (cpt) {
    case 4:
      if (nt) hipLaunchKernelGGL((k_loop_step<4, true>), dim3(grid), dim3(kBlock), 0, st, PP2_LOOP_ARGS);
      else hipLaunchKernelGGL((k_loop_step<4, false>), dim3(grid), dim3(kBlock), 0, st, PP2_LOOP_ARGS);
      break;
    case 2: hipLaunchKernelGGL((k_loop_step<2, false>), dim3(grid), dim3(kBlock), 0, st, PP2_LOOP_ARGS); break;
    default: hipLaunchKernelGGL((k_loop_step<1, false>), dim3(grid), dim3(kBlock), 0, st, PP2_LOOP_ARGS); break;
  }
#undef PP2_LOOP_ARGS
  return hipGetLastError();
}

// ============================================================================
// (a5) FIB Bellman backup -- cudaFIBValueIteration
// (src/pomdp/fast_informed_bound_cuda.cu:97-204):
//   a'[x][a] = R[x][a] + gamma * sum_o max_a' sum_s' (T[x][a][s']*L[s'][o]) * a[s'][a']
// with the reference's loop order, -FLT_MAX start and strict < in the max.
// VALU-bound (~25 kflop/cell); one cell per lane.
// ============================================================================
__global__ __launch_bounds__(kBlock) void k_fib_sweep(
    Geom g, float gamma, PlaneSet T, PlaneSet L, PlaneSet R, PlaneSet a_in,
    PlaneSet a_out) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int y = (int)(t / g.wp);
  const int x = (int)(t % g.wp);
  if (y >= g.rows) return;
  float la[9][9];
#pragma unroll
  for (int sp = 0; sp < 9; ++sp) {
    const int oy = sp / 3 - 1, nx = x + sp % 3 - 1;
    const bool ok = nx >= 0 && nx < g.wp;
    const float* ap = a_in.p + (long long)(y + oy) * a_in.rs + nx;
#pragma unroll
    for (int q = 0; q < 9; ++q) la[sp][q] = ok ? ap[(long long)q * a_in.ps] : 0.0f;
  }
  for (int a = 0; a < 9; ++a) {
    float tpa[9];
#pragma unroll
    for (int sp = 0; sp < 9; ++sp)
      tpa[sp] = T.p[(long long)y * T.rs + (long long)(9 * a + sp) * T.ps + x];
    const float reward = R.p[(long long)y * R.rs + (long long)a * R.ps + x];
    float rtg = 0.0f;
    for (int o = 0; o < 16; ++o) {
      float tm[9];
#pragma unroll
      for (int sp = 0; sp < 9; ++sp) {
        const int oy = sp / 3 - 1, nx = x + sp % 3 - 1;
        const bool ok = nx >= 0 && nx < g.wp;
        const float lv = ok ? L.p[(long long)(y + oy) * L.rs + (long long)o * L.ps + nx] : 0.0f;
        tm[sp] = tpa[sp] * lv;
      }
      float rtgo = -FLT_MAX;
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        float s = 0.0f;
#pragma unroll
        for (int sp = 0; sp < 9; ++sp) s = __builtin_fmaf(tm[sp], la[sp][q], s);
        if (rtgo < s) rtgo = s;
      }
      rtg = rtg + rtgo;
    }
    a_out.p[(long long)y * a_out.rs + (long long)a * a_out.ps + x] =
        __builtin_fmaf(gamma, rtg, reward);
  }
}

// k_fib_sweep for models whose T rows are +0.0 off each action's base-kernel
// support kSup[a] (every generated model; build_model_dict checks it): per
// action, per observation, only the <= 4 support neighbours' T * L enter the
// 9 next-action chains, so the likelihood loads drop from 144 to 4 per
// (action, observation) and the flops by 2.2x.  Dropped terms are
// fmaf(0 * L, alpha, s) == s (the chain starts at +0 and never holds -0), so
// alphas are bit-identical to k_fib_sweep's full 9-term chains.
//
// The 9 next-action chains of an (action, observation) run as packed pairs:
// q = 0..7 in four v_pk_fma_f32 pairs (each element the same IEEE fma, in the
// same j order, as the scalar chain) and q = 8 alone, and the max over q is a
// v_max3 chain (fmaxf: the chains are fma results, never NaN, and the max is
// the same value as the strict-< scan).  Neighbour alphas and likelihoods are
// buffer loads: 32-bit lane offsets, the plane offsets in SGPRs, and +0.0
// for off-grid neighbours from an out-of-range offset.  <= 128 VGPRs (4 waves
// per SIMD) against 158 for the scalar chains.
typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int kOffRange = 0x7ffffff0;  // num_records of the FIB resources: loads at or past it return 0

__global__ __launch_bounds__(kBlock, 4) void k_fib_sweep_sparse(
    Geom g, float gamma, PlaneSet T, PlaneSet L, PlaneSet R, PlaneSet a_in,
    PlaneSet a_out) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int y = (int)(t / g.wp);
  const int x = (int)(t % g.wp);
  if (y >= g.rows) return;
  const int ars = (int)a_in.rs, aps = (int)a_in.ps, lrs = (int)L.rs, lps = (int)L.ps;
  // buffer resources at row -1 of plane 0: per-lane row/column offsets in
  // VGPRs, the plane offsets (q * aps, o * lps) uniform in SGPRs
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(a_in.p - ars, 0, kOffRange, 0x00020000);
  const __amdgpu_buffer_rsrc_t rl =
      __builtin_amdgcn_make_buffer_rsrc(L.p - lrs, 0, kOffRange, 0x00020000);
  auto ldb = [](__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  };
  f2v lap[9][4];  // alpha_q of neighbour sp, q = 0..7 in pairs
  float la8[9];   // alpha_8 of neighbour sp
  bool ok[9];
#pragma unroll
  for (int sp = 0; sp < 9; ++sp) {
    const int oy = sp / 3 - 1, nx = x + sp % 3 - 1;
    ok[sp] = nx >= 0 && nx < g.wp;
    // off-grid neighbours: an offset past the resource's range, which a
    // buffer load answers with +0.0 (no select)
    const int vo = ok[sp] ? ((y + oy + 1) * ars + nx) * 4 : kOffRange;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      lap[sp][p].x = ldb(ra, vo, (2 * p) * aps * 4);
      lap[sp][p].y = ldb(ra, vo, (2 * p + 1) * aps * 4);
    }
    la8[sp] = ldb(ra, vo, 8 * aps * 4);
  }
#pragma unroll
  for (int a = 0; a < 9; ++a) {
    float ts[4];
    int lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int sp = kSup[a][j], oy = sp / 3 - 1, nx = x + sp % 3 - 1;
      ts[j] = j < kSupN[a] ? T.p[(long long)y * T.rs + (long long)(9 * a + sp) * T.ps + x] : 0.0f;
      lo[j] = ok[sp] ? ((y + oy + 1) * lrs + nx) * 4 : kOffRange;
    }
    float rtg = 0.0f;
#pragma unroll 2
    for (int o = 0; o < 16; ++o) {
      float tm[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        tm[j] = j < kSupN[a] ? ts[j] * ldb(rl, lo[j], o * lps * 4) : 0.0f;
      f2v sq[4] = {f2v{0.0f, 0.0f}, f2v{0.0f, 0.0f}, f2v{0.0f, 0.0f}, f2v{0.0f, 0.0f}};
      float sq8 = 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= kSupN[a]) continue;
        const f2v tj = {tm[j], tm[j]};
#pragma unroll
        for (int p = 0; p < 4; ++p) sq[p] = __builtin_elementwise_fma(tj, lap[kSup[a][j]][p], sq[p]);
        sq8 = __builtin_fmaf(tm[j], la8[kSup[a][j]], sq8);
      }
      float rtgo = fmaxf(fmaxf(-FLT_MAX, sq[0].x), sq[0].y);
#pragma unroll
      for (int p = 1; p < 4; ++p) rtgo = fmaxf(fmaxf(rtgo, sq[p].x), sq[p].y);
      rtgo = fmaxf(rtgo, sq8);
      rtg = rtg + rtgo;
    }
    a_out.p[(long long)y * a_out.rs + (long long)a * a_out.ps + x] =
        __builtin_fmaf(gamma, rtg, R.p[(long long)y * R.rs + (long long)a * R.ps + x]);
  }
}

// k_fib_sweep_sparse with the block's likelihood rows staged in LDS: a block
// of 2 rows x 256 cells first copies L of rows y0-1 .. y0+2, columns
// x0-1 .. x0+256, all 16 observations (66.5 KB) by LDS-DMA (buffer loads
// straight into LDS, no VGPRs; offsets past the resource read +0.0, like
// the sparse kernel's off-grid loads), so each neighbour likelihood comes
// from L2 / HBM once per block instead of once per action that reaches it
// (4 of 9 on average) and the (action, observation) loop reads LDS
// (consecutive lanes, consecutive words) instead of issuing 464
// vector-memory loads per cell.  The alpha loads go out before the staging
// and overlap it; each action's T support and R are loaded one action ahead.
// Same values, same arithmetic: the alphas are k_fib_sweep_sparse's bit for
// bit.  2 blocks (16 waves) per CU.
constexpr int kFibCols = 256, kFibRows = 2, kFibLs = kFibCols + 4;
// observations per unrolled step of the (action, observation) loop (A/B
// builds: 1, 2, 4 and 8 within 2 %; the next observation's likelihoods read
// ahead in registers: 3 % slower, profiles/r05/ab_fib_prefetch.txt)
#ifndef PP2_FIB_UNROLL
#define PP2_FIB_UNROLL 2
#endif
#define PP2_STR_(x) #x
#define PP2_UNROLL_(n) _Pragma(PP2_STR_(unroll n))
constexpr int kFibPlane = (kFibRows + 2) * kFibLs;  // observation plane stride in LDS
typedef __attribute__((address_space(3))) void fib_lds_void;

__global__ __launch_bounds__(kFibCols * kFibRows, 4) void k_fib_sweep_lds(
    Geom g, float gamma, PlaneSet T, PlaneSet L, PlaneSet R, PlaneSet a_in,
    PlaneSet a_out) {
  __shared__ __attribute__((aligned(16))) float sL[16 * kFibPlane];
  const int tx = threadIdx.x % kFibCols, ty = threadIdx.x / kFibCols;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int x0 = blockIdx.x * kFibCols, y0 = blockIdx.y * kFibRows;
  const int x = x0 + tx, y = y0 + ty;
  const bool cell = y < g.rows && x < g.wp;
  const int xc = cell ? x : 0, yc = cell ? y : 0;  // (lanes past the grid compute cell (0, 0), unstored)
  const int ars = (int)a_in.rs, aps = (int)a_in.ps;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(a_in.p - ars, 0, kOffRange, 0x00020000);
  auto ldb = [](__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  };
  // 1. the neighbours' alphas (registers for the whole kernel)
  f2v lap[9][4];  // alpha_q of neighbour sp, q = 0..7 in pairs
  float la8[9];   // alpha_8 of neighbour sp
#pragma unroll
  for (int sp = 0; sp < 9; ++sp) {
    const int oy = sp / 3 - 1, nx = xc + sp % 3 - 1;
    const bool ok = nx >= 0 && nx < g.wp;
    const int vo = ok ? ((yc + oy + 1) * ars + nx) * 4 : kOffRange;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      lap[sp][p].x = ldb(ra, vo, (2 * p) * aps * 4);
      lap[sp][p].y = ldb(ra, vo, (2 * p + 1) * aps * 4);
    }
    la8[sp] = ldb(ra, vo, 8 * aps * 4);
  }
  // 2. L rows by LDS-DMA: per (o, r) row five wave copies of 64 columns, at
  //    c = 0, 64, 128, 192 and 194 (the last one covers c = 256, 257 and
  //    rewrites 194 .. 255 with the same values); rows past `rows` (the halo
  //    row) and columns outside [0, wp) read +0.0
  {
    const int lrs = (int)L.rs, lps = (int)L.ps;
    const __amdgpu_buffer_rsrc_t rl =
        __builtin_amdgcn_make_buffer_rsrc(L.p - lrs, 0, kOffRange, 0x00020000);
    const int rows_in = min(kFibRows + 2, g.rows - y0 + 2);  // staged rows y0-1 .. rows (halo)
    for (int i = wv; i < 16 * (kFibRows + 2) * 5; i += kFibCols * kFibRows / 64) {
      const int row = i / 5, piece = i % 5;
      const int o = row / (kFibRows + 2), r = row % (kFibRows + 2);
      const int c = (piece < 4 ? 64 * piece : 194) + lane;
      const int xx = x0 - 1 + c;
      const bool ok = r < rows_in && xx >= 0 && xx < g.wp;
      const int vo = ok ? ((y0 + r) * lrs + xx) * 4 : kOffRange;  // row y0-1+r at (y0+r) * lrs
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rl, (fib_lds_void*)&sL[o * kFibPlane + r * kFibLs + (piece < 4 ? 64 * piece : 194)], 4, vo,
          o * lps * 4, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 3. per action: T of its support, loaded one action ahead (R at the
  //    action's start: it is consumed after the observation loop)
  auto load_t = [&](int a, float (&ts)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int sp = kSup[a][j];
      ts[j] = j < kSupN[a] ? T.p[(long long)yc * T.rs + (long long)(9 * a + sp) * T.ps + xc] : 0.0f;
    }
  };
  // the window's LDS base: row ty + oy + 1, column tx + ox + 1 of sL[o]
  const float* wl = &sL[ty * kFibLs + tx];
  float tsn[4];
  load_t(0, tsn);
#pragma unroll
  for (int a = 0; a < 9; ++a) {
    float ts[4] = {tsn[0], tsn[1], tsn[2], tsn[3]};
    const float rv = R.p[(long long)yc * R.rs + (long long)a * R.ps + xc];
    if (a + 1 < 9) load_t(a + 1, tsn);
    int lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int sp = kSup[a][j];
      lo[j] = (sp / 3) * kFibLs + sp % 3;
    }
    float rtg = 0.0f;
PP2_UNROLL_(PP2_FIB_UNROLL)
    for (int o = 0; o < 16; ++o) {
      const float* wo = wl + o * kFibPlane;
      float tm[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) tm[j] = j < kSupN[a] ? ts[j] * wo[lo[j]] : 0.0f;
      f2v sq[4] = {f2v{0.0f, 0.0f}, f2v{0.0f, 0.0f}, f2v{0.0f, 0.0f}, f2v{0.0f, 0.0f}};
      float sq8 = 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= kSupN[a]) continue;
        const f2v tj = {tm[j], tm[j]};
#pragma unroll
        for (int p = 0; p < 4; ++p) sq[p] = __builtin_elementwise_fma(tj, lap[kSup[a][j]][p], sq[p]);
        sq8 = __builtin_fmaf(tm[j], la8[kSup[a][j]], sq8);
      }
      // (no -FLT_MAX seed: the chains are finite -- finite alphas, finite
      // T * L -- so the max of the nine equals the reference's scan from
      // -FLT_MAX with strict <)
      float rtgo = fmaxf(sq[0].x, sq[0].y);
#pragma unroll
      for (int p = 1; p < 4; ++p) rtgo = fmaxf(fmaxf(rtgo, sq[p].x), sq[p].y);
      rtgo = fmaxf(rtgo, sq8);
      rtg = rtg + rtgo;
    }
    if (cell) a_out.p[(long long)y * a_out.rs + (long long)a * a_out.ps + x] = __builtin_fmaf(gamma, rtg, rv);
  }
}

hipError_t launch_fib_sweep(hipStream_t st, const Geom& g, float gamma,
                            PlaneSet T, PlaneSet L, PlaneSet R,
                            PlaneSet a_in, PlaneSet a_out, bool sparse) {
  const int grid = cells_grid(g, 1);
  // the staging kernel needs several blocks per CU to hide its per-block
  // start (alpha loads + L staging); small grids keep the sparse kernel.
  // PP2_FIB_LDS=1 / 0 forces one or the other (tests, A/B).
  const long long lds_blocks = (long long)((g.wp + kFibCols - 1) / kFibCols) *
                               ((g.rows + kFibRows - 1) / kFibRows);
  const char* force = getenv("PP2_FIB_LDS");
  const bool use_lds = force && *force ? *force == '1' : lds_blocks >= 1024;
  if (sparse && use_lds)
    hipLaunchKernelGGL(k_fib_sweep_lds, dim3((g.wp + kFibCols - 1) / kFibCols,
                                             (g.rows + kFibRows - 1) / kFibRows),
                       dim3(kFibCols * kFibRows), 0, st, g, gamma, T, L, R, a_in, a_out);
  else if (sparse)
    hipLaunchKernelGGL(k_fib_sweep_sparse, dim3(grid), dim3(kBlock), 0, st, g, gamma, T, L, R,
                       a_in, a_out);
  else
    hipLaunchKernelGGL(k_fib_sweep, dim3(grid), dim3(kBlock), 0, st, g, gamma, T,
                       L, R, a_in, a_out);
  return hipGetLastError();
}

// ============================================================================
// Convergence check of the VI / FIB drivers (path_planning_2d.cu:243-250,
// fast_informed_bound_cuda.cu:246-257): max |cur - snap| over the owned
// cells and planes, then snap := cur.
// ============================================================================
__global__ __launch_bounds__(kBlock) void k_absdiff_max(Geom g, int K, PlaneSet cur,
                                                         PlaneSet snap, float* partials) {
  __shared__ float lds4[4];
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long ncell = (long long)g.rows * g.wp;
  float m = 0.0f;
  if (t < ncell) {
    const int y = (int)(t / g.wp), x = (int)(t % g.wp);
    for (int k = 0; k < K; ++k) {
      const long long ic = (long long)y * cur.rs + (long long)k * cur.ps + x;
      const long long is = (long long)y * snap.rs + (long long)k * snap.ps + x;
      const float c = cur.p[ic];
      m = fmaxf(m, fabsf(snap.p[is] - c));
      snap.p[is] = c;
    }
  }
  const float r = block_max(m, lds4);
  if (threadIdx.x == 0) partials[blockIdx.x] = r;
}

hipError_t launch_absdiff_max(hipStream_t st, const Geom& g, int planes,
                              PlaneSet cur, PlaneSet snap, float* partials,
                              int* nparts) {
  const long long n = (long long)g.rows * g.wp;
  const int grid = (int)((n + kBlock - 1) / kBlock);
  *nparts = grid;
  hipLaunchKernelGGL(k_absdiff_max, dim3(grid), dim3(kBlock), 0, st, g, planes,
                     cur, snap, partials);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_sum_cells(Geom g, const float* __restrict__ b,
                                                       float* partials) {
    const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long n = (long long)g.rows * g.wp;
  const float v = t < n ? b[t] : 0.0f;
  write_wave_partial(v, partials, blockIdx.x);
}

hipError_t launch_sum_cells(hipStream_t st, const Geom& g, const float* b,
                            float* partials, int* nparts) {
  const long long n = (long long)g.rows * g.wp;
  const int grid = (int)((n + kBlock - 1) / kBlock);
  *nparts = 4 * grid;
  hipLaunchKernelGGL(k_sum_cells, dim3(grid), dim3(kBlock), 0, st, g, b, partials);
  return hipGetLastError();
}

// ============================================================================
// (a6/a7) QV-tree expansion, batched.  One VNode::expand
// (src/pomdp/search_tree_cuda.cu:437-450) builds 9 QNodes, each running the
// belief update for every sampled observation z, renormalising, and scoring
// the child with the FIB upper bound (fast_informed_bound_cuda.cu:278-297).
// Here the 9 predictions pred_a = T_a^T b are computed once (k_expand_pred),
// then every (a, z) child's mass  m[a][z] = sum_x pred_a(x) L_z(x)  and FIB
// dots d[a][z][i] = sum_x (pred_a(x) L_z(x)) alpha_i(x) come out of one pass
// (k_expand_stats), whatever subset the sampler later keeps.  The child
// belief pred_a * L_z is the reference kernel's output bit for bit; the sums
// are fixed-order tree reductions.
// ============================================================================
constexpr int kStats = 10;  // per child: mass + 9 FIB dots

template <int CPT>
__global__ __launch_bounds__(kBlock) void k_expand_pred(
    Geom g, PlaneSet T, const float* __restrict__ b, PlaneSet R, PlaneSet P,
    float* __restrict__ rpartials) {
  __shared__ float red[4][9];
  const int tpr = g.wp / CPT;
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int y = (int)(t / tpr);
  const int x0 = (int)(t % tpr) * CPT;
  float rew[9];
#pragma unroll
  for (int a = 0; a < 9; ++a) rew[a] = 0.0f;
  if (y < g.rows) {
    const bool le = x0 == 0, re = x0 + CPT == g.wp;
    float bv[9][CPT];
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const int oy = s / 3 - 1, ox = s % 3 - 1;
      const float* bp = b + (long long)(y + oy) * g.wp + x0 + ox;
      if (ox == 0) ldv<CPT, true>(bp, bv[s]);
      else ldv<CPT, false>(bp, bv[s]);
      if (ox < 0 && le) bv[s][0] = 0.0f;
      if (ox > 0 && re) bv[s][CPT - 1] = 0.0f;
    }
    for (int a = 0; a < 9; ++a) {
      float p[CPT];
#pragma unroll
      for (int k = 0; k < CPT; ++k) p[k] = 0.0f;
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        const int oy = s / 3 - 1, ox = s % 3 - 1;
        const float* tp = T.p + (long long)(y + oy) * T.rs +
                          (long long)(9 * a + 8 - s) * T.ps + x0 + ox;
        float tv[CPT];
        if (ox == 0) ldv<CPT, true>(tp, tv);
        else ldv<CPT, false>(tp, tv);
        if (ox < 0 && le) tv[0] = 0.0f;
        if (ox > 0 && re) tv[CPT - 1] = 0.0f;
#pragma unroll
        for (int k = 0; k < CPT; ++k) p[k] = __builtin_fmaf(tv[k], bv[s][k], p[k]);
      }
      stv<CPT>(P.p + (long long)y * P.rs + (long long)a * P.ps + x0, p);
      float rv[CPT];
      ldv<CPT, true>(R.p + (long long)y * R.rs + (long long)a * R.ps + x0, rv);
#pragma unroll
      for (int k = 0; k < CPT; ++k) rew[a] += bv[4][k] * rv[k];
    }
  }
  // QNode reward <b, R[:,a]> partials (search_tree_cuda.cu:168-173)
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < 9; ++a) {
    const float v = wave_sum(rew[a]);
    if ((threadIdx.x & 63) == 0) red[w][a] = v;
  }
  __syncthreads();
  if (threadIdx.x < 9) {
    const int a = threadIdx.x;
    rpartials[(long long)blockIdx.x * 9 + a] = ((red[0][a] + red[1][a]) + red[2][a]) + red[3][a];
  }
}

// grid = (cell tiles) x 16 observations; partials[tile][z][a][kStats]
template <int CPT>
__global__ __launch_bounds__(kBlock) void k_expand_stats(
    Geom g, PlaneSet P, PlaneSet L, PlaneSet F, float* __restrict__ partials) {
  __shared__ float red[4][9 * kStats];
  const int z = blockIdx.y;
  const int tpr = g.wp / CPT;
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int y = (int)(t / tpr);
  const int x0 = (int)(t % tpr) * CPT;
  // [a * kStats + i] as two 64-float halves, zero-padded to 128 for
  // wave_sum_scatter128
  float acl[64], ach[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) acl[j] = ach[j] = 0.0f;
#define PP2_ACC(m) (*((m) < 64 ? &acl[(m) & 63] : &ach[(m) & 63]))
  if (y < g.rows) {
    float lv[CPT], fv[9][CPT];
    ldv<CPT, true>(L.p + (long long)y * L.rs + (long long)z * L.ps + x0, lv);
#pragma unroll
    for (int i = 0; i < 9; ++i)
      ldv<CPT, true>(F.p + (long long)y * F.rs + (long long)i * F.ps + x0, fv[i]);
#pragma unroll
    for (int a = 0; a < 9; ++a) {
      float pv[CPT];
      ldv<CPT, true>(P.p + (long long)y * P.rs + (long long)a * P.ps + x0, pv);
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const float c = pv[k] * lv[k];  // the reference kernel's child value
        PP2_ACC(a * kStats) += c;
#pragma unroll
        for (int i = 0; i < 9; ++i)
          PP2_ACC(a * kStats + 1 + i) = __builtin_fmaf(c, fv[i][k], PP2_ACC(a * kStats + 1 + i));
      }
    }
  }
  const int w = threadIdx.x >> 6;
  // the 90 wave totals by one reduce-scatter (wave_sum's association): lane l
  // gets totals 2l, 2l + 1
#undef PP2_ACC
  float tot[2];
  wave_sum_scatter128(acl, ach, tot);
  {
    const int l = threadIdx.x & 63;
    if (2 * l < 9 * kStats) red[w][2 * l] = tot[0];
    if (2 * l + 1 < 9 * kStats) red[w][2 * l + 1] = tot[1];
  }
  __syncthreads();
  if (threadIdx.x < 9 * kStats) {
    const int j = threadIdx.x;
    partials[((long long)blockIdx.x * 16 + z) * (9 * kStats) + j] =
        ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
  }
}

// sum / FIB dots of one belief: out[0] = sum b, out[1+i] = sum b*alpha_i
template <int CPT>
__global__ __launch_bounds__(kBlock) void k_belief_dots(Geom g, const float* __restrict__ b,
                                                        PlaneSet F, float* __restrict__ partials) {
  __shared__ float red[4][kStats];
  const int tpr = g.wp / CPT;
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const int y = (int)(t / tpr);
  const int x0 = (int)(t % tpr) * CPT;
  float acc[kStats];
#pragma unroll
  for (int i = 0; i < kStats; ++i) acc[i] = 0.0f;
  if (y < g.rows) {
    float bv[CPT];
    ldv<CPT, true>(b + (long long)y * g.wp + x0, bv);
#pragma unroll
    for (int k = 0; k < CPT; ++k) acc[0] += bv[k];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      float fv[CPT];
      ldv<CPT, true>(F.p + (long long)y * F.rs + (long long)i * F.ps + x0, fv);
#pragma unroll
      for (int k = 0; k < CPT; ++k) acc[1 + i] = __builtin_fmaf(bv[k], fv[k], acc[1 + i]);
    }
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < kStats; ++i) {
    const float v = wave_sum(acc[i]);
    if ((threadIdx.x & 63) == 0) red[w][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < kStats)
    partials[(long long)blockIdx.x * kStats + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// out[j] = sum_r partials[r][j], fixed order over r (r = 0..rows-1);
// *scalar_out = *scalar when given (a mass riding along to a host mirror)
__global__ __launch_bounds__(kBlock) void k_reduce_columns(const float* __restrict__ partials,
                                                           int rows, int cols, float* __restrict__ out,
                                                           const float* __restrict__ scalar,
                                                           float* __restrict__ scalar_out) {
  const int j = blockIdx.x * kBlock + threadIdx.x;
  if (scalar_out && j == 0) *scalar_out = *scalar;
  if (j >= cols) return;
  // 16 loads in flight ahead of the in-order adds (one L2 round trip per 16
  // rows instead of per row)
  float s = 0.0f;
  int r = 0;
  for (; r + 16 <= rows; r += 16) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = partials[(long long)(r + i) * cols + j];
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i];
  }
  for (; r < rows; ++r) s += partials[(long long)r * cols + j];
  out[j] = s;
}

// Both column reductions of one expansion in one launch: blocks [0, nb) sum
// the stats columns, the last block the 9 reward columns (k_reduce_columns'
// order).
__global__ __launch_bounds__(kBlock) void k_reduce_expand(const float* __restrict__ rpartials,
                                                          const float* __restrict__ spartials,
                                                          int rows, int scols,
                                                          float* __restrict__ rewards_out,
                                                          float* __restrict__ stats_out) {
  const int nb = (scols + kBlock - 1) / kBlock;
  const bool rew = (int)blockIdx.x == nb;
  const int j = rew ? (int)threadIdx.x : (int)blockIdx.x * kBlock + threadIdx.x;
  const int cols = rew ? 9 : scols;
  const float* __restrict__ part = rew ? rpartials : spartials;
  if (j >= cols) return;
  float s = 0.0f;
  int r = 0;
  for (; r + 16 <= rows; r += 16) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = part[(long long)(r + i) * cols + j];
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i];
  }
  for (; r < rows; ++r) s += part[(long long)r * cols + j];
  (rew ? rewards_out : stats_out)[j] = s;
}

// b := b / *mass over owned cells (materialise a normalised belief in place)
__global__ __launch_bounds__(kBlock) void k_scale(Geom g, float* __restrict__ b,
                                                  const float* __restrict__ mass) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (long long)g.rows * g.wp) return;
  b[t] = b[t] / *mass;
}

hipError_t launch_expand(hipStream_t st, const Geom& g, int cpt, PlaneSet T,
                         const float* b, PlaneSet R, PlaneSet L, PlaneSet F,
                         PlaneSet P, float* rpartials, float* spartials,
                         float* rewards_out, float* stats_out) {
  const int tiles = cells_grid(g, cpt);
  switch (cpt) {
    case 4:
      hipLaunchKernelGGL(k_expand_pred<4>, dim3(tiles), dim3(kBlock), 0, st, g, T, b, R, P, rpartials);
      hipLaunchKernelGGL(k_expand_stats<4>, dim3(tiles, 16), dim3(kBlock), 0, st, g, P, L, F, spartials);
      break;
    default:
      hipLaunchKernelGGL(k_expand_pred<1>, dim3(tiles), dim3(kBlock), 0, st, g, T, b, R, P, rpartials);
      hipLaunchKernelGGL(k_expand_stats<1>, dim3(tiles, 16), dim3(kBlock), 0, st, g, P, L, F, spartials);
      break;
  }
  const int cols = 16 * 9 * kStats;
  hipLaunchKernelGGL(k_reduce_expand, dim3((cols + kBlock - 1) / kBlock + 1), dim3(kBlock), 0, st,
                     rpartials, spartials, tiles, cols, rewards_out, stats_out);
  return hipGetLastError();
}

hipError_t launch_belief_dots(hipStream_t st, const Geom& g, int cpt, const float* b,
                              PlaneSet F, float* partials, float* out, const float* mass,
                              float* mass_out) {
  const int tiles = cells_grid(g, cpt);
  if (cpt == 4)
    hipLaunchKernelGGL(k_belief_dots<4>, dim3(tiles), dim3(kBlock), 0, st, g, b, F, partials);
  else
    hipLaunchKernelGGL(k_belief_dots<1>, dim3(tiles), dim3(kBlock), 0, st, g, b, F, partials);
  hipLaunchKernelGGL(k_reduce_columns, dim3(1), dim3(kBlock), 0, st, partials, tiles, kStats, out,
                     mass, mass_out);
  return hipGetLastError();
}

hipError_t launch_scale(hipStream_t st, const Geom& g, float* b, const float* mass) {
  const long long n = (long long)g.rows * g.wp;
  hipLaunchKernelGGL(k_scale, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                     g, b, mass);
  return hipGetLastError();
}

// ============================================================================
// Batched fp16 QV-tree rollouts (BASELINE configs[4]): the per-copy
// reduction of the step kernel's partials, the FIB leaf pass
// (fast_informed_bound_cuda.cu:278-297).  The step kernel itself
// (k_rollout_band) is in pp2_rollout_dev.hip; its first step reads the root
// image for every copy (no broadcast).
//  * beliefs live as fp16 planes [copy][row][x] (2 B per cell-copy), each
//    copy max-normalised, math in fp32;
//  * per (copy, wave) partial sums of {stored sum, stored max, reward dot} are
//    reduced per copy by k_rollout_reduce, in a fixed order.
// ============================================================================

template <bool ALIGNED>
__device__ __forceinline__ void ldh4(const _Float16* __restrict__ p, float (&v)[4]) {
  h4 t;
  if constexpr (ALIGNED) t = *reinterpret_cast<const h4*>(p);
  else t = *reinterpret_cast<const h4u*>(p);
  v[0] = (float)t[0]; v[1] = (float)t[1]; v[2] = (float)t[2]; v[3] = (float)t[3];
}

constexpr int kRollStats = 3;  // stored sum, stored max, reward dot
constexpr int kRollIter = 8;   // 1024-cell slabs per leaf-pass block tile
constexpr int kRollChunk = 8;  // copies per leaf-pass block

// per copy: out[c] = {sum, max, reward} over its nwaves partials (fixed order)
__global__ __launch_bounds__(64) void k_rollout_reduce(const float* __restrict__ partials,
                                                       int nwaves, int copies,
                                                       float* __restrict__ out) {
  const int c = blockIdx.x;
  if (c >= copies) return;
  const float* pp = partials + (long long)c * nwaves * kRollStats;
  float s = 0.0f, m = 0.0f, r = 0.0f;
  for (int i = threadIdx.x; i < nwaves; i += 64) {
    s += pp[i * kRollStats + 0];
    m = fmaxf(m, pp[i * kRollStats + 1]);
    r += pp[i * kRollStats + 2];
  }
  s = wave_sum(s);
  m = wave_max(m);
  r = wave_sum(r);
  if (threadIdx.x == 0) {
    out[c * kRollStats + 0] = s;
    out[c * kRollStats + 1] = m;
    out[c * kRollStats + 2] = r;
  }
}

// Leaf FIB dots of every copy: partials[c][wave][10] = {sum, dot_0..dot_8};
// 1024-cell slabs of kRollChunk copies per block, the alpha planes loaded
// once per slab.
__global__ __launch_bounds__(kBlock) void k_rollout_leaf(Geom g, PlaneSet F,
                                                         const _Float16* __restrict__ b,
                                                         long long cstride, int copies,
                                                         float* __restrict__ partials,
                                                         int nwaves) {
  // branch-free like k_rollout_band: copies past the end repeat the last one
  // (identical partials), lanes past the grid end add nothing
  const int c0 = blockIdx.y * kRollChunk;
  const int wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const long long ncells = (long long)g.rows * g.wp;
  const long long tile0 = (long long)blockIdx.x * kRollIter * (kBlock * 4);
  const int iters = (int)min((long long)kRollIter, (ncells - tile0 + kBlock * 4 - 1) / (kBlock * 4));
  long long cbase[kRollChunk];
  float acc[kRollChunk][kStats];
#pragma unroll
  for (int j = 0; j < kRollChunk; ++j) {
    cbase[j] = (long long)min(c0 + j, copies - 1) * cstride;
#pragma unroll
    for (int i = 0; i < kStats; ++i) acc[j][i] = 0.0f;
  }
  for (int it = 0; it < iters; ++it) {
    const long long cell_raw = tile0 + (long long)it * (kBlock * 4) + threadIdx.x * 4;
    const bool valid = cell_raw < ncells;
    const long long cell = valid ? cell_raw : ncells - 4;
    const int y = (int)(cell / g.wp), x0 = (int)(cell % g.wp);
    const long long off = (long long)y * g.wp + x0;
    float bq[kRollChunk][4];
#pragma unroll
    for (int j = 0; j < kRollChunk; ++j) ldh4<true>(b + cbase[j] + off, bq[j]);
    float fv[9][4];
#pragma unroll
    for (int i = 0; i < 9; ++i)
      ldv<4, true>(F.p + (long long)y * F.rs + (long long)i * F.ps + x0, fv[i]);
#pragma unroll
    for (int j = 0; j < kRollChunk; ++j) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float bv = valid ? bq[j][k] : 0.0f;
        acc[j][0] += bv;
#pragma unroll
        for (int i = 0; i < 9; ++i) acc[j][1 + i] = __builtin_fmaf(bv, fv[i][k], acc[j][1 + i]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kRollChunk; ++j) {
#pragma unroll
    for (int i = 0; i < kStats; ++i) acc[j][i] = wave_sum(acc[j][i]);
    if ((threadIdx.x & 63) == 0) {
      float* pp = partials + ((long long)min(c0 + j, copies - 1) * nwaves + wave) * kStats;
#pragma unroll
      for (int i = 0; i < kStats; ++i) pp[i] = acc[j][i];
    }
  }
}

__global__ __launch_bounds__(64) void k_rollout_leaf_reduce(const float* __restrict__ partials,
                                                            int nwaves, int copies,
                                                            float* __restrict__ out) {
  const int c = blockIdx.x;
  if (c >= copies) return;
  const float* pp = partials + (long long)c * nwaves * kStats;
  for (int i = 0; i < kStats; ++i) {
    float s = 0.0f;
    for (int w = threadIdx.x; w < nwaves; w += 64) s += pp[w * kStats + i];
    s = wave_sum(s);
    if (threadIdx.x == 0) out[c * kStats + i] = s;
  }
}

int rollout_tiles(const Geom& g) {
  const long long cells = (long long)g.rows * g.wp;
  const long long per = (long long)kRollIter * kBlock * 4;
  return (int)((cells + per - 1) / per);
}
int rollout_leaf_waves(const Geom& g) { return rollout_tiles(g) * (kBlock / 64); }
int rollout_waves(const Geom& g) {
  const int a = rollout_leaf_waves(g), b = rollout_step_waves(g);
  return a > b ? a : b;
}

hipError_t launch_rollout_reduce(hipStream_t st, const float* partials, int nwaves,
                                 int ncopies, float* stats_out) {
  hipLaunchKernelGGL(k_rollout_reduce, dim3(ncopies), dim3(64), 0, st, partials, nwaves, ncopies,
                     stats_out);
  return hipGetLastError();
}

hipError_t launch_rollout_leaf(hipStream_t st, const Geom& g, PlaneSet F, const void* b,
                               long long cstride, int ncopies, float* partials,
                               float* out) {
  const int tiles = rollout_tiles(g);
  const int nw = rollout_leaf_waves(g);
  const int gy = (ncopies + kRollChunk - 1) / kRollChunk;
  hipLaunchKernelGGL(k_rollout_leaf, dim3(tiles, gy), dim3(kBlock), 0, st, g, F,
                     (const _Float16*)b + g.wp, cstride, ncopies, partials, nw);
  hipLaunchKernelGGL(k_rollout_leaf_reduce, dim3(ncopies), dim3(64), 0, st, partials, nw,
                     ncopies, out);
  return hipGetLastError();
}

// ============================================================================
// Layout conversion between the reference's AoS host arrays
// (T[hw][9][9], L[hw][16], R[hw][9], beliefs[hw]) and the SoA planes.
// ============================================================================
__global__ __launch_bounds__(kBlock) void k_pack(Geom g, int K, PlaneSet src,
                                                 float* __restrict__ dense,
                                                 const float* __restrict__ divide_by,
                                                 float* __restrict__ mass_out) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long n = (long long)g.rows * g.width * K;
  if (mass_out && i == 0) *mass_out = *divide_by;
  if (i >= n) return;
  const long long cell = i / K;
  const int k = (int)(i % K);
  const int y = (int)(cell / g.width), x = (int)(cell % g.width);
  float v = src.p[(long long)y * src.rs + (long long)k * src.ps + x];
  if (divide_by) v = v / *divide_by;
  dense[i] = v;
}

__global__ __launch_bounds__(kBlock) void k_unpack(Geom g, int K,
                                                   const float* __restrict__ dense,
                                                   PlaneSet dst) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long n = (long long)g.rows * g.width * K;
  if (i >= n) return;
  const long long cell = i / K;
  const int k = (int)(i % K);
  const int y = (int)(cell / g.width), x = (int)(cell % g.width);
  dst.p[(long long)y * dst.rs + (long long)k * dst.ps + x] = dense[i];
}

__global__ __launch_bounds__(kBlock) void k_pack_u8(Geom g, const uint8_t* __restrict__ src,
                                                    uint8_t* __restrict__ dense) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long n = (long long)g.rows * g.width;
  if (i >= n) return;
  const int y = (int)(i / g.width), x = (int)(i % g.width);
  dense[i] = src[(long long)y * g.wp + x];
}

hipError_t launch_pack(hipStream_t st, const Geom& g, int K, PlaneSet src,
                       float* dense, const float* divide_by, float* mass_out) {
  if (mass_out && !divide_by) return hipErrorInvalidValue;
  const long long n = (long long)g.rows * g.width * K;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                     g, K, src, dense, divide_by, mass_out);
  return hipGetLastError();
}

hipError_t launch_unpack(hipStream_t st, const Geom& g, int K,
                         const float* dense, PlaneSet dst) {
  const long long n = (long long)g.rows * g.width * K;
  hipLaunchKernelGGL(k_unpack, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                     g, K, dense, dst);
  return hipGetLastError();
}

hipError_t launch_pack_u8(hipStream_t st, const Geom& g, const uint8_t* src,
                          uint8_t* dense) {
  const long long n = (long long)g.rows * g.width;
  hipLaunchKernelGGL(k_pack_u8, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                     g, src, dense);
  return hipGetLastError();
}

}  // namespace pp2
