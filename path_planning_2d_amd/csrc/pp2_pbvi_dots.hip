// pp2_pbvi_dots.hip -- the planner's reference-order PBVI leaf dots with the
// rows handed to the products by DPP broadcasts (k_pair_dot_bq).  Same
// arithmetic as k_pair_dot_1 (pp2_pbvi_host.hip): per (child, alpha) pair one
// x-ordered chain acc = acc + a[x] * b[x] from +0 (evaluatePbviCpu,
// point_based_value_iteration_cuda.cu:678-699), IEEE, no denormal flushing.
// Built with -fno-slp-vectorize (Makefile): paired into v_pk_mul_f32, the
// products would keep each broadcast as a separate v_mov_b32_dpp.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "pp2_pbvi_internal.h"

namespace pp2 {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kOff = 0x7ffffff0, kNo = kOff / 4;  // buffer offset past any range: reads +0.0

// v_mov_b32_dpp row_newbcast:K -- lane K of each 16-lane row to the whole
// row; folded into the consuming v_mul_f32 as v_mul_f32_dpp
template <int K>
__device__ __forceinline__ float bcast16(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150 + K, 0xf,
                                                               0xf, true));
}

template <int NB>
struct Ring {
  f4 b[NB];
};
template <int G, int NB>
__device__ __forceinline__ void ring_read(Ring<NB>& r, uint32_t ba) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.b[G % NB]) : "v"(ba), "n"(16 * G));
}
template <int G, int LA, int NB>
__device__ __forceinline__ void ring_prologue(Ring<NB>& r, uint32_t ba) {
  if constexpr (G < LA) {
    ring_read<G, NB>(r, ba);
    ring_prologue<G + 1, LA, NB>(r, ba);
  }
}
// wait for group G's alphas (groups issued so far: up to min(G - 1 + LA, NG - 1)),
// then its 4 products: cell 64 q + 4 s + c of the row sits in lane s of each
// 16-lane row, component c
template <int G, int NG, int LA, int NB, int NQ>
__device__ __forceinline__ void products(Ring<NB>& r, const f4 (&av)[NQ], float (&p)[4]) {
  constexpr int left = (NG - 1 - G) < (LA - 1) ? (NG - 1 - G) : (LA - 1);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(left) : "memory");
  asm volatile("" : "+v"(r.b[G % NB]));
  const f4 b = r.b[G % NB];
  constexpr int q = G / 16, s = G % 16;
  p[0] = bcast16<s>(av[q].x) * b.x;
  p[1] = bcast16<s>(av[q].y) * b.y;
  p[2] = bcast16<s>(av[q].z) * b.z;
  p[3] = bcast16<s>(av[q].w) * b.w;
}
// group G's adds after group G + 1's products (their latency under the adds)
template <int G, int NG, int LA, int NB, int NQ>
__device__ __forceinline__ void group(Ring<NB>& r, uint32_t ba, const f4 (&av)[NQ], float& acc, float (&pr)[4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG) ring_read<G + LA, NB>(r, ba);
    if constexpr (G + 1 < NG) {
      float pn[4];
      products<G + 1, NG, LA, NB, NQ>(r, av, pn);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc = acc + pr[k];
        pr[k] = pn[k];
      }
      group<G + 1, NG, LA, NB, NQ>(r, ba, av, acc, pr);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = acc + pr[k];
    }
  }
}

// The live tiles (ntiles: known on the device only, from acount) numbered
// per XCD: block b runs on XCD b % 8 and takes tile (b % 8) * per + b / 8, so
// each XCD's blocks cover whole alpha tiles and the live tiles spread over
// all 8 XCDs whatever the launch's grid (sized for every row); past them
// INT_MAX (the block exits).
__device__ __forceinline__ int xcd_tile(int ntiles) {
  const int per = (ntiles + 7) / 8, k = (int)(blockIdx.x / 8);
  return k < per ? (int)(blockIdx.x % 8) * per + k : INT_MAX;
}

// Block = 4 waves = 16 children x 16 alphas (k_pair_dot_1's tile, its tiles
// numbered per XCD the same way).  Wave w, 16-lane row r: child row
// i0 + 4 w + r; lane k of that row: alpha j0 + k.  The child row reaches the
// lanes as one float4 per lane (lane k: cells 64 q + 4 k .. + 3, one
// buffer_load_dwordx4 per 64 cells, a chunk ahead) and the products through
// v_mul_f32_dpp row_newbcast: the rows cost no LDS traffic.  The block stages
// only its 16 alphas (one ds_read_b128 per 4 cells, LA groups ahead, counted
// waits).  Past na / nb / n the loads read +0.0, whose products leave a chain
// from +0 unchanged.  tools/micro/pair_dots.hip: 16.1 cycles per cell per
// wave against k_pair_dot_1's 20.9 (profiles/r05/pair_dots_dpp_mfma.txt).
template <int CH, int LAV>
__global__ __launch_bounds__(256) void k_pair_dot_bq(const float* __restrict__ Ag, int na,
                                                     const float* __restrict__ Bg, int nb, int ld, int n,
                                                     float* __restrict__ out, int ldo,
                                                     const int* __restrict__ alist,
                                                     const int* __restrict__ acount) {
  constexpr int NT = 256, C4 = CH / 4, ROW = CH + 4, NI = 16 * C4, L4 = NI / NT, NQ = CH / 64;
  static_assert(NI % NT == 0 && CH % 64 == 0, "whole float4 columns per thread, whole 64-cell blocks");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (alist) na = min(na, *acount);
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, rr = l >> 4, kk = l & 15;
  const int nrt = (na + 15) / 16, ntiles = nrt * ((nb + 15) / 16);
  const int t = xcd_tile(ntiles);
  if (t >= ntiles) return;  // (uniform over the block)
  const int i0 = (t % nrt) * 16, j0 = (t / nrt) * 16;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)Ag, 0, kOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Bg + (long long)j0 * ld), 0, kOff, 0x00020000);
  const int row = i0 + 4 * w + rr;
  const int arow = row < na ? (alist ? alist[row] : row) : -1;
  const int ao = arow >= 0 ? arow * ld + 4 * kk : kNo;
  int bo[L4], bc4[L4];
#pragma unroll
  for (int k = 0; k < L4; ++k) {
    const int e = tid + NT * k, br = e / C4;
    bc4[k] = (e % C4) * 4;
    bo[k] = j0 + br < nb ? br * ld + bc4[k] : kNo;
  }
  f4 rg[L4], an[NQ], av[NQ];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const bool in = (bo[k] != kNo) & (x0 + bc4[k] < n);
      rg[k] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsb, in ? (bo[k] + x0) * 4 : kOff, 0, 0));
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool in = (ao != kNo) & (x0 + 64 * q + 4 * kk < n);
      an[q] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsa, in ? (ao + x0 + 64 * q) * 4 : kOff,
                                                                           0, 0));
    }
  };
  const uint32_t ba = (uint32_t)(uintptr_t)(smem + kk * ROW);
  float acc = 0.0f;
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += CH) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int e = tid + NT * k;
      *(f4*)(smem + (e / C4) * ROW + (e % C4) * 4) = rg[k];
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) av[q] = an[q];
    __syncthreads();
    if (x0 + CH < n) fetch(x0 + CH);
    constexpr int NG = CH / 4, LA = LAV, NB = LA + 1;  // one read per group: lgkmcnt <= 15
    Ring<NB> ring;
    ring_prologue<0, LA, NB>(ring, ba);
    float pr[4];
    products<0, NG, LA, NB, NQ>(ring, av, pr);
    group<0, NG, LA, NB, NQ>(ring, ba, av, acc, pr);
    __syncthreads();
  }
  if (arow >= 0 && j0 + kk < nb) out[(long long)arow * ldo + j0 + kk] = acc;
}

}  // namespace

hipError_t launch_pair_dot_bq(hipStream_t st, const float* A, int na, const float* B, int nb, int ld, int n,
                              float* out, int ldo, const int* alist, const int* acount) {
  constexpr int CH = 512, LA = 8;
  static unsigned long long attr = 0ull;
  allow_lds(reinterpret_cast<const void*>(&k_pair_dot_bq<CH, LA>), attr);
  const int tiles = (int)(((long long)na + 15) / 16 * ((nb + 15) / 16));
  hipLaunchKernelGGL((k_pair_dot_bq<CH, LA>), dim3((tiles + 7) / 8 * 8), dim3(256),
                     (size_t)16 * (CH + 4) * sizeof(float), st, A, na, B, nb, ld, n, out, ldo, alist, acount);
  return hipGetLastError();
}

}  // namespace pp2
