// pp2_pbvi_host.hip -- PBVI kernels that restate the reference's HOST (x86,
// IEEE, no FMA) and cuBLAS arithmetic.  Built WITHOUT denormal flushing; the
// only fused multiply-adds are the MFMA's (the pinned Sgemm chain).
//
//   k_rows_chain    std::accumulate / std::partial_sum / std::inner_product of
//                   rows (normalizeProbDensity :135-145, sampleFromProbDensity
//                   :147-163, the action values :610-622)
//   k_rows_div      x /= sum (:142-143)
//   k_pair_chain    the L1 distances of generateBeliefSet (:238-246) and
//                   all-pairs inner products
//   k_pbvi_sample   the three draws of generateBeliefSet (:212-222)
//   k_pbvi_pick     min over the set / max_element over actions (:238-255)
//   k_gemm_nt       the per-(a,o) Sgemm (:505-513) on v_mfma_f32_32x32x2_f32
//   k_argmax_rows   max_element over each belief's row (:531-537)
//   k_pbvi_gamma_a  Gamma_a = R + sum_o alphas_ao_max (:459-467, Sgeam :542-550)
//   k_pbvi_select   the best action per belief and its alpha (:610-626)
#include <hip/hip_runtime.h>
#include <float.h>

#include <algorithm>
#include <type_traits>
#include <limits.h>
#include <stdlib.h>

#include "pp2_pbvi_internal.h"

namespace pp2 {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int xcd_map(int b, int n) {
  const int q = n / 8, r = n % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// ---------------------------------------------------------------- row chains
// One x-ordered chain per row (std::accumulate, partial_sum, inner_product).
// A block owns kChainRows rows: all 256 threads stream kChainX-wide tiles of
// them into LDS with coalesced loads (the next tile's loads in flight while
// the current one is summed), and lane r of wave 0 walks row r of the tile.
// Row stride kChainXP = kChainX + 4 keeps the per-lane float4 LDS reads on
// distinct banks.
constexpr int kChainRows = 16, kChainX = 256, kChainXP = kChainX + 4;
constexpr int kChainVec = kChainRows * kChainX / 4 / 256;  // float4 per thread per tile

enum { CH_SUM = 0, CH_CDF = 1, CH_DOT = 2 };

template <int MODE>
__global__ __launch_bounds__(256) void k_rows_chain(const float* __restrict__ A, int amod,
                                                    const float* __restrict__ B, int ld, int rows,
                                                    int n, float* __restrict__ sums,
                                                    float* __restrict__ cdf) {
  constexpr int NOP = MODE == CH_DOT ? 2 : 1;
  __shared__ __attribute__((aligned(16))) float t[2][NOP][kChainRows * kChainXP];
  const int tid = threadIdx.x, r0 = blockIdx.x * kChainRows;
  const int lrow = tid >> 4, lcol = tid & 15;  // staging: 16 threads per row
  const int grow = r0 + lrow;
  const bool rin = grow < rows;
  const float* __restrict__ pa = A + (long long)(rin ? grow % amod : 0) * ld;
  const float* __restrict__ pb = MODE == CH_DOT ? B + (long long)(rin ? grow : 0) * ld : nullptr;
  f4 ra[kChainVec], rb[kChainVec];
  auto gload = [&](int x0) {
#pragma unroll
    for (int k = 0; k < kChainVec; ++k) {
      const int x = x0 + 4 * (lcol + 16 * k);
      const bool in = rin && x < ld;
      ra[k] = in ? *(const f4*)(pa + x) : f4{0, 0, 0, 0};
      if (MODE == CH_DOT) rb[k] = in ? *(const f4*)(pb + x) : f4{0, 0, 0, 0};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int k = 0; k < kChainVec; ++k) {
      *(f4*)&t[buf][0][lrow * kChainXP + 4 * (lcol + 16 * k)] = ra[k];
      if (MODE == CH_DOT) *(f4*)&t[buf][NOP - 1][lrow * kChainXP + 4 * (lcol + 16 * k)] = rb[k];
    }
  };
  float acc = 0.0f;
  gload(0);
  lstore(0);
  __syncthreads();
  int buf = 0;
  for (int x0 = 0; x0 < n; x0 += kChainX) {
    const bool more = x0 + kChainX < n;
    if (more) gload(x0 + kChainX);
    if (tid < kChainRows) {
      float* __restrict__ ta = &t[buf][0][tid * kChainXP];
      const float* __restrict__ tb = &t[buf][NOP - 1][tid * kChainXP];
      const int m = min(kChainX, n - x0);
      int j = 0;
      for (; j + 4 <= m; j += 4) {
        f4 v = *(const f4*)(ta + j);
        if (MODE == CH_DOT) {
          const f4 w = *(const f4*)(tb + j);
          acc = acc + v.x * w.x;
          acc = acc + v.y * w.y;
          acc = acc + v.z * w.z;
          acc = acc + v.w * w.w;
        } else {
          acc = acc + v.x;
          v.x = acc;
          acc = acc + v.y;
          v.y = acc;
          acc = acc + v.z;
          v.z = acc;
          acc = acc + v.w;
          v.w = acc;
          if (MODE == CH_CDF) *(f4*)(ta + j) = v;
        }
      }
      for (; j < m; ++j) {
        if (MODE == CH_DOT) {
          acc = acc + ta[j] * tb[j];
        } else {
          acc = acc + ta[j];
          if (MODE == CH_CDF) ta[j] = acc;
        }
      }
    }
    __syncthreads();
    if (MODE == CH_CDF && rin) {
      float* __restrict__ pc = cdf + (long long)grow * ld;
#pragma unroll
      for (int k = 0; k < kChainVec; ++k) {
        const int x = x0 + 4 * (lcol + 16 * k);
        if (x < n) {
          const f4 v = *(const f4*)&t[buf][0][lrow * kChainXP + 4 * (lcol + 16 * k)];
          if (x + 4 <= n) {
            *(f4*)(pc + x) = v;
          } else {
            for (int e = 0; e < n - x; ++e) pc[x + e] = v[e];
          }
        }
      }
    }
    if (more) lstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  if (tid < kChainRows && r0 + tid < rows) {
    if (MODE == CH_DOT)
      sums[r0 + tid] = acc;
    else if (sums)
      sums[r0 + tid] = acc;
  }
}

// ---------------------------------------------------------------- lane chains
// The same x-ordered chains when there are few of them (the reference-order
// planner: 144 child renormalisations, 144 x 9 FIB dots, 9 rewards per
// expansion).  Each chain is a dependent fp32 add per element, so its floor
// is the add latency (~4 cycles, 65536 cells: ~0.11 ms); k_rows_chain's
// load -> barrier -> sum per 256-x tile runs it at ~0.8 ms, k_pair_chain's
// 32-x tiles at ~7 ms.  Here one wave per block owns a few chains, one per
// lane (chain (r, i) = A row r, B row i), and streams its NROW rows through
// an LDS ring by LDS-DMA (global_load_lds, one 1-KiB wave instruction per row
// and chunk) up to three chunks ahead of the adds, waiting on its own vmcnt
// only -- no barrier.  One wave's LDS-DMA lands ~16 KiB per 0.65 us
// (MI355X_MICROARCH.md ldsdma-fill), so a block stages at most ~8 rows: a
// 256-x chunk of adds takes ~0.43 us.  Lanes that share a row read the same
// LDS address (a broadcast); rows sit 16 B apart in bank space.  Per element:
// the product (DOT) first, then the add (x86 std::inner_product).
constexpr int kLaneCH = 256;            // floats per row and chunk
constexpr int kLaneRowF = kLaneCH + 4;  // LDS row stride (16-B bank skew)
constexpr int kLaneSlots = 4;           // ring slots: 3 chunks in flight + 1 summed
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// Block (bx, by): A rows [bx * ra, + ra), B rows [by * rb, + rb) (DOT), NROW
// = ra + rb staged rows (fewer real ones at the grid's edge: the DMA repeats
// row 0, so the vmcnt arithmetic stays fixed).
template <int MODE, int NROW>
__global__ __launch_bounds__(64) void k_lane_chains(const float* __restrict__ A, int na, int ra,
                                                    const float* __restrict__ B, int nb, int rb,
                                                    int ld, int n, float* __restrict__ out,
                                                    int ldo) {
  __shared__ __attribute__((aligned(16))) float ring[kLaneSlots][NROW][kLaneRowF];
  const int lane = threadIdx.x;
  const int r0 = blockIdx.x * ra, i0 = blockIdx.y * rb;
  const int nra = min(ra, na - r0);
  const int nrb = MODE == CH_DOT ? min(rb, nb - i0) : 0;
  const int nrow = nra + (MODE == CH_DOT ? rb : 0);  // staged row j: A row j < ra.. (see src)
  const int nch = (n + kLaneCH - 1) / kLaneCH;
  // chunk c of every staged row into slot c % kLaneSlots
  auto issue = [&](int c) {
    const int x = c * kLaneCH + 4 * lane;
    const int xs = x + 4 <= ld ? x : 0;  // past the row: an in-bounds address, never summed
#pragma unroll
    for (int j = 0; j < NROW; ++j) {
      const float* src;
      if (MODE == CH_DOT && j >= ra) {
        const int ib = i0 + (j - ra < nrb ? j - ra : 0);
        src = B + (long long)ib * ld;
      } else {
        src = A + (long long)(r0 + (j < nra ? j : 0)) * ld;
      }
      __builtin_amdgcn_global_load_lds((glb_void_t*)(src + xs),
                                       (lds_void_t*)&ring[c % kLaneSlots][j][0], 16, 0, 0);
    }
  };
  (void)nrow;
  const int r = MODE == CH_DOT ? lane / rb : lane;
  const int i = MODE == CH_DOT ? lane - r * rb : 0;
  const bool active = MODE == CH_DOT ? (r < nra && i < nrb) : lane < nra;
  const int ra_ = active ? r : 0, rb_ = MODE == CH_DOT && active ? ra + i : 0;
  float acc = 0.0f;
  for (int c = 0; c < 3 && c < nch; ++c) issue(c);
  for (int c = 0; c < nch; ++c) {
    // chunk c has landed once at most the younger chunks' loads are pending
    if (c + 2 < nch) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NROW) : "memory");
    else if (c + 1 < nch) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NROW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const float* pa = &ring[c % kLaneSlots][ra_][0];
    const float* pb = &ring[c % kLaneSlots][rb_][0];
    const int m = min(kLaneCH, n - c * kLaneCH);
    if (m == kLaneCH) {
      // groups of 8 elements, their LDS reads (inline asm) issued LA groups
      // ahead of the dependent adds, each group waited for with a counted
      // lgkmcnt that leaves the younger groups' reads in flight (the
      // compiler's own waits drain to lgkmcnt(0) every few groups: a full
      // LDS round trip per 24 adds); the empty asm pins the adds below it
      constexpr int G = 8, NG = kLaneCH / G;
      constexpr int R = MODE == CH_DOT ? 4 : 2;  // b128 reads per group
      constexpr int LA = 3, NB = LA + 1;          // lookahead (LA * R <= 15), register groups
      f4 ga[NB][2], gb[NB][2];
      const uint32_t la = (uint32_t)(uintptr_t)pa, lb = (uint32_t)(uintptr_t)pb;
      auto rd = [&](int g) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          asm volatile("ds_read_b128 %0, %1" : "=v"(ga[g % NB][q]) : "v"(la + 4u * (G * g + 4 * q)));
          if (MODE == CH_DOT)
            asm volatile("ds_read_b128 %0, %1" : "=v"(gb[g % NB][q]) : "v"(lb + 4u * (G * g + 4 * q)));
        }
      };
#pragma unroll
      for (int g = 0; g < LA; ++g) rd(g);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if (g + LA < NG) {
          rd(g + LA);
          asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(LA * R) : "memory");
        } else if (g + 2 < NG) {
          asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(2 * R) : "memory");
        } else if (g + 1 < NG) {
          asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(R) : "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          asm volatile("" : "+v"(ga[g % NB][q]));
          if (MODE == CH_DOT) asm volatile("" : "+v"(gb[g % NB][q]));
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if (MODE == CH_DOT) {
            const f4 pr = ga[g % NB][q] * gb[g % NB][q];  // the products, then the chain
            acc = acc + pr.x;
            acc = acc + pr.y;
            acc = acc + pr.z;
            acc = acc + pr.w;
          } else {
            acc = acc + ga[g % NB][q].x;
            acc = acc + ga[g % NB][q].y;
            acc = acc + ga[g % NB][q].z;
            acc = acc + ga[g % NB][q].w;
          }
        }
      }
    } else {
      for (int j = 0; j < m; ++j) acc = MODE == CH_DOT ? acc + pa[j] * pb[j] : acc + pa[j];
    }
    // slot c % kLaneSlots is read (the LDS reads above returned: the adds
    // consumed them); chunk c + 3 reuses the slot of chunk c - 1
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (c + 3 < nch) issue(c + 3);
  }
  if (active) {
    if (MODE == CH_DOT) out[(long long)(r0 + r) * ldo + i0 + i] = acc;
    else out[r0 + r] = acc;
  }
}

__global__ __launch_bounds__(256) void k_rows_div(float* __restrict__ A, int ld, int n,
                                                  const float* __restrict__ sums) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= n) return;
  float* p = A + (long long)blockIdx.y * ld + x;
  *p = *p / sums[blockIdx.y];
}

// ---------------------------------------------------------------- pair chains
// TA A rows x TB = (256 / TA) * NC B rows per 256-thread block; thread (la =
// tid % TA, jg = tid / TA) keeps the NC chains (la, jg * NC + m), each one
// x-ordered fp32 chain (multiply then add, or |a - b| then add).  A is staged
// transposed ([x][row]: the lanes of one la read one word), B row-major.
// Two shapes: 64 x 64 pairs per block with 16 chains per thread for many
// pairs (ILP), 16 x 16 with one chain per thread and 128-value chunks when
// the pair grid is small (the planner's reference-order PBVI bounds: 144
// children x S = 500 alphas give 24 blocks of the large shape for 256 CUs,
// 288 of the small one; measured 2 and 4 chains per thread ran 1.3x and 1.9x
// slower there).
// the device's flush of a product (the FTZ reference kernel's product, as
// pp2_fchain.hip's ftz)
__device__ __forceinline__ float ftz_f(float v) { return fabsf(v) < FLT_MIN ? copysignf(0.0f, v) : v; }

template <int OP>
__device__ __forceinline__ float pair_step(float acc, float a, float b) {
  if constexpr (OP == PAIR_L1)
    return acc + fabsf(a - b);
  else if constexpr (OP == PAIR_CHILD)  // cudaBayesBeliefUpdate's p *= L, flushed (a: L, b: p)
    return acc + ftz_f(b * ftz_f(a));
  else
    return acc + a * b;
}

// CH x-values per chunk; the next chunk's loads are issued into registers
// before the current chunk's chains run (one global round trip per chunk
// would otherwise bound the small shape: 2048 chunks x ~1 us at 256^2).
// With alist, A row i is row alist[i] of A (i < *acount, the block's rows
// past it idle) and its results go to out row alist[i].
template <int OP, int TA, int NC, int CH>
__global__ __launch_bounds__(256) void k_pair_chain(const float* __restrict__ A, int na,
                                                    const float* __restrict__ B, int nb, int ld,
                                                    int n, float* __restrict__ out, int ldo,
                                                    const int* __restrict__ alist,
                                                    const int* __restrict__ acount) {
  constexpr int G = 256 / TA, TB = G * NC;
  constexpr int kRowVec = CH / 4;                      // float4 per row of a chunk
  constexpr int LA = (TA * kRowVec + 255) / 256;       // float4 loads per thread
  constexpr int LB = (TB * kRowVec + 255) / 256;
  __shared__ float sAT[CH][TA + 1];
  __shared__ __attribute__((aligned(16))) float sB[TB][CH + 4];
  const int tid = threadIdx.x, la = tid % TA, jg = tid / TA;
  const int i0 = blockIdx.x * TA, j0 = blockIdx.y * TB;
  if (alist) {
    na = min(na, *acount);
    if (i0 >= na) return;  // (uniform over the block)
  }
  auto arow = [&](int i) { return alist ? alist[i] : i; };
  float acc[NC];
#pragma unroll
  for (int m = 0; m < NC; ++m) acc[m] = 0.0f;
  f4 ra[LA], rb[LB];
  auto fetch = [&](int x0) {  // this thread's share of the chunk at x0 (zeros past n)
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int e = tid + 256 * q, row = e / kRowVec, c4 = (e % kRowVec) * 4, ia = i0 + row;
      ra[q] = e < TA * kRowVec && ia < na && x0 + c4 < n
                  ? *(const f4*)(A + (long long)arow(ia) * ld + x0 + c4) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int e = tid + 256 * q, row = e / kRowVec, c4 = (e % kRowVec) * 4, jb = j0 + row;
      rb[q] = e < TB * kRowVec && jb < nb && x0 + c4 < n
                  ? *(const f4*)(B + (long long)jb * ld + x0 + c4) : f4{0, 0, 0, 0};
    }
  };
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += CH) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int e = tid + 256 * q, row = e / kRowVec, c4 = (e % kRowVec) * 4;
      if (e < TA * kRowVec) {
        sAT[c4 + 0][row] = ra[q].x;
        sAT[c4 + 1][row] = ra[q].y;
        sAT[c4 + 2][row] = ra[q].z;
        sAT[c4 + 3][row] = ra[q].w;
      }
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int e = tid + 256 * q, row = e / kRowVec, c4 = (e % kRowVec) * 4;
      if (e < TB * kRowVec) *(f4*)&sB[row][c4] = rb[q];
    }
    __syncthreads();
    if (x0 + CH < n) fetch(x0 + CH);  // in flight during this chunk's chains
    const int m = min(CH, n - x0);
    int xx = 0;
    for (; xx + 4 <= m; xx += 4) {
      const float a0 = sAT[xx][la], a1 = sAT[xx + 1][la], a2 = sAT[xx + 2][la],
                  a3 = sAT[xx + 3][la];
#pragma unroll
      for (int mm = 0; mm < NC; ++mm) {
        const f4 b = *(const f4*)&sB[jg * NC + mm][xx];
        float v = acc[mm];
        v = pair_step<OP>(v, a0, b.x);
        v = pair_step<OP>(v, a1, b.y);
        v = pair_step<OP>(v, a2, b.z);
        v = pair_step<OP>(v, a3, b.w);
        acc[mm] = v;
      }
    }
    for (; xx < m; ++xx) {
      const float av = sAT[xx][la];
#pragma unroll
      for (int mm = 0; mm < NC; ++mm) acc[mm] = pair_step<OP>(acc[mm], av, sB[jg * NC + mm][xx]);
    }
    __syncthreads();
  }
  if (i0 + la < na) {
    const long long orow = arow(i0 + la);
#pragma unroll
    for (int mm = 0; mm < NC; ++mm) {
      const int j = j0 + jg * NC + mm;
      if (j < nb) out[orow * ldo + j] = acc[mm];
    }
  }
}

// The pair chains of few long rows -- the planner's PBVI leaf dots: <= 144
// rows x S = 500 alphas of 65536 cells, about one chain per lane of the chip
// -- are bound by each chain's own latency per element.  k_pair_chain's
// small shape waits for every 4-element group's LDS reads before its adds (a
// full LDS round trip per 4 adds).  Here 16 A rows x 16 B rows per 256-thread
// block, one chain per thread (thread (la, jb) = A row la, B row jb, so a
// wave holds 16 A rows x 4 B rows: its A reads hit 16 rows 4 banks apart, its
// B reads are 4 broadcasts), both operands row-major in LDS (one ds_read_b128
// per operand and 4 elements), 512-element chunks staged from registers
// loaded one chunk ahead, and the reads of each 8-element group issued three
// groups ahead of the dependent adds (inline asm, counted lgkmcnt waits, as
// k_lane_chains).  Rows past na / nb and cells past n read as 0: their
// products +-0 leave the chain unchanged (a chain from +0 is never -0).
// TB: B rows per block.  16 (measured: 20, which fits the planner's 144 x
// 500 grid in one block per CU, ran 5 % slower, profiles/r05/pbvi_plan_modes_ab.txt).
inline int cdiv(long long a, int b) { return (int)((a + b - 1) / b); }
constexpr int kSeqCH = 512, kSeqRow = kSeqCH + 4;
constexpr size_t seq_lds(int tb) { return (size_t)(16 + tb) * kSeqRow * sizeof(float); }

template <int OP, int TA, int TB>
__global__ __launch_bounds__(TA * TB) void k_pair_seq(const float* __restrict__ A, int na,
                                                      const float* __restrict__ B, int nb, int ld,
                                                      int n, float* __restrict__ out, int ldo,
                                                      const int* __restrict__ alist,
                                                      const int* __restrict__ acount) {
  constexpr int NT = TA * TB;
  static_assert(NT % 64 == 0, "whole waves");
  constexpr int LA4 = (TA * 128 + NT - 1) / NT, LB4 = (TB * 128 + NT - 1) / NT;  // float4 per thread
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sA = smem;
  float* sB = smem + TA * kSeqRow;
  const int tid = threadIdx.x, la = tid % TA, jb = tid / TA;
  const int i0 = blockIdx.x * TA, j0 = blockIdx.y * TB;
  if (alist) {
    na = min(na, *acount);
    if (i0 >= na) return;  // (uniform over the block)
  }
  auto arow = [&](int i) { return alist ? alist[i] : i; };
  // staging: float4 e of a tile = row e / 128, column 4 (e % 128); thread t
  // takes e = t + NT q
  f4 ra[LA4], rb[LB4];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int q = 0; q < LA4; ++q) {
      const int e = tid + NT * q, row = e >> 7, c4 = (e & 127) * 4, ia = i0 + row;
      ra[q] = e < TA * 128 && ia < na && x0 + c4 < n
                  ? *(const f4*)(A + (long long)arow(ia) * ld + x0 + c4) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int q = 0; q < LB4; ++q) {
      const int e = tid + NT * q, row = e >> 7, c4 = (e & 127) * 4, jj = j0 + row;
      rb[q] = e < TB * 128 && jj < nb && x0 + c4 < n
                  ? *(const f4*)(B + (long long)jj * ld + x0 + c4) : f4{0, 0, 0, 0};
    }
  };
  const uint32_t la_addr = (uint32_t)(uintptr_t)(sA + la * kSeqRow);
  const uint32_t lb_addr = (uint32_t)(uintptr_t)(sB + jb * kSeqRow);
  float acc = 0.0f;
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += kSeqCH) {
#pragma unroll
    for (int q = 0; q < LA4; ++q) {
      const int e = tid + NT * q;
      if (e < TA * 128) *(f4*)(sA + (e >> 7) * kSeqRow + (e & 127) * 4) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < LB4; ++q) {
      const int e = tid + NT * q;
      if (e < TB * 128) *(f4*)(sB + (e >> 7) * kSeqRow + (e & 127) * 4) = rb[q];
    }
    __syncthreads();
    if (x0 + kSeqCH < n) fetch(x0 + kSeqCH);  // in flight during this chunk's chains
    constexpr int G = 8, NG = kSeqCH / G, R = 4, LA = 3, NB = LA + 1;
    f4 ga[NB][2], gb[NB][2];
    auto rd = [&](int g) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        asm volatile("ds_read_b128 %0, %1" : "=v"(ga[g % NB][q]) : "v"(la_addr + 4u * (G * g + 4 * q)));
        asm volatile("ds_read_b128 %0, %1" : "=v"(gb[g % NB][q]) : "v"(lb_addr + 4u * (G * g + 4 * q)));
      }
    };
#pragma unroll
    for (int g = 0; g < LA; ++g) rd(g);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g + LA < NG) {
        rd(g + LA);
        asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(LA * R) : "memory");
      } else if (g + 2 < NG) {
        asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(2 * R) : "memory");
      } else if (g + 1 < NG) {
        asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(R) : "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        asm volatile("" : "+v"(ga[g % NB][q]));
        asm volatile("" : "+v"(gb[g % NB][q]));
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f4 a = ga[g % NB][q], b = gb[g % NB][q];
        acc = pair_step<OP>(acc, a.x, b.x);
        acc = pair_step<OP>(acc, a.y, b.y);
        acc = pair_step<OP>(acc, a.z, b.z);
        acc = pair_step<OP>(acc, a.w, b.w);
      }
    }
    __syncthreads();
  }
  if (i0 + la < na && j0 + jb < nb) out[(long long)arow(i0 + la) * ldo + j0 + jb] = acc;
}

// ---------------------------------------------------------------- PBVI leaf dots
// The planner's reference-order PBVI leaf dots (evaluatePbviCpu,
// point_based_value_iteration_cuda.cu:678-699: acc = acc + a[x] * b[x] from
// +0, x in order): <= 144 kept children x S alphas of up to a grid's cells,
// each pair one chain whose length alone sets the time once every chain has
// a lane (tools/micro/pair_dots.hip measures the shapes).  Two shapes, both
// with branch-free staging (buffer loads; past the matrix they read +0.0,
// whose products leave a chain unchanged), the chunk's LDS reads issued LA
// groups ahead of their use (the compiler counts the in-order LDS returns)
// and the blocks' tiles numbered per XCD (each XCD takes whole alpha tiles
// against every row tile):
//   k_pair_dot_pk  a lane keeps two chains (rows 2p, 2p + 1 against one
//                  alpha) as one packed pair: v_pk_mul_f32 / v_pk_add_f32,
//                  the IEEE products and sums of the scalar ops; the row
//                  pair is staged interleaved, so one ds_read_b128 returns
//                  two cells of both rows already paired;
//   k_pair_dot_1   one chain per lane (k_pair_seq's thread layout).
// PP2_PAIR_DOT selects: 1 packed, 2 one chain per lane, 0 k_pair_seq (3, the
// default: k_pair_dot_bq in pp2_pbvi_dots.hip).
constexpr int kDotOff = 0x7ffffff0;  // buffer offset past any range: the load reads +0.0
__device__ __forceinline__ f4 ldq_rs(__amdgpu_buffer_rsrc_t rs, int off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
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

typedef float f2p __attribute__((ext_vector_type(2)));

// The chains' LDS reads: ds_read_b128 at immediate offsets into a ring of NB
// register groups, LA groups ahead of their use, with counted lgkmcnt waits
// (the compiler, left to itself, waits for each group as it issues it).
// One group = 4 cells: R reads (the packed kernel: the row pair's two
// float4 and the alpha's; the one-chain kernel: the row's and the alpha's).
template <int NB, int R>
struct DotRing {
  f4 v[NB][R];
};
template <int G, int NB>
__device__ __forceinline__ void dot_read_pk(DotRing<NB, 3>& r, uint32_t pa, uint32_t ba) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.v[G % NB][0]) : "v"(pa), "n"(32 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.v[G % NB][1]) : "v"(pa), "n"(32 * G + 16));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.v[G % NB][2]) : "v"(ba), "n"(16 * G));
}
template <int G, int NB>
__device__ __forceinline__ void dot_read_1(DotRing<NB, 2>& r, uint32_t aa, uint32_t ba) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.v[G % NB][0]) : "v"(aa), "n"(16 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.v[G % NB][1]) : "v"(ba), "n"(16 * G));
}
// wait until group G has landed (groups issued so far: up to min(G - 1 + LA, NG - 1))
template <int G, int NG, int LA, int NB, int R>
__device__ __forceinline__ void dot_wait(DotRing<NB, R>& r) {
  constexpr int left = (NG - 1 - G) < (LA - 1) ? (NG - 1 - G) : (LA - 1);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(R * left) : "memory");
#pragma unroll
  for (int k = 0; k < R; ++k) asm volatile("" : "+v"(r.v[G % NB][k]));
}
// packed: the products of group G (row pair x the alpha's cell, broadcast)
template <int G, int NB>
__device__ __forceinline__ void dot_products_pk(const DotRing<NB, 3>& r, f2p (&pr)[4]) {
  const f4 a0 = r.v[G % NB][0], a1 = r.v[G % NB][1], b = r.v[G % NB][2];
  pr[0] = f2p{a0.x, a0.y} * f2p{b.x, b.x};
  pr[1] = f2p{a0.z, a0.w} * f2p{b.y, b.y};
  pr[2] = f2p{a1.x, a1.y} * f2p{b.z, b.z};
  pr[3] = f2p{a1.z, a1.w} * f2p{b.w, b.w};
}
template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void dot_chunk_pk(DotRing<NB, 3>& r, uint32_t pa, uint32_t ba, f2p& acc,
                                             f2p (&pr)[4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG) dot_read_pk<G + LA, NB>(r, pa, ba);
    if constexpr (G + 1 < NG) {
      // group G + 1's products between group G's dependent adds
      dot_wait<G + 1, NG, LA, NB, 3>(r);
      f2p pn[4];
      dot_products_pk<G + 1, NB>(r, pn);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc = acc + pr[k];
        pr[k] = pn[k];
      }
      dot_chunk_pk<G + 1, NG, LA, NB>(r, pa, ba, acc, pr);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = acc + pr[k];
    }
  }
}
template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void dot_chunk_1(DotRing<NB, 2>& r, uint32_t aa, uint32_t ba, float& acc,
                                            float (&pr)[4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG) dot_read_1<G + LA, NB>(r, aa, ba);
    if constexpr (G + 1 < NG) {
      dot_wait<G + 1, NG, LA, NB, 2>(r);
      const f4 a = r.v[(G + 1) % NB][0], b = r.v[(G + 1) % NB][1];
      const float pn[4] = {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc = acc + pr[k];
        pr[k] = pn[k];
      }
      dot_chunk_1<G + 1, NG, LA, NB>(r, aa, ba, acc, pr);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = acc + pr[k];
    }
  }
}
template <int G, int LA, int NB>
__device__ __forceinline__ void dot_prologue_pk(DotRing<NB, 3>& r, uint32_t pa, uint32_t ba) {
  if constexpr (G < LA) {
    dot_read_pk<G, NB>(r, pa, ba);
    dot_prologue_pk<G + 1, LA, NB>(r, pa, ba);
  }
}
template <int G, int LA, int NB>
__device__ __forceinline__ void dot_prologue_1(DotRing<NB, 2>& r, uint32_t aa, uint32_t ba) {
  if constexpr (G < LA) {
    dot_read_1<G, NB>(r, aa, ba);
    dot_prologue_1<G + 1, LA, NB>(r, aa, ba);
  }
}

template <int RP, int A, int CH>
__global__ __launch_bounds__((RP * A + 63) / 64 * 64) void k_pair_dot_pk(
    const float* __restrict__ Ag, int na, const float* __restrict__ Bg, int nb, int ld, int n,
    float* __restrict__ out, int ldo, const int* __restrict__ alist, const int* __restrict__ acount) {
  constexpr int NT = (RP * A + 63) / 64 * 64, C4 = CH / 4;
  constexpr int PROW = 2 * CH + 4, ROW = CH + 4;  // floats; both = 4 (mod 64) banks
  constexpr int NPI = RP * C4, NAI = A * C4;      // staging items: pair float4 columns, alpha float4s
  constexpr int LP = (NPI + NT - 1) / NT, LB = (NAI + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sP = smem;
  float* sB = smem + RP * PROW;
  if (alist) na = min(na, *acount);
  const int tid = threadIdx.x;
  const int nrt = (na + 2 * RP - 1) / (2 * RP), ntiles = nrt * ((nb + A - 1) / A);
  const int t = xcd_tile(ntiles);
  if (t >= ntiles) return;  // (uniform over the block)
  const int i0 = (t % nrt) * 2 * RP, j0 = (t / nrt) * A;
  // rows through the full A (alist: any row of it), alphas from the tile's first
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)Ag, 0, kDotOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Bg + (long long)j0 * ld), 0, kDotOff, 0x00020000);
  auto arow = [&](int i) { return alist ? alist[i] : i; };
  int ro0[LP], ro1[LP];  // the staged rows' word offsets (kDotOff / 4: past the matrix)
#pragma unroll
  for (int k = 0; k < LP; ++k) {
    const int e = tid + NT * k, r = i0 + 2 * (e / C4);
    ro0[k] = e < NPI && r < na ? arow(r) * ld : kDotOff / 4;
    ro1[k] = e < NPI && r + 1 < na ? arow(r + 1) * ld : kDotOff / 4;
  }
  f4 rp0[LP], rp1[LP], rb[LB];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const int c4 = ((tid + NT * k) % C4) * 4;
      const bool in = x0 + c4 < n;
      rp0[k] = ldq_rs(rsa, in && ro0[k] != kDotOff / 4 ? (ro0[k] + x0 + c4) * 4 : kDotOff);
      rp1[k] = ldq_rs(rsa, in && ro1[k] != kDotOff / 4 ? (ro1[k] + x0 + c4) * 4 : kDotOff);
    }
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int e = tid + NT * k, a = e / C4, c4 = (e % C4) * 4;
      rb[k] = ldq_rs(rsb, e < NAI && j0 + a < nb && x0 + c4 < n ? (a * ld + x0 + c4) * 4 : kDotOff);
    }
  };
  const int q = tid < RP * A ? tid : 0, qa = q % A, qr = q / A;
  const uint32_t pa = (uint32_t)(uintptr_t)(sP + qr * PROW);
  const uint32_t ba = (uint32_t)(uintptr_t)(sB + qa * ROW);
  f2p acc = f2p{0.0f, 0.0f};
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += CH) {
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const int e = tid + NT * k;
      if (e < NPI) {
        float* d = sP + (e / C4) * PROW + (e % C4) * 8;
        *(f4*)d = f4{rp0[k].x, rp1[k].x, rp0[k].y, rp1[k].y};
        *(f4*)(d + 4) = f4{rp0[k].z, rp1[k].z, rp0[k].w, rp1[k].w};
      }
    }
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int e = tid + NT * k;
      if (e < NAI) *(f4*)(sB + (e / C4) * ROW + (e % C4) * 4) = rb[k];
    }
    __syncthreads();
    if (x0 + CH < n) fetch(x0 + CH);
    constexpr int NG = CH / 4, LA = 5, NB = LA + 1;  // 3 reads per group: lgkmcnt <= 15
    DotRing<NB, 3> ring;
    dot_prologue_pk<0, LA, NB>(ring, pa, ba);
    dot_wait<0, NG, LA, NB, 3>(ring);
    f2p pr[4];
    dot_products_pk<0, NB>(ring, pr);
    dot_chunk_pk<0, NG, LA, NB>(ring, pa, ba, acc, pr);
    __syncthreads();
  }
  if (tid < RP * A) {
    const int j = j0 + qa, i = i0 + 2 * qr;
    if (j < nb) {
      if (i < na) out[(long long)arow(i) * ldo + j] = acc[0];
      if (i + 1 < na) out[(long long)arow(i + 1) * ldo + j] = acc[1];
    }
  }
}

template <int TA, int TB, int CH>
__global__ __launch_bounds__(TA * TB) void k_pair_dot_1(
    const float* __restrict__ Ag, int na, const float* __restrict__ Bg, int nb, int ld, int n,
    float* __restrict__ out, int ldo, const int* __restrict__ alist, const int* __restrict__ acount) {
  constexpr int NT = TA * TB, C4 = CH / 4, ROW = CH + 4;
  constexpr int NI = (TA + TB) * C4, L4 = (NI + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (alist) na = min(na, *acount);
  const int tid = threadIdx.x, la = tid % TA, jb = tid / TA;
  const int nrt = (na + TA - 1) / TA, ntiles = nrt * ((nb + TB - 1) / TB);
  const int t = xcd_tile(ntiles);
  if (t >= ntiles) return;  // (uniform over the block)
  const int i0 = (t % nrt) * TA, j0 = (t / nrt) * TB;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)Ag, 0, kDotOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Bg + (long long)j0 * ld), 0, kDotOff, 0x00020000);
  auto arow = [&](int i) { return alist ? alist[i] : i; };
  int ro[L4];  // staged row e / C4: A rows first (word offsets in A), then the alphas (in B)
#pragma unroll
  for (int k = 0; k < L4; ++k) {
    const int e = tid + NT * k, r = e / C4;
    ro[k] = e >= NI ? kDotOff / 4
            : r < TA ? (i0 + r < na ? arow(i0 + r) * ld : kDotOff / 4)
                     : (j0 + r - TA < nb ? (r - TA) * ld : kDotOff / 4);
  }
  f4 rg[L4];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int e = tid + NT * k, c4 = (e % C4) * 4;
      const int off = ro[k] != kDotOff / 4 && x0 + c4 < n ? (ro[k] + x0 + c4) * 4 : kDotOff;
      rg[k] = ldq_rs(e / C4 < TA ? rsa : rsb, off);
    }
  };
  const uint32_t aa = (uint32_t)(uintptr_t)(smem + la * ROW);
  const uint32_t ba = (uint32_t)(uintptr_t)(smem + (TA + jb) * ROW);
  float acc = 0.0f;
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += CH) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int e = tid + NT * k;
      if (e < NI) *(f4*)(smem + (e / C4) * ROW + (e % C4) * 4) = rg[k];
    }
    __syncthreads();
    if (x0 + CH < n) fetch(x0 + CH);
    constexpr int NG = CH / 4, LA = 7, NB = LA + 1;  // 2 reads per group: lgkmcnt <= 15
    DotRing<NB, 2> ring;
    dot_prologue_1<0, LA, NB>(ring, aa, ba);
    dot_wait<0, NG, LA, NB, 2>(ring);
    float pr[4];
    {
      const f4 a = ring.v[0][0], b = ring.v[0][1];
      pr[0] = a.x * b.x;
      pr[1] = a.y * b.y;
      pr[2] = a.z * b.z;
      pr[3] = a.w * b.w;
    }
    dot_chunk_1<0, NG, LA, NB>(ring, aa, ba, acc, pr);
    __syncthreads();
  }
  if (i0 + la < na && j0 + jb < nb) out[(long long)arow(i0 + la) * ldo + j0 + jb] = acc;
}

template <int OP, int TA, int TB>
hipError_t launch_pair_seq(hipStream_t st, const float* A, int na, const float* B, int nb, int ld,
                           int n, float* out, int ldo, const int* alist, const int* acount) {
  static unsigned long long attr = 0ull;
  allow_lds(reinterpret_cast<const void*>(&k_pair_seq<OP, TA, TB>), attr);
  hipLaunchKernelGGL((k_pair_seq<OP, TA, TB>), dim3(cdiv(na, TA), cdiv(nb, TB)), dim3(TA * TB),
                     seq_lds(TA + TB), st, A, na, B, nb, ld, n, out, ldo, alist, acount);
  return hipGetLastError();
}

// The running sums of one row, sequentially: one wave stages 1024-value
// chunks in LDS, lane 0 walks them (4 values per LDS read, the next reads
// issued ahead), the wave stores the running sums; sum[0] = the total.
// (std::partial_sum / accumulate from +0, x-ordered, search_tree_cuda.cu:
// 176-183, 225-229.)
constexpr int kCdfCH = 1024;
__global__ __launch_bounds__(64) void k_row_cdf_seq(const float* __restrict__ row, int n,
                                                    float* __restrict__ cdf,
                                                    float* __restrict__ sum) {
  __shared__ __attribute__((aligned(16))) float sIn[kCdfCH], sOut[kCdfCH];
  const int lane = threadIdx.x;
  float acc = 0.0f;
  for (int x0 = 0; x0 < n; x0 += kCdfCH) {
    const int m = min(kCdfCH, n - x0);
#pragma unroll
    for (int q = 0; q < kCdfCH / 256; ++q) {
      const int c4 = 4 * (lane + 64 * q);
      f4 v = f4{0, 0, 0, 0};
      if (c4 + 4 <= m) {
        v = *(const f4*)(row + x0 + c4);
      } else {
        for (int k = 0; k < 4; ++k)
          if (c4 + k < m) v[k] = row[x0 + c4 + k];
      }
      *(f4*)(sIn + c4) = v;
    }
    __syncthreads();
    if (lane == 0) {
      for (int j = 0; j + 4 <= kCdfCH; j += 4) {
        const f4 v = *(const f4*)(sIn + j);
        f4 o;
        acc = acc + v.x;
        o.x = acc;
        acc = acc + v.y;
        o.y = acc;
        acc = acc + v.z;
        o.z = acc;
        acc = acc + v.w;
        o.w = acc;
        *(f4*)(sOut + j) = o;
        if (j + 4 >= m) break;
      }
    }
    __syncthreads();
    for (int j = lane; j < m; j += 64) cdf[x0 + j] = sOut[j];
    __syncthreads();
  }
  if (lane == 0) *sum = acc;
}

// ---------------------------------------------------------------- small-grid chains
// A chain of a small grid (n <= kWalkMax cells) is bound by its own
// dependent adds, not by the chip: one wave per chain forms all n terms
// in parallel (each lane its cells' IEEE products, the reference's) into
// LDS, then lane 0 alone walks them -- 32-term blocks read 8 float4 ahead of
// their adds -- so a term costs about one dependent v_add_f32.  (A lane per
// chain instead pays the LDS delivery of both operands per term, ~20 cycles,
// tools/micro/pair_dots.hip; the exact parallel chain sets need three
// launches.)  Chains (i, j), i < na (or the first *acount entries of alist),
// j < nb: grid na x nb one-wave blocks.  CDF: one chain of A's row 0, every
// running sum to cdf, the total to out[0].
constexpr int kWalkMax = 8192;
constexpr int kWalkLA = 6, kWalkNB = 8;
// floats of LDS the terms take: n rounded up to whole walk iterations, plus
// the kWalkLA groups read ahead of the last one
__host__ __device__ constexpr int walk_cap(int n) {
  return ((n + 4 * kWalkNB - 1) / (4 * kWalkNB)) * 4 * kWalkNB + 4 * kWalkLA;
}
template <int B, int E, typename F>
__device__ __forceinline__ void static_for_h(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for_h<B + 1, E>(f);
  }
}
enum { WALK_DOT = 0, WALK_CHILD = 1, WALK_CDF = 2 };

template <int K, int LA, int NB>
__device__ __forceinline__ void walk_prologue(f4 (&ring)[NB], uint32_t base) {
  if constexpr (K < LA) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ring[K]) : "v"(base), "n"(16 * K));
    walk_prologue<K + 1, LA, NB>(ring, base);
  }
}
// group K of an iteration: read group K + LA ahead, wait for group K, its
// four dependent adds (and, for a cdf, its four running sums to LDS)
template <int K, int LA, int NB, int W, bool CDF>
__device__ __forceinline__ void walk_groups(f4 (&ring)[NB], uint32_t ad, uint32_t od, float& acc) {
  if constexpr (K < NB) {
    asm volatile("ds_read_b128 %0, %1 offset:%2"
                 : "=v"(ring[(K + LA) % NB]) : "v"(ad), "n"(16 * (K + LA)));
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(W) : "memory");
    asm volatile("" : "+v"(ring[K]));
    const f4 v = ring[K];
    f4 r;
    acc = acc + v.x;
    r.x = acc;
    acc = acc + v.y;
    r.y = acc;
    acc = acc + v.z;
    r.z = acc;
    acc = acc + v.w;
    r.w = acc;
    if constexpr (CDF)
      asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(od), "v"(r), "n"(16 * K) : "memory");
    walk_groups<K + 1, LA, NB, W, CDF>(ring, ad, od, acc);
  }
}

template <int MODE>
__global__ __launch_bounds__(64) void k_chain_walk(const float* __restrict__ A, int na,
                                                  const float* __restrict__ B, int nb, int ld,
                                                  int n, float* __restrict__ out, int ldo,
                                                  const int* __restrict__ alist,
                                                  const int* __restrict__ acount,
                                                  float* __restrict__ cdf) {
  extern __shared__ __attribute__((aligned(16))) float sT[];  // n terms (+ n running sums)
  const int lane = threadIdx.x;
  const int i = blockIdx.x / nb, j = blockIdx.x % nb;
  if (alist && i >= *acount) return;  // (uniform)
  const int row = alist ? alist[i] : i;
  const float* __restrict__ a = A + (long long)row * ld;
  const float* __restrict__ b = MODE == WALK_CDF ? nullptr : B + (long long)j * ld;
  const int n4 = (n + 3) & ~3;
  const int tcap = walk_cap(n);  // terms + zero padding the walk reads past the end
  // the terms, 4 cells per lane per step, the loads of 8 steps in flight
  // together (cells past n are +0: they leave the chain unchanged -- it
  // starts at +0 and so is never -0)
  constexpr int KB = 8;
  for (int x0 = 4 * lane; x0 < tcap; x0 += 256 * KB) {
    f4 va[KB], vb[KB];
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const int x = x0 + 256 * q;
      va[q] = vb[q] = f4{0, 0, 0, 0};
      if (x + 3 < n) {
        va[q] = *(const f4*)(a + x);
        if (MODE != WALK_CDF) vb[q] = *(const f4*)(b + x);
      } else if (x < n) {
        for (int k = 0; k < 4; ++k)
          if (x + k < n) {
            va[q][k] = a[x + k];
            if (MODE != WALK_CDF) vb[q][k] = b[x + k];
          }
      }
    }
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const int x = x0 + 256 * q;
      if (x >= tcap) break;
      f4 t;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (MODE == WALK_DOT) t[k] = va[q][k] * vb[q][k];
        else if (MODE == WALK_CHILD) t[k] = ftz_f(vb[q][k] * ftz_f(va[q][k]));  // (a: L row, b: prediction)
        else t[k] = va[q][k];
      }
      *(f4*)(sT + x) = t;
    }
  }
  __syncthreads();
  if (lane == 0) {
    // lane 0 walks: group = 4 terms, read kWalkLA groups ahead at immediate
    // offsets with counted waits, kWalkNB groups per iteration (the padding
    // keeps every read in bounds and adds +0 past the end); in order, the
    // CDF's LDS writes count in lgkmcnt too
    constexpr int LA = kWalkLA, NB = kWalkNB, W = (MODE == WALK_CDF ? 2 : 1) * LA;
    const int ng = n4 / 4;
    const uint32_t base = (uint32_t)(uintptr_t)sT;
    const uint32_t obase = base + 4u * (uint32_t)tcap;
    f4 ring[NB];
    walk_prologue<0, LA, NB>(ring, base);
    float acc = 0.0f;
    for (int g0 = 0; g0 < ng; g0 += NB) {
      const uint32_t ad = base + 16u * (uint32_t)g0, od = obase + 16u * (uint32_t)g0;
      // a cdf's first groups have fewer than LA sums writes behind their
      // read: wait as the dot does (the writes complete too)
      if (g0 == 0) walk_groups<0, LA, NB, LA, MODE == WALK_CDF>(ring, ad, od, acc);
      else walk_groups<0, LA, NB, W, MODE == WALK_CDF>(ring, ad, od, acc);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    out[(long long)row * ldo + j] = acc;
  }
  if (MODE == WALK_CDF) {
    __syncthreads();
    for (int x = lane; x < n; x += 64) cdf[x] = sT[walk_cap(n) + x];
  }
}

// The same walk with its terms formed beside it (PP2_CHAIN_WALK=2; no faster
// on the node's plan step, profiles/r05/chain_walk2_ab.txt): wave 1 forms
// chunk k's terms (and loads chunk k + 1's cells) while lane 0 of wave 0
// walks chunk k - 1, one barrier per chunk, terms (and a cdf's running sums)
// double-buffered in LDS -- k_chain_walk forms all n terms before its walk
// starts.  Same terms, same order of adds: bit-identical results.
constexpr int kWalk2C = 512;  // terms per chunk: whole walk iterations (4 * kWalkNB)
static_assert(kWalk2C % (4 * kWalkNB) == 0 && kWalk2C % 256 == 0, "whole iterations, whole lane steps");
template <int MODE>
__global__ __launch_bounds__(128) void k_chain_walk2(const float* __restrict__ A, int na,
                                                    const float* __restrict__ B, int nb, int ld,
                                                    int n, float* __restrict__ out, int ldo,
                                                    const int* __restrict__ alist,
                                                    const int* __restrict__ acount,
                                                    float* __restrict__ cdf) {
  constexpr int C = kWalk2C, CP = C + 4 * kWalkLA, Q = C / 256;
  constexpr bool CDF = MODE == WALK_CDF;
  __shared__ __attribute__((aligned(16))) float sT[2][CP];  // terms (+ the walk's read-ahead slack)
  __shared__ __attribute__((aligned(16))) float sS[2][CDF ? C : 4];  // a cdf's running sums
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = blockIdx.x / nb, j = blockIdx.x % nb;
  if (alist && i >= *acount) return;  // (uniform over the block)
  const int row = alist ? alist[i] : i;
  const float* __restrict__ a = A + (long long)row * ld;
  const float* __restrict__ b = CDF ? nullptr : B + (long long)j * ld;
  const int nch = (n + C - 1) / C;
  // wave 1: the cells of chunk k, 4 per lane per 256-cell step (past n: +0,
  // which leaves the chain unchanged -- it starts at +0, so is never -0)
  f4 va[Q], vb[Q];
  auto load = [&](int k) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int x = k * C + 4 * lane + 256 * q;
      va[q] = vb[q] = f4{0, 0, 0, 0};
      if (x + 3 < n) {
        va[q] = *(const f4*)(a + x);
        if (!CDF) vb[q] = *(const f4*)(b + x);
      } else if (x < n) {
        for (int c = 0; c < 4; ++c)
          if (x + c < n) {
            va[q][c] = a[x + c];
            if (!CDF) vb[q][c] = b[x + c];
          }
      }
    }
  };
  float acc = 0.0f;
  if (w == 1) load(0);
  for (int k = 0; k <= nch; ++k) {
    if (w == 1) {
      if (k < nch) {
        float* t = sT[k & 1];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          f4 tv;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (MODE == WALK_DOT) tv[c] = va[q][c] * vb[q][c];
            else if (MODE == WALK_CHILD) tv[c] = ftz_f(vb[q][c] * ftz_f(va[q][c]));  // (a: L row, b: prediction)
            else tv[c] = va[q][c];
          }
          *(f4*)(t + 4 * lane + 256 * q) = tv;
        }
        if (k + 1 < nch) load(k + 1);  // in flight during the next walk
      }
      if (CDF && k >= 2)  // chunk k - 2's running sums (written in iteration k - 1)
        for (int x = lane; x < C && (k - 2) * C + x < n; x += 64) cdf[(k - 2) * C + x] = sS[k & 1][x];
    } else if (k >= 1 && lane == 0) {
      // lane 0 walks chunk k - 1: group = 4 terms, read kWalkLA groups ahead
      // (the last ones into the buffer's slack, unused) with counted waits
      constexpr int LA = kWalkLA, NB = kWalkNB, W = (CDF ? 2 : 1) * LA;
      const uint32_t base = (uint32_t)(uintptr_t)sT[(k - 1) & 1];
      const uint32_t obase = (uint32_t)(uintptr_t)sS[(k - 1) & 1];
      f4 ring[NB];
      walk_prologue<0, LA, NB>(ring, base);
      // (the first NB groups: fewer than LA sums writes behind each read, so
      // the dot's count; the writes complete too)
      walk_groups<0, LA, NB, LA, CDF>(ring, base, obase, acc);
      for (int g0 = NB; g0 < C / 4; g0 += NB)
        walk_groups<0, LA, NB, W, CDF>(ring, base + 16u * (uint32_t)g0, obase + 16u * (uint32_t)g0, acc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the sums and reads done before the barrier)
    }
    __syncthreads();
  }
  if (CDF) {  // the last chunk's running sums
    const int k = nch - 1;
    for (int x = tid; x < C && k * C + x < n; x += 128) cdf[k * C + x] = sS[k & 1][x];
  }
  if (w == 0 && lane == 0) out[(long long)row * ldo + j] = acc;
}

// ---------------------------------------------------------------- sampling
// find_if(partial_sum >= r) over `cnt` values at stride `stride`; when the
// sum never reaches r, the last index at which it grew (the reference would
// run past the end).
__device__ __forceinline__ int sample_small(const float* p, long long stride, int cnt, float r) {
  float acc = 0.0f;
  int last = 0;
  for (int j = 0; j < cnt; ++j) {
    const float prev = acc;
    acc = acc + p[(long long)j * stride];
    if (acc >= r) return j;
    if (acc != prev) last = j;
  }
  return last;
}

__global__ __launch_bounds__(256) void k_pbvi_sample(Geom g, PlaneSet T, PlaneSet L,
                                                     const float* __restrict__ cdf, int ld,
                                                     int rows, const float* __restrict__ rnd,
                                                     uint8_t* __restrict__ z_out,
                                                     int* __restrict__ s_out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= 9 * rows) return;
  const int i = c / 9, a = c - 9 * i;
  const int W = g.width, H = g.rows, n = H * W;
  const float* __restrict__ cd = cdf + (long long)i * ld;
  const float r1 = rnd[3 * c], r2 = rnd[3 * c + 1], r3 = rnd[3 * c + 2];
  // the cdf is non-decreasing: lower_bound is find_if(x >= r1)
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cd[mid] >= r1) hi = mid; else lo = mid + 1;
  }
  if (lo >= n) {  // first index at which the sum reaches its final value
    const float last = cd[n - 1];
    lo = 0;
    hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cd[mid] >= last) hi = mid; else lo = mid + 1;
    }
  }
  const int s = lo, ys = s / W, xs = s - ys * W;
  const int nl = sample_small(T.p + (long long)ys * T.rs + (long long)(9 * a) * T.ps + xs, T.ps,
                              9, r2);
  int ny = ys + nl / 3 - 1, nx = xs + nl % 3 - 1;
  if (ny < 0 || ny >= H || nx < 0 || nx >= W) ny = ys, nx = xs;  // rand() == 0 on a zero entry
  const int z = sample_small(L.p + (long long)ny * L.rs + nx, L.ps, 16, r3);
  z_out[c] = (uint8_t)z;
  if (s_out) s_out[c] = s;
}

__global__ __launch_bounds__(256) void k_pbvi_pick(const float* __restrict__ l1, int ldo, int n,
                                                   int nset, float* __restrict__ best_l1,
                                                   int* __restrict__ best_a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float m[9];
  for (int a = 0; a < 9; ++a) {
    const float* row = l1 + (long long)(9 * i + a) * ldo;
    float v = FLT_MAX;
    for (int j = 0; j < nset; ++j)
      if (row[j] < v) v = row[j];
    m[a] = v;
  }
  int ba = 0;
  for (int a = 1; a < 9; ++a)
    if (m[ba] < m[a]) ba = a;
  best_a[i] = ba;
  best_l1[i] = m[ba];
}

// ---------------------------------------------------------------- MFMA GEMM
// C[i][k] = sum_x A[i][x] * B[k][x] with x in ascending order: each
// v_mfma_f32_32x32x2_f32 step is fma(a[x+1], b[x+1], fma(a[x], b[x], c)),
// lane half h holding x = 2t + h.  128x128 tiles, 4 waves of 64x64 (2x2
// MFMA blocks), x-chunks of GK staged through LDS with each row's 8-float
// groups stored as [h][s] (x = 8q + 2s + h -> 8q + 4h + s) so a lane reads
// four consecutive steps with one ds_read_b128.  The next chunk's global
// loads and LDS stores overlap the current chunk's MFMAs (double-buffered
// LDS, one barrier per chunk), and each 4-step group's fragments are read
// while the previous group multiplies.
constexpr int GT = kGemmTile, GK = 32, GLD = GK + 4;
constexpr int GQ = GK / 8;               // 8-float groups per row chunk
constexpr int GPAIRS = GT * GQ / 256;    // (row, group) pairs per thread per operand

__global__ __launch_bounds__(256, 2) void k_gemm_nt(const float* __restrict__ A,
                                                    const float* __restrict__ B,
                                                    float* __restrict__ C, int Mp, int Np, int ld,
                                                    long long bstride, long long cstride,
                                                    int ksplit, int kchunk, long long sstride) {
  __shared__ __attribute__((aligned(16))) float sA[2][GT * GLD];
  __shared__ __attribute__((aligned(16))) float sB[2][GT * GLD];
  const int ti_n = Mp / GT, tk_n = Np / GT;
  const int L = xcd_map(blockIdx.x, gridDim.x);
  const int ti = L % ti_n;
  int rest = L / ti_n;
  const int tk = rest % tk_n;
  rest /= tk_n;
  const int sp = rest % ksplit, z = rest / ksplit;
  const int i0 = ti * GT, k0 = tk * GT;
  const int xb = sp * kchunk, xe = min(ld, xb + kchunk);
  const float* __restrict__ Ab = A + (long long)i0 * ld;
  const float* __restrict__ Bb = B + z * bstride + (long long)k0 * ld;
  float* __restrict__ Cb = C + z * cstride + sp * sstride;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wi = w & 1, wk = w >> 1;
  const int r = lane & 31, h = lane >> 5;

  f4 ra[GPAIRS][2], rb[GPAIRS][2];
  auto gload = [&](int x0) {
#pragma unroll
    for (int q = 0; q < GPAIRS; ++q) {
      const int p = tid + 256 * q, row = p / GQ, c8 = (p % GQ) * 8;
      const f4* pa = (const f4*)(Ab + (long long)row * ld + x0 + c8);
      const f4* pb = (const f4*)(Bb + (long long)row * ld + x0 + c8);
      ra[q][0] = pa[0];
      ra[q][1] = pa[1];
      rb[q][0] = pb[0];
      rb[q][1] = pb[1];
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < GPAIRS; ++q) {
      const int p = tid + 256 * q, row = p / GQ, c8 = (p % GQ) * 8;
      float* da = sA[buf] + row * GLD + c8;
      float* db = sB[buf] + row * GLD + c8;
      *(f4*)da = f4{ra[q][0].x, ra[q][0].z, ra[q][1].x, ra[q][1].z};
      *(f4*)(da + 4) = f4{ra[q][0].y, ra[q][0].w, ra[q][1].y, ra[q][1].w};
      *(f4*)db = f4{rb[q][0].x, rb[q][0].z, rb[q][1].x, rb[q][1].z};
      *(f4*)(db + 4) = f4{rb[q][0].y, rb[q][0].w, rb[q][1].y, rb[q][1].w};
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[ib][kb][v] = 0.0f;

  // LDS double buffer: chunk c is multiplied from buffer c&1 while chunk c+1
  // goes global -> registers -> buffer (c+1)&1; one barrier per chunk.
  if (xb < xe) {
    gload(xb);
    lstore(0);
  }
  __syncthreads();
  int buf = 0;
  for (int x0 = xb; x0 < xe; x0 += GK) {
    const bool more = x0 + GK < xe;
    if (more) gload(x0 + GK);
    const float* __restrict__ pa = sA[buf] + (wi * 64 + r) * GLD + 4 * h;
    const float* __restrict__ pb = sB[buf] + (wk * 64 + r) * GLD + 4 * h;
    f4 a[2], b[2], an[2], bn[2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) a[ib] = *(const f4*)(pa + ib * 32 * GLD);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) b[kb] = *(const f4*)(pb + kb * 32 * GLD);
#pragma unroll
    for (int q = 0; q < GQ; ++q) {
      if (q + 1 < GQ) {  // next group's fragments in flight during this group's MFMAs
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) an[ib] = *(const f4*)(pa + ib * 32 * GLD + 8 * (q + 1));
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) bn[kb] = *(const f4*)(pb + kb * 32 * GLD + 8 * (q + 1));
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
            acc[ib][kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ib][s], b[kb][s], acc[ib][kb],
                                                               0, 0, 0);
      if (q + 1 < GQ) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          a[e] = an[e];
          b[e] = bn[e];
        }
      }
    }
    if (more) lstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // C/D map of the 32x32 forms: register v of lane l is row (v&3) + 8(v>>2) + 4h, column r
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int i = i0 + wi * 64 + ib * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        const int k = k0 + wk * 64 + kb * 32 + r;
        Cb[(long long)i * Np + k] = acc[ib][kb][v];
      }
}

__global__ __launch_bounds__(256) void k_argmax_rows(const float* __restrict__ C, int rows, int n,
                                                     int ldc, int* __restrict__ out,
                                                     float* __restrict__ vmax) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* __restrict__ p = C + (long long)row * ldc;
  float bv = -INFINITY;
  int bi = INT_MAX;
  // 8 loads per lane in flight together (a row of S <= 512 alphas in one go)
  for (int k0 = lane; k0 < n; k0 += 512) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = k0 + 64 * q < n ? p[k0 + 64 * q] : 0.0f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = k0 + 64 * q;
      if (k < n && (bi == INT_MAX || v[q] > bv)) {
        bv = v[q];
        bi = k;
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float ov = __shfl_xor(bv, off);
    const int oi = __shfl_xor(bi, off);
    if (oi != INT_MAX && (bi == INT_MAX || ov > bv || (ov == bv && oi < bi))) {
      bv = ov;
      bi = oi;
    }
  }
  if (lane == 0) {
    out[row] = bi;
    if (vmax) vmax[row] = bv;
  }
}

__global__ __launch_bounds__(256) void k_pbvi_gamma_a(Geom g, PlaneSet R,
                                                      const float* __restrict__ G,
                                                      long long gstride, int ld, int a0,
                                                      const int* __restrict__ kstar, int kstride,
                                                      float* __restrict__ Ga) {
  const int W = g.width, H = g.rows;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= H * W) return;
  const int i = blockIdx.y, y = idx / W, x = idx - y * W;
  const int a = a0 + blockIdx.z;
  G += (long long)blockIdx.z * 16 * gstride;
  kstar += blockIdx.z * 16 * kstride;
  Ga += (long long)a * gstride;
  float v = R.p[(long long)y * R.rs + (long long)a * R.ps + x];
#pragma unroll
  for (int o = 0; o < 16; ++o)
    v = v + G[o * gstride + (long long)kstar[o * kstride + i] * ld + idx];
  Ga[(long long)i * ld + idx] = v;
}

__global__ __launch_bounds__(256) void k_pbvi_select(const float* __restrict__ V,
                                                     const float* __restrict__ Ga, int Sp, int ld,
                                                     float* __restrict__ alpha_out,
                                                     uint8_t* __restrict__ actions) {
  const int i = blockIdx.y, x = blockIdx.x * 256 + threadIdx.x;
  float opt = -FLT_MAX;
  int oa = 0;
  for (int a = 0; a < 9; ++a) {
    const float v = V[a * Sp + i];
    if (v > opt) {
      opt = v;
      oa = a;
    }
  }
  if (x < ld) alpha_out[(long long)i * ld + x] = Ga[((long long)oa * Sp + i) * ld + x];
  if (blockIdx.x == 0 && threadIdx.x == 0) actions[i] = (uint8_t)oa;
}

__global__ __launch_bounds__(256) void k_sum_splits(const float* __restrict__ C, int splits,
                                                    long long sstride, int n,
                                                    float* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  float v = C[e];
  for (int s = 1; s < splits; ++s) v = v + C[s * sstride + e];
  out[e] = v;
}


}  // namespace

hipError_t launch_rows_seq(hipStream_t st, int mode, const float* A, int ld, int rows, int n,
                           float* sums, float* cdf) {
  if (rows <= 0) return hipSuccess;
  const dim3 grid(cdiv(rows, kChainRows));
  if (mode == ROW_CDF)
    hipLaunchKernelGGL(k_rows_chain<CH_CDF>, grid, dim3(256), 0, st, A, rows, nullptr, ld, rows,
                       n, sums, cdf);
  else
    hipLaunchKernelGGL(k_rows_chain<CH_SUM>, grid, dim3(256), 0, st, A, rows, nullptr, ld, rows,
                       n, sums, nullptr);
  return hipGetLastError();
}

hipError_t launch_lane_sums(hipStream_t st, const float* A, int ld, int rows, int n,
                            float* sums) {
  if (rows <= 0) return hipSuccess;
  if (ld % 4 != 0) return hipErrorInvalidValue;
  if (rows == 1)
    hipLaunchKernelGGL((k_lane_chains<CH_SUM, 1>), dim3(1), dim3(64), 0, st, A, rows, 1, nullptr,
                       0, 1, ld, n, sums, 1);
  else  // 4 rows per block: ~0.16 us of LDS-DMA per 0.43-us chunk of adds
    hipLaunchKernelGGL((k_lane_chains<CH_SUM, 4>), dim3(cdiv(rows, 4)), dim3(64), 0, st, A, rows,
                       4, nullptr, 0, 1, ld, n, sums, 1);
  return hipGetLastError();
}

hipError_t launch_lane_dots(hipStream_t st, const float* A, int na, const float* B, int nb,
                            int ld, int n, float* out, int ldo) {
  if (na <= 0 || nb <= 0) return hipSuccess;
  if (ld % 4 != 0) return hipErrorInvalidValue;
  // 3 A rows x 3 B rows per block: 9 chains, 6 rows staged per chunk
  hipLaunchKernelGGL((k_lane_chains<CH_DOT, 6>), dim3(cdiv(na, 3), cdiv(nb, 3)), dim3(64), 0, st,
                     A, na, 3, B, nb, 3, ld, n, out, ldo);
  return hipGetLastError();
}

hipError_t launch_rows_div(hipStream_t st, float* A, int ld, int rows, int n,
                           const float* sums) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rows_div, dim3(cdiv(n, 256), rows), dim3(256), 0, st, A, ld, n, sums);
  return hipGetLastError();
}

hipError_t launch_rows_dot(hipStream_t st, const float* A, int amod, const float* B, int ld,
                           int rows, int n, float* out) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rows_chain<CH_DOT>, dim3(cdiv(rows, kChainRows)), dim3(256), 0, st, A,
                     amod, B, ld, rows, n, out, nullptr);
  return hipGetLastError();
}

// The planner's PBVI leaf dots: one chain per lane with the child rows
// through DPP broadcasts (k_pair_dot_bq, pp2_pbvi_dots.hip) by default;
// PP2_PAIR_DOT: 3 that, 2 one chain per lane from LDS (k_pair_dot_1; beside
// the FIB dots 0-10 % faster than the packed shape,
// profiles/r05/pbvi_plan_dots_*.txt), 1 packed, 0 k_pair_seq.
static hipError_t launch_pair_dot(hipStream_t st, const float* A, int na, const float* B, int nb,
                                  int ld, int n, float* out, int ldo, const int* alist,
                                  const int* acount) {
  const char* env = getenv("PP2_PAIR_DOT");
  const int mode = env && *env ? atoi(env) : 3;
  // 32-bit buffer offsets: the rows (alist entries index the na rows of A)
  // and a tile's alphas
  const bool fits = (long long)na * ld < (long long)kDotOff / 4 && 18LL * ld < (long long)kDotOff / 4;
  if (mode == 0 || !fits)
    return launch_pair_seq<PAIR_DOT, 16, 16>(st, A, na, B, nb, ld, n, out, ldo, alist, acount);
  if (mode == 3) return launch_pair_dot_bq(st, A, na, B, nb, ld, n, out, ldo, alist, acount);
  if (mode == 2) {
    constexpr int TA = 16, TB = 16, CH = 512;
    static unsigned long long attr = 0ull;
    allow_lds(reinterpret_cast<const void*>(&k_pair_dot_1<TA, TB, CH>), attr);
    const int tiles = cdiv(na, TA) * cdiv(nb, TB);
    hipLaunchKernelGGL((k_pair_dot_1<TA, TB, CH>), dim3(cdiv(tiles, 8) * 8), dim3(TA * TB),
                       (size_t)(TA + TB) * (CH + 4) * sizeof(float), st, A, na, B, nb, ld, n, out, ldo,
                       alist, acount);
    return hipGetLastError();
  }
  constexpr int RP = 8, AL = 18, CH = 512;  // 144 x 500: 9 x 28 = 252 blocks, one per CU
  static unsigned long long attr = 0ull;
  allow_lds(reinterpret_cast<const void*>(&k_pair_dot_pk<RP, AL, CH>), attr);
  const int tiles = cdiv(na, 2 * RP) * cdiv(nb, AL);
  hipLaunchKernelGGL((k_pair_dot_pk<RP, AL, CH>), dim3(cdiv(tiles, 8) * 8), dim3((RP * AL + 63) / 64 * 64),
                     (size_t)(RP * (2 * CH + 4) + AL * (CH + 4)) * sizeof(float), st, A, na, B, nb, ld,
                     n, out, ldo, alist, acount);
  return hipGetLastError();
}

hipError_t launch_pair_chain(hipStream_t st, int op, const float* A, int na, const float* B,
                             int nb, int ld, int n, float* out, int ldo, const int* alist,
                             const int* acount) {
  if (na <= 0 || nb <= 0) return hipSuccess;
  if ((alist == nullptr) != (acount == nullptr)) return hipErrorInvalidValue;
  // the large shape while it gives the CUs a block each, else the small one
#ifndef PP2_PAIR_NC  // (A/B builds: chains per thread of the small shape)
#define PP2_PAIR_NC 1
#endif
#ifndef PP2_PAIR_CH
#define PP2_PAIR_CH 128
#endif
  constexpr int kNc = PP2_PAIR_NC, kCh = PP2_PAIR_CH;
  const bool big = (long long)cdiv(na, 64) * cdiv(nb, 64) >= 256;
  // few long chains (the planner's PBVI leaf dots): the lookahead kernel
  const char* seq = getenv("PP2_PAIR_SEQ");
  if (!big && n >= 1024 && !(seq && seq[0] == '0')) {
    if (op == PAIR_L1)
      return launch_pair_seq<PAIR_L1, 16, 16>(st, A, na, B, nb, ld, n, out, ldo, alist, acount);
    if (op == PAIR_CHILD)
      return launch_pair_seq<PAIR_CHILD, 16, 16>(st, A, na, B, nb, ld, n, out, ldo, alist, acount);
    return launch_pair_dot(st, A, na, B, nb, ld, n, out, ldo, alist, acount);
  }
  const dim3 grid = big ? dim3(cdiv(na, 64), cdiv(nb, 64)) : dim3(cdiv(na, 16), cdiv(nb, 16 * kNc));
#define PP2_PAIR(OPV, TAV, NCV, CHV)                                                        \
  hipLaunchKernelGGL((k_pair_chain<OPV, TAV, NCV, CHV>), grid, dim3(256), 0, st, A, na, B, nb, ld, \
                     n, out, ldo, alist, acount)
  if (op == PAIR_L1) {
    if (big) PP2_PAIR(PAIR_L1, 64, 16, 32);
    else PP2_PAIR(PAIR_L1, 16, kNc, kCh);
  } else {
    if (big) PP2_PAIR(PAIR_DOT, 64, 16, 32);
    else PP2_PAIR(PAIR_DOT, 16, kNc, kCh);
  }
#undef PP2_PAIR
  return hipGetLastError();
}

hipError_t launch_pair_seq_small(hipStream_t st, int op, const float* A, int na, const float* B,
                                 int nb, int ld, int n, float* out, int ldo, const int* alist,
                                 const int* acount) {
  if (na <= 0 || nb <= 0) return hipSuccess;
  if ((alist == nullptr) != (acount == nullptr) || n <= 0 || ld < n) return hipErrorInvalidValue;
  if (op != PAIR_DOT && op != PAIR_CHILD) return hipErrorInvalidValue;
  const char* env = getenv("PP2_CHAIN_WALK");
  if (n <= kWalkMax && env && env[0] == '2') {
    // PP2_CHAIN_WALK=2: the walk with its terms formed beside it (two waves per chain)
    if (op == PAIR_DOT)
      hipLaunchKernelGGL(k_chain_walk2<WALK_DOT>, dim3(na * nb), dim3(128), 0, st, A, na, B, nb, ld, n,
                         out, ldo, alist, acount, nullptr);
    else
      hipLaunchKernelGGL(k_chain_walk2<WALK_CHILD>, dim3(na * nb), dim3(128), 0, st, A, na, B, nb, ld,
                         n, out, ldo, alist, acount, nullptr);
    return hipGetLastError();
  }
  if (n <= kWalkMax && !(env && env[0] == '0')) {
    // one wave per chain, all terms formed, then lane 0 walks them
    const size_t lds = (size_t)walk_cap(n) * sizeof(float);
    static unsigned long long attr[2] = {0ull, 0ull};
    allow_lds(reinterpret_cast<const void*>(&k_chain_walk<WALK_DOT>), attr[0]);
    allow_lds(reinterpret_cast<const void*>(&k_chain_walk<WALK_CHILD>), attr[1]);
    if (op == PAIR_DOT)
      hipLaunchKernelGGL(k_chain_walk<WALK_DOT>, dim3(na * nb), dim3(64), lds, st, A, na, B, nb, ld,
                         n, out, ldo, alist, acount, nullptr);
    else
      hipLaunchKernelGGL(k_chain_walk<WALK_CHILD>, dim3(na * nb), dim3(64), lds, st, A, na, B, nb,
                         ld, n, out, ldo, alist, acount, nullptr);
    return hipGetLastError();
  }
  // one wave per block (4 A rows x 16 B rows): few chains, each block on a CU of its own
  if (op == PAIR_DOT)
    return launch_pair_seq<PAIR_DOT, 4, 16>(st, A, na, B, nb, ld, n, out, ldo, alist, acount);
  return launch_pair_seq<PAIR_CHILD, 4, 16>(st, A, na, B, nb, ld, n, out, ldo, alist, acount);
}

hipError_t launch_row_cdf_seq(hipStream_t st, const float* row, int n, float* cdf, float* sum) {
  if (n <= 0 || !row || !cdf || !sum) return hipErrorInvalidValue;
  const char* env = getenv("PP2_CHAIN_WALK");
  if (n <= kWalkMax && env && env[0] == '2') {
    hipLaunchKernelGGL(k_chain_walk2<WALK_CDF>, dim3(1), dim3(128), 0, st, row, 1, nullptr, 1, n, n, sum,
                       0, nullptr, nullptr, cdf);
    return hipGetLastError();
  }
  if (n <= kWalkMax && !(env && env[0] == '0')) {
    const size_t lds = 2 * (size_t)walk_cap(n) * sizeof(float);
    static unsigned long long attr = 0ull;
    allow_lds(reinterpret_cast<const void*>(&k_chain_walk<WALK_CDF>), attr);
    hipLaunchKernelGGL(k_chain_walk<WALK_CDF>, dim3(1), dim3(64), lds, st, row, 1, nullptr, 1, n,
                       n, sum, 0, nullptr, nullptr, cdf);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_row_cdf_seq, dim3(1), dim3(64), 0, st, row, n, cdf, sum);
  return hipGetLastError();
}

hipError_t launch_pbvi_sample(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet L,
                              const float* cdf, int ld, int rows, const float* rnd,
                              uint8_t* z_out, int* s_out) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pbvi_sample, dim3(cdiv(9LL * rows, 256)), dim3(256), 0, st, g, T, L, cdf,
                     ld, rows, rnd, z_out, s_out);
  return hipGetLastError();
}

hipError_t launch_pbvi_pick(hipStream_t st, const float* l1, int ldo, int n, int nset,
                            float* best_l1, int* best_a) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pbvi_pick, dim3(cdiv(n, 256)), dim3(256), 0, st, l1, ldo, n, nset,
                     best_l1, best_a);
  return hipGetLastError();
}

int gemm_kchunk(int ld, int ksplit) {
  const int kchunk = (ld + ksplit - 1) / ksplit;
  return (kchunk + GK - 1) / GK * GK;
}

hipError_t launch_gemm_nt(hipStream_t st, const float* A, const float* B, float* C, int Mp,
                          int Np, int ld, int batch, long long bstride, long long cstride,
                          int ksplit, long long sstride) {
  if (Mp % GT || Np % GT || ld % GK || ksplit < 1) return hipErrorInvalidValue;
  const int kchunk = gemm_kchunk(ld, ksplit);
  const long long blocks = (long long)(Mp / GT) * (Np / GT) * ksplit * batch;
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gemm_nt, dim3((unsigned)blocks), dim3(256), 0, st, A, B, C, Mp, Np, ld,
                     bstride, cstride, ksplit, kchunk, sstride);
  return hipGetLastError();
}

hipError_t launch_argmax_rows(hipStream_t st, const float* C, int rows, int n, int ldc, int* out,
                              float* vmax) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_argmax_rows, dim3(cdiv(rows, 4)), dim3(256), 0, st, C, rows, n, ldc, out,
                     vmax);
  return hipGetLastError();
}

hipError_t launch_pbvi_gamma_a(hipStream_t st, const Geom& g, PlaneSet R, const float* G,
                               long long gstride, int ld, int S, int a0, int a1,
                               const int* kstar, int kstride, float* Ga) {
  if (S <= 0 || a1 <= a0) return hipSuccess;
  dim3 grid(cdiv((long long)g.rows * g.width, 256), S, a1 - a0);
  hipLaunchKernelGGL(k_pbvi_gamma_a, grid, dim3(256), 0, st, g, R, G, gstride, ld, a0, kstar,
                     kstride, Ga);
  return hipGetLastError();
}

hipError_t launch_pbvi_select(hipStream_t st, const float* V, const float* Ga, int Sp, int S,
                              int ld, float* alpha_out, uint8_t* actions) {
  if (S <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pbvi_select, dim3(cdiv(ld, 256), S), dim3(256), 0, st, V, Ga, Sp, ld,
                     alpha_out, actions);
  return hipGetLastError();
}

hipError_t launch_sum_splits(hipStream_t st, const float* C, int splits, long long sstride,
                             int n, float* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_sum_splits, dim3(cdiv(n, 256)), dim3(256), 0, st, C, splits, sstride, n,
                     out);
  return hipGetLastError();
}

}  // namespace pp2
