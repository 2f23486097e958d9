// The planner's reference-order PBVI leaf dots in isolation: na rows (the
// expansion's normalised children) x nb alphas, each pair one x-ordered fp32
// chain acc = acc + a[x] * b[x] (evaluatePbviCpu,
// point_based_value_iteration_cuda.cu:678-699), n cells.  Times the library's
// k_pair_seq shape (16 x 16 pairs per block, one chain per lane) against
// register-tiled shapes in which each wave holds RR rows (the same for every
// lane: uniform LDS reads) and each lane CA alphas, the RR x CA chains of a
// lane advancing together as packed fp32 ops (v_pk_mul_f32 / v_pk_add_f32:
// the same IEEE products and sums as the scalar ops).  Every variant's
// results are compared bit for bit with the first one, and a sample of
// chains with the host's sequential fp32 loop.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form=1 -o tools/micro/pair_dots tools/micro/pair_dots.hip
//   tools/micro/pair_dots [na nb n]     (default 144 500 65536: 256^2, S = 500)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <cmath>
#include <type_traits>
#include <vector>

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      exit(1);                                                       \
    }                                                                \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

static int cdiv(long long a, int b) { return (int)((a + b - 1) / b); }

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// ---------------------------------------------------------------- v0: the library shape
constexpr int kCH = 512, kRow = kCH + 4;

// XCD: the grid is 1-D; block L runs on XCD L % 8 (dispatch order), and
// the tiles are numbered so that each XCD's blocks cover whole alpha tiles
// against every row tile (the alphas' chunks then come from that XCD's L2)
template <bool XCD>
__global__ __launch_bounds__(256) void k_v0(const float* __restrict__ A, int na,
                                            const float* __restrict__ B, int nb, int ld, int n,
                                            float* __restrict__ out, int ldo) {
  constexpr int TA = 16, TB = 16, NT = 256;
  constexpr int LA4 = TA * 128 / NT, LB4 = TB * 128 / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sA = smem;
  float* sB = smem + TA * kRow;
  const int tid = threadIdx.x, la = tid % TA, jb = tid / TA;
  int bx = blockIdx.x, by = blockIdx.y;
  if (XCD) {
    const int nrt = (na + TA - 1) / TA, ntiles = nrt * ((nb + TB - 1) / TB);
    const int per = (gridDim.x + 7) / 8, t = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (t >= ntiles) return;
    bx = t % nrt;
    by = t / nrt;
  }
  const int i0 = bx * TA, j0 = by * TB;
  f4 ra[LA4], rb[LB4];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int q = 0; q < LA4; ++q) {
      const int e = tid + NT * q, row = e >> 7, c4 = (e & 127) * 4, ia = i0 + row;
      ra[q] = ia < na && x0 + c4 < n ? *(const f4*)(A + (long long)ia * ld + x0 + c4) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int q = 0; q < LB4; ++q) {
      const int e = tid + NT * q, row = e >> 7, c4 = (e & 127) * 4, jj = j0 + row;
      rb[q] = jj < nb && x0 + c4 < n ? *(const f4*)(B + (long long)jj * ld + x0 + c4) : f4{0, 0, 0, 0};
    }
  };
  const uint32_t la_addr = (uint32_t)(uintptr_t)(sA + la * kRow);
  const uint32_t lb_addr = (uint32_t)(uintptr_t)(sB + jb * kRow);
  float acc = 0.0f;
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += kCH) {
#pragma unroll
    for (int q = 0; q < LA4; ++q) {
      const int e = tid + NT * q;
      *(f4*)(sA + (e >> 7) * kRow + (e & 127) * 4) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < LB4; ++q) {
      const int e = tid + NT * q;
      *(f4*)(sB + (e >> 7) * kRow + (e & 127) * 4) = rb[q];
    }
    __syncthreads();
    if (x0 + kCH < n) fetch(x0 + kCH);
    constexpr int G = 8, NG = kCH / G, R = 4, LA = 3, NB = LA + 1;
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
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(LA * R) : "memory");
      } else if (g + 2 < NG) {
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(2 * R) : "memory");
      } else if (g + 1 < NG) {
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(R) : "memory");
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
        acc = acc + a.x * b.x;
        acc = acc + a.y * b.y;
        acc = acc + a.z * b.z;
        acc = acc + a.w * b.w;
      }
    }
    __syncthreads();
  }
  if (i0 + la < na && j0 + jb < nb) out[(long long)(i0 + la) * ldo + j0 + jb] = acc;
}

// ---------------------------------------------------------------- register tiles
// Block = W waves sharing 64*CA alphas (LDS, row-major); wave w owns rows
// i0 + w*RR .. +RR (LDS, read at one address by every lane); lane l owns
// alphas j0 + l + 64*c.  CH cells per chunk, staged through registers
// loaded one chunk ahead.  Per 4 cells a lane issues RR + CA ds_read_b128.
template <int RR, int CA, int W, int CH>
__global__ __launch_bounds__(64 * W) void k_tile(const float* __restrict__ A, int na,
                                                 const float* __restrict__ B, int nb, int ld,
                                                 int n, float* __restrict__ out, int ldo) {
  static_assert(RR % 2 == 0 || CA % 2 == 0, "pairs of chains per packed op");
  constexpr int NT = 64 * W, ROW = CH + 4, NRA = W * RR, NRB = 64 * CA;
  constexpr int C4 = CH / 4;                       // float4 per row per chunk
  constexpr int LA4 = (NRA * C4 + NT - 1) / NT, LB4 = (NRB * C4 + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sA = smem;
  float* sB = smem + NRA * ROW;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int i0 = blockIdx.x * NRA, j0 = blockIdx.y * NRB;
  f4 ra[LA4], rb[LB4];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int q = 0; q < LA4; ++q) {
      const int e = tid + NT * q, row = e / C4, c4 = (e % C4) * 4, ia = i0 + row;
      ra[q] = e < NRA * C4 && ia < na && x0 + c4 < n ? *(const f4*)(A + (long long)ia * ld + x0 + c4)
                                                    : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int q = 0; q < LB4; ++q) {
      const int e = tid + NT * q, row = e / C4, c4 = (e % C4) * 4, jj = j0 + row;
      rb[q] = e < NRB * C4 && jj < nb && x0 + c4 < n ? *(const f4*)(B + (long long)jj * ld + x0 + c4)
                                                    : f4{0, 0, 0, 0};
    }
  };
  uint32_t a_addr[RR], b_addr[CA];
#pragma unroll
  for (int r = 0; r < RR; ++r) a_addr[r] = (uint32_t)(uintptr_t)(sA + (w * RR + r) * ROW);
#pragma unroll
  for (int c = 0; c < CA; ++c) b_addr[c] = (uint32_t)(uintptr_t)(sB + (l + 64 * c) * ROW);
  // chains: RR x CA; packed along the even dimension
  constexpr int NP = RR * CA / 2;
  f2 acc[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) acc[p] = f2{0.0f, 0.0f};
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += CH) {
#pragma unroll
    for (int q = 0; q < LA4; ++q) {
      const int e = tid + NT * q;
      if (e < NRA * C4) *(f4*)(sA + (e / C4) * ROW + (e % C4) * 4) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < LB4; ++q) {
      const int e = tid + NT * q;
      if (e < NRB * C4) *(f4*)(sB + (e / C4) * ROW + (e % C4) * 4) = rb[q];
    }
    __syncthreads();
    if (x0 + CH < n) fetch(x0 + CH);
    constexpr int NG = CH / 4, R = RR + CA, LA = (15 / R) < 4 ? (15 / R) : 4, NB = LA + 1;
    f4 ga[NB][RR], gb[NB][CA];
    auto rd = [&](int g) {
#pragma unroll
      for (int r = 0; r < RR; ++r)
        asm volatile("ds_read_b128 %0, %1" : "=v"(ga[g % NB][r]) : "v"(a_addr[r] + 16u * g));
#pragma unroll
      for (int c = 0; c < CA; ++c)
        asm volatile("ds_read_b128 %0, %1" : "=v"(gb[g % NB][c]) : "v"(b_addr[c] + 16u * g));
    };
#pragma unroll
    for (int g = 0; g < LA; ++g) rd(g);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g + LA < NG) rd(g + LA);
      // groups still in flight once group g has landed
      const int left = NG - 1 - g < LA ? NG - 1 - g : LA;
      switch (left) {
        case 4: asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(4 * R < 15 ? 4 * R : 15) : "memory"); break;
        case 3: asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(3 * R < 15 ? 3 * R : 15) : "memory"); break;
        case 2: asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(2 * R) : "memory"); break;
        case 1: asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(R) : "memory"); break;
        default: asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break;
      }
#pragma unroll
      for (int r = 0; r < RR; ++r) asm volatile("" : "+v"(ga[g % NB][r]));
#pragma unroll
      for (int c = 0; c < CA; ++c) asm volatile("" : "+v"(gb[g % NB][c]));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if constexpr (RR % 2 == 0) {
          // pairs of rows against one alpha
#pragma unroll
          for (int r = 0; r < RR; r += 2)
#pragma unroll
            for (int c = 0; c < CA; ++c) {
              const f2 a = f2{ga[g % NB][r][k], ga[g % NB][r + 1][k]};
              const f2 b = f2{gb[g % NB][c][k], gb[g % NB][c][k]};
              f2& s = acc[(r / 2) * CA + c];
              s = s + a * b;
            }
        } else {
#pragma unroll
          for (int r = 0; r < RR; ++r)
#pragma unroll
            for (int c = 0; c < CA; c += 2) {
              const f2 a = f2{ga[g % NB][r][k], ga[g % NB][r][k]};
              const f2 b = f2{gb[g % NB][c][k], gb[g % NB][c + 1][k]};
              f2& s = acc[r * (CA / 2) + c / 2];
              s = s + a * b;
            }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < RR; ++r)
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int i = i0 + w * RR + r, j = j0 + l + 64 * c;
      float v;
      if constexpr (RR % 2 == 0) v = acc[(r / 2) * CA + c][r & 1];
      else v = acc[r * (CA / 2) + c / 2][c & 1];
      if (i < na && j < nb) out[(long long)i * ldo + j] = v;
    }
}


// ---------------------------------------------------------------- lanes of two chains, one block per CU
// Block = 2*RP rows x A alphas; lane q < RP*A: alpha q % A, rows 2(q / A),
// 2(q / A) + 1 (a packed pair of chains, v_pk_mul_f32 / v_pk_add_f32);
// ceil(RP*A / 64) waves (at most one per SIMD).  Grid 1-D, tiles numbered
// per XCD as k_v0<true> (each XCD: whole alpha tiles x every row tile).
// Per 4 cells a lane reads 3 float4 (its alpha, its two rows); the products
// of the next group are formed between the dependent adds of this one.
// MODE 0: the product; 1: chunk 0 only fetched (no global loads after it);
// 2: no chains (fetch + LDS stores only)
template <int RP, int A, int CH, int MODE = 0>
__global__ __launch_bounds__((RP * A + 63) / 64 * 64) void k_t2(const float* __restrict__ Ag, int na,
                                                                const float* __restrict__ Bg, int nb,
                                                                int ld, int n, float* __restrict__ out,
                                                                int ldo) {
  constexpr int NT = (RP * A + 63) / 64 * 64, ROW = CH + 4, NR = 2 * RP + A, C4 = CH / 4;
  constexpr int L4 = (NR * C4 + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int nrt = (na + 2 * RP - 1) / (2 * RP), ntiles = nrt * ((nb + A - 1) / A);
  const int per = (gridDim.x + 7) / 8, t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= ntiles) return;
  const int i0 = (t % nrt) * 2 * RP, j0 = (t / nrt) * A;
  // LDS rows: 0 .. 2RP-1 the A rows, 2RP .. the alphas
  f4 rg[L4];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int e = tid + NT * k, r = e / C4, c4 = (e % C4) * 4;
      f4 v = f4{0, 0, 0, 0};
      if (e < NR * C4 && x0 + c4 < n) {
        if (r < 2 * RP) {
          if (i0 + r < na) v = *(const f4*)(Ag + (long long)(i0 + r) * ld + x0 + c4);
        } else if (j0 + r - 2 * RP < nb) {
          v = *(const f4*)(Bg + (long long)(j0 + r - 2 * RP) * ld + x0 + c4);
        }
      }
      rg[k] = v;
    }
  };
  const int q = tid < RP * A ? tid : 0, qa = q % A, qr = q / A;
  const uint32_t r0_addr = (uint32_t)(uintptr_t)(smem + (2 * qr) * ROW);
  const uint32_t r1_addr = (uint32_t)(uintptr_t)(smem + (2 * qr + 1) * ROW);
  const uint32_t b_addr = (uint32_t)(uintptr_t)(smem + (2 * RP + qa) * ROW);
  f2 acc = f2{0.0f, 0.0f};
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += CH) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int e = tid + NT * k;
      if (e < NR * C4) *(f4*)(smem + (e / C4) * ROW + (e % C4) * 4) = rg[k];
    }
    __syncthreads();
    if (x0 + CH < n && MODE != 1) fetch(x0 + CH);
    if (MODE == 2) {
      acc[0] += smem[tid];
      __syncthreads();
      continue;
    }
    constexpr int NG = CH / 4, R = 3, LA = 4, NB = LA + 1;
    f4 g0[NB], g1[NB], gb[NB];
    auto rd = [&](int g) {
      asm volatile("ds_read_b128 %0, %1" : "=v"(g0[g % NB]) : "v"(r0_addr + 16u * g));
      asm volatile("ds_read_b128 %0, %1" : "=v"(g1[g % NB]) : "v"(r1_addr + 16u * g));
      asm volatile("ds_read_b128 %0, %1" : "=v"(gb[g % NB]) : "v"(b_addr + 16u * g));
    };
    auto wait_for = [&](int g) {
      // groups issued so far: up to min(h - 1 + LA, NG - 1) for h = g
      const int left = NG - 1 - g < LA - 1 ? NG - 1 - g : LA - 1;
      switch (left) {
        case 3: asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory"); break;
        default: asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break;
      }
      asm volatile("" : "+v"(g0[g % NB]), "+v"(g1[g % NB]), "+v"(gb[g % NB]));
    };
    auto products = [&](int g, f2 p[4]) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        p[k] = f2{g0[g % NB][k], g1[g % NB][k]} * f2{gb[g % NB][k], gb[g % NB][k]};
    };
#pragma unroll
    for (int g = 0; g < LA; ++g) rd(g);
    f2 p[4], pn[4];
    wait_for(0);
    products(0, p);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g + LA < NG) rd(g + LA);
      if (g + 1 < NG) {
        wait_for(g + 1);
        products(g + 1, pn);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = acc + p[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] = pn[k];
    }
    __syncthreads();
  }
  if (tid < RP * A) {
    const int j = j0 + qa;
    if (j < nb) {
      if (i0 + 2 * qr < na) out[(long long)(i0 + 2 * qr) * ldo + j] = acc[0];
      if (i0 + 2 * qr + 1 < na) out[(long long)(i0 + 2 * qr + 1) * ldo + j] = acc[1];
    }
  }
}


// ---------------------------------------------------------------- packed pairs, interleaved rows
// As k_t2, but each row pair is staged interleaved ([x][2]: r0[x], r1[x]),
// so one ds_read_b128 returns two cells of both rows already paired for
// v_pk_mul_f32 (no register shuffles), the alpha broadcast by op_sel; LDS
// reads take immediate offsets (no address arithmetic per group).
// MODE 0: the product; 1: no global loads after chunk 0; 3: also no LDS
// reads after each chunk's first LA groups (the ring's registers reused,
// opaque to the compiler) -- diagnostics, wrong results.  clk (when given):
// block 0 thread 0 writes its s_memtime / s_memrealtime span.
template <int RP, int A, int CH, int MODE = 0>
__global__ __launch_bounds__((RP * A + 63) / 64 * 64) void k_t3(const float* __restrict__ Ag, int na,
                                                                const float* __restrict__ Bg, int nb,
                                                                int ld, int n, float* __restrict__ out,
                                                                int ldo, unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int NT = (RP * A + 63) / 64 * 64, C4 = CH / 4;
  constexpr int PROW = 2 * CH + 4, ROW = CH + 4;  // floats; both = 4 mod 64 banks
  constexpr int NPI = RP * C4, NAI = A * C4;      // staging items: pair f4-columns, alpha f4s
  constexpr int LP = (NPI + NT - 1) / NT, LB = (NAI + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sP = smem;
  float* sB = smem + RP * PROW;
  const int tid = threadIdx.x;
  const int nrt = (na + 2 * RP - 1) / (2 * RP), ntiles = nrt * ((nb + A - 1) / A);
  const int per = (gridDim.x + 7) / 8, t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= ntiles) return;
  const int i0 = (t % nrt) * 2 * RP, j0 = (t / nrt) * A;
  f4 rp0[LP], rp1[LP], rb[LB];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const int e = tid + NT * k, p = e / C4, c4 = (e % C4) * 4, r = i0 + 2 * p;
      const bool ok = e < NPI && x0 + c4 < n;
      rp0[k] = ok && r < na ? *(const f4*)(Ag + (long long)r * ld + x0 + c4) : f4{0, 0, 0, 0};
      rp1[k] = ok && r + 1 < na ? *(const f4*)(Ag + (long long)(r + 1) * ld + x0 + c4) : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int e = tid + NT * k, a = e / C4, c4 = (e % C4) * 4;
      rb[k] = e < NAI && j0 + a < nb && x0 + c4 < n ? *(const f4*)(Bg + (long long)(j0 + a) * ld + x0 + c4)
                                                  : f4{0, 0, 0, 0};
    }
  };
  const int q = tid < RP * A ? tid : 0, qa = q % A, qr = q / A;
  f2 acc = f2{0.0f, 0.0f};
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
    if (x0 + CH < n && MODE == 0) fetch(x0 + CH);
    constexpr int NG = CH / 4, LA = 4, NB = LA + 1;
    // plain LDS loads into a ring, LA groups ahead: the compiler numbers
    // the in-order LDS returns and waits for exactly the group it uses
    const f4* pp = (const f4*)(sP + qr * PROW);
    const f4* pb = (const f4*)(sB + qa * ROW);
    f4 gp0[NB], gp1[NB], gb[NB];
#pragma unroll
    for (int g = 0; g < LA; ++g) {
      gp0[g] = pp[2 * g];
      gp1[g] = pp[2 * g + 1];
      gb[g] = pb[g];
    }
    f2 pr[4];
    {
      const f4 a0 = gp0[0], a1 = gp1[0], b = gb[0];
      pr[0] = f2{a0.x, a0.y} * f2{b.x, b.x};
      pr[1] = f2{a0.z, a0.w} * f2{b.y, b.y};
      pr[2] = f2{a1.x, a1.y} * f2{b.z, b.z};
      pr[3] = f2{a1.z, a1.w} * f2{b.w, b.w};
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (MODE == 3) {
        asm volatile("" : "+v"(gp0[(g + 1) % NB]), "+v"(gp1[(g + 1) % NB]), "+v"(gb[(g + 1) % NB]));
      } else if (g + LA < NG) {
        gp0[(g + LA) % NB] = pp[2 * (g + LA)];
        gp1[(g + LA) % NB] = pp[2 * (g + LA) + 1];
        gb[(g + LA) % NB] = pb[g + LA];
      }
      f2 pn[4];
      if (g + 1 < NG) {
        const f4 a0 = gp0[(g + 1) % NB], a1 = gp1[(g + 1) % NB], b = gb[(g + 1) % NB];
        pn[0] = f2{a0.x, a0.y} * f2{b.x, b.x};
        pn[1] = f2{a0.z, a0.w} * f2{b.y, b.y};
        pn[2] = f2{a1.x, a1.y} * f2{b.z, b.z};
        pn[3] = f2{a1.z, a1.w} * f2{b.w, b.w};
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = acc + pr[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) pr[k] = pn[k];
    }
    __syncthreads();
  }
  if (tid < RP * A) {
    const int j = j0 + qa;
    if (j < nb) {
      if (i0 + 2 * qr < na) out[(long long)(i0 + 2 * qr) * ldo + j] = acc[0];
      if (i0 + 2 * qr + 1 < na) out[(long long)(i0 + 2 * qr + 1) * ldo + j] = acc[1];
    }
  }
  if (clk && blockIdx.x == 0 && tid == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}


// ---------------------------------------------------------------- t4: t3 with the inner loop in asm
// Reads by ds_read_b128 with immediate offsets LA groups ahead and counted
// lgkmcnt waits; products by v_pk_mul_f32 with the alpha broadcast by
// op_sel straight from its float4's register pair; the pair's dependent
// v_pk_add_f32 of group g interleaved with the products of group g + 1.
__device__ __forceinline__ f2 lo2(f4 v) { return __builtin_shufflevector(v, v, 0, 1); }
__device__ __forceinline__ f2 hi2(f4 v) { return __builtin_shufflevector(v, v, 2, 3); }
#ifdef PD_ASM_ARITH
__device__ __forceinline__ f2 pk_mul_blo(f2 a, f2 b) {  // (a.x * b.x, a.y * b.x)
  f2 r;
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 pk_mul_bhi(f2 a, f2 b) {  // (a.x * b.y, a.y * b.y)
  f2 r;
  asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ void pk_acc(f2& acc, f2 p) {
  asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc) : "v"(p));
}
__device__ __forceinline__ float mul_f(float a, float b) {
  float r;
  asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ void add_f(float& acc, float p) {
  asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc) : "v"(p));
}
#else
// plain arithmetic (the compiler's hazard recognizer pads inline-asm VALU
// ops with s_nop; these compile to the same v_pk_mul_f32 / v_pk_add_f32 /
// v_mul_f32 / v_add_f32, in an order the scheduler may change)
__device__ __forceinline__ f2 pk_mul_blo(f2 a, f2 b) { return a * f2{b.x, b.x}; }
__device__ __forceinline__ f2 pk_mul_bhi(f2 a, f2 b) { return a * f2{b.y, b.y}; }
__device__ __forceinline__ void pk_acc(f2& acc, f2 p) { acc = acc + p; }
__device__ __forceinline__ float mul_f(float a, float b) { return a * b; }
__device__ __forceinline__ void add_f(float& acc, float p) { acc = acc + p; }
#endif

template <int NB>
struct T4Ring {
  f4 p0[NB], p1[NB], b[NB];
};

template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void t4_read(T4Ring<NB>& r, uint32_t pa, uint32_t ba) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.p0[G % NB]) : "v"(pa), "n"(32 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.p1[G % NB]) : "v"(pa), "n"(32 * G + 16));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.b[G % NB]) : "v"(ba), "n"(16 * G));
}

template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void t4_products(T4Ring<NB>& r, f2 (&pr)[4]) {
  // groups issued: up to min(G - 1 + LA, NG - 1); wait for group G
  constexpr int left = (NG - 1 - G) < (LA - 1) ? (NG - 1 - G) : (LA - 1);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(3 * left) : "memory");
  asm volatile("" : "+v"(r.p0[G % NB]), "+v"(r.p1[G % NB]), "+v"(r.b[G % NB]));
  const f4 a0 = r.p0[G % NB], a1 = r.p1[G % NB], b = r.b[G % NB];
  pr[0] = pk_mul_blo(lo2(a0), lo2(b));
  pr[1] = pk_mul_bhi(hi2(a0), lo2(b));
  pr[2] = pk_mul_blo(lo2(a1), hi2(b));
  pr[3] = pk_mul_bhi(hi2(a1), hi2(b));
}

template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void t4_group(T4Ring<NB>& r, uint32_t pa, uint32_t ba, f2& acc, f2 (&pr)[4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG) t4_read<G + LA, NG, LA, NB>(r, pa, ba);
    f2 pn[4];
    if constexpr (G + 1 < NG) {
      // wait for group G + 1, then its products between this group's adds
      constexpr int left = (NG - 2 - G) < (LA - 1) ? (NG - 2 - G) : (LA - 1);
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(3 * left) : "memory");
      constexpr int H = (G + 1) % NB;
      asm volatile("" : "+v"(r.p0[H]), "+v"(r.p1[H]), "+v"(r.b[H]));
      pn[0] = pk_mul_blo(lo2(r.p0[H]), lo2(r.b[H]));
      pk_acc(acc, pr[0]);
      pn[1] = pk_mul_bhi(hi2(r.p0[H]), lo2(r.b[H]));
      pk_acc(acc, pr[1]);
      pn[2] = pk_mul_blo(lo2(r.p1[H]), hi2(r.b[H]));
      pk_acc(acc, pr[2]);
      pn[3] = pk_mul_bhi(hi2(r.p1[H]), hi2(r.b[H]));
      pk_acc(acc, pr[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) pk_acc(acc, pr[k]);
    }
    if constexpr (G + 1 < NG) {
#pragma unroll
      for (int k = 0; k < 4; ++k) pr[k] = pn[k];
      t4_group<G + 1, NG, LA, NB>(r, pa, ba, acc, pr);
    }
  }
}

template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void t4_prologue(T4Ring<NB>& r, uint32_t pa, uint32_t ba) {
  if constexpr (G < LA) {
    t4_read<G, NG, LA, NB>(r, pa, ba);
    t4_prologue<G + 1, NG, LA, NB>(r, pa, ba);
  }
}

template <int RP, int A, int CH, int LAV = 4>
__global__ __launch_bounds__((RP * A + 63) / 64 * 64) void k_t4(const float* __restrict__ Ag, int na,
                                                                const float* __restrict__ Bg, int nb,
                                                                int ld, int n, float* __restrict__ out,
                                                                int ldo, unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int NT = (RP * A + 63) / 64 * 64, C4 = CH / 4;
  constexpr int PROW = 2 * CH + 4, ROW = CH + 4;
  constexpr int NPI = RP * C4, NAI = A * C4;
  constexpr int LP = (NPI + NT - 1) / NT, LB = (NAI + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sP = smem;
  float* sB = smem + RP * PROW;
  const int tid = threadIdx.x;
  const int nrt = (na + 2 * RP - 1) / (2 * RP), ntiles = nrt * ((nb + A - 1) / A);
  const int per = (gridDim.x + 7) / 8, t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= ntiles) return;
  const int i0 = (t % nrt) * 2 * RP, j0 = (t / nrt) * A;
  f4 rp0[LP], rp1[LP], rb[LB];
  // buffer resources from the block's first row / alpha: loads past the
  // matrix (rows >= na / nb, cells >= n) are given an offset past the range
  // and read +0.0, with no branch
  constexpr int kOff = 0x7ffffff0;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Ag + (long long)i0 * ld), 0, kOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Bg + (long long)j0 * ld), 0, kOff, 0x00020000);
  auto ldq = [](__amdgpu_buffer_rsrc_t rs, int off) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  };
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < LP; ++k) {
      const int e = tid + NT * k, p = e / C4, c4 = (e % C4) * 4, r = 2 * p;
      const bool ok = e < NPI && x0 + c4 < n;
      rp0[k] = ldq(rsa, ok && i0 + r < na ? (r * ld + x0 + c4) * 4 : kOff);
      rp1[k] = ldq(rsa, ok && i0 + r + 1 < na ? ((r + 1) * ld + x0 + c4) * 4 : kOff);
    }
#pragma unroll
    for (int k = 0; k < LB; ++k) {
      const int e = tid + NT * k, a = e / C4, c4 = (e % C4) * 4;
      rb[k] = ldq(rsb, e < NAI && j0 + a < nb && x0 + c4 < n ? (a * ld + x0 + c4) * 4 : kOff);
    }
  };
  const int q = tid < RP * A ? tid : 0, qa = q % A, qr = q / A;
  const uint32_t pa = (uint32_t)(uintptr_t)(sP + qr * PROW);
  const uint32_t ba = (uint32_t)(uintptr_t)(sB + qa * ROW);
  f2 acc = f2{0.0f, 0.0f};
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
    constexpr int NG = CH / 4, LA = LAV, NB = LA + 1;
    T4Ring<NB> ring;
    f2 pr[4];
    t4_prologue<0, NG, LA, NB>(ring, pa, ba);
    t4_products<0, NG, LA, NB>(ring, pr);
    t4_group<0, NG, LA, NB>(ring, pa, ba, acc, pr);
    __syncthreads();
  }
  if (tid < RP * A) {
    const int j = j0 + qa;
    if (j < nb) {
      if (i0 + 2 * qr < na) out[(long long)(i0 + 2 * qr) * ldo + j] = acc[0];
      if (i0 + 2 * qr + 1 < na) out[(long long)(i0 + 2 * qr + 1) * ldo + j] = acc[1];
    }
  }
  if (clk && blockIdx.x == 0 && tid == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}


template <int NB>
struct T1Ring {
  f4 a[NB], b[NB];
};
template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void t1_read(T1Ring<NB>& r, uint32_t aa, uint32_t ba) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.a[G % NB]) : "v"(aa), "n"(16 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.b[G % NB]) : "v"(ba), "n"(16 * G));
}
template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void t1_prologue(T1Ring<NB>& r, uint32_t aa, uint32_t ba) {
  if constexpr (G < LA) {
    t1_read<G, NG, LA, NB>(r, aa, ba);
    t1_prologue<G + 1, NG, LA, NB>(r, aa, ba);
  }
}
template <int G, int NG, int LA, int NB, int MODE = 0>
__device__ __forceinline__ void t1_group(T1Ring<NB>& r, uint32_t aa, uint32_t ba, float& acc, float (&pr)[4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG && MODE != 3) t1_read<G + LA, NG, LA, NB>(r, aa, ba);
    constexpr int left = MODE == 3 ? 0 : (NG - 1 - G) < LA ? (NG - 1 - G) : LA;
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(2 * left) : "memory");
    constexpr int H = G % NB;
    asm volatile("" : "+v"(r.a[H]), "+v"(r.b[H]));
    const f4 a = r.a[H], b = r.b[H];
    // products of this group between the adds of the previous one
    float pn[4];
    pn[0] = mul_f(a.x, b.x);
    if (G > 0) add_f(acc, pr[0]);
    pn[1] = mul_f(a.y, b.y);
    if (G > 0) add_f(acc, pr[1]);
    pn[2] = mul_f(a.z, b.z);
    if (G > 0) add_f(acc, pr[2]);
    pn[3] = mul_f(a.w, b.w);
    if (G > 0) add_f(acc, pr[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) pr[k] = pn[k];
    if constexpr (G + 1 == NG) {
#pragma unroll
      for (int k = 0; k < 4; ++k) add_f(acc, pr[k]);
    }
    t1_group<G + 1, NG, LA, NB, MODE>(r, aa, ba, acc, pr);
  }
}

// ---------------------------------------------------------------- v1: one chain per lane, tuned
// k_pair_seq's shape (TA A rows x TB alphas per block, thread (la, jb), one
// scalar chain) with t4's machinery: branch-free buffer-load staging, LDS
// reads with immediate offsets LA groups ahead, XCD-grouped tiles.
// MODE 1: no global loads after chunk 0; 3: also the LDS ring refilled only
// once per chunk (diagnostics, wrong results)
template <int TA, int TB, int CH, int MODE = 0, int LAV = 4>
__global__ __launch_bounds__(TA * TB) void k_v1(const float* __restrict__ Ag, int na,
                                               const float* __restrict__ Bg, int nb, int ld, int n,
                                               float* __restrict__ out, int ldo, unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int NT = TA * TB, C4 = CH / 4, ROW = CH + 4;
  constexpr int NI = (TA + TB) * C4, L4 = (NI + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, la = tid % TA, jb = tid / TA;
  const int nrt = (na + TA - 1) / TA, ntiles = nrt * ((nb + TB - 1) / TB);
  const int per = (gridDim.x + 7) / 8, t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= ntiles) return;
  const int i0 = (t % nrt) * TA, j0 = (t / nrt) * TB;
  constexpr int kOff = 0x7ffffff0;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Ag + (long long)i0 * ld), 0, kOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Bg + (long long)j0 * ld), 0, kOff, 0x00020000);
  f4 rg[L4];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int e = tid + NT * k, r = e / C4, c4 = (e % C4) * 4;
      int off = kOff;
      __amdgpu_buffer_rsrc_t rs = rsa;
      if (r < TA) {
        if (i0 + r < na && x0 + c4 < n) off = (r * ld + x0 + c4) * 4;
      } else {
        rs = rsb;
        if (e < NI && j0 + r - TA < nb && x0 + c4 < n) off = ((r - TA) * ld + x0 + c4) * 4;
      }
      rg[k] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
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
    if (x0 + CH < n && MODE == 0) fetch(x0 + CH);
    constexpr int NG = CH / 4, LA = LAV, NB = LA + 1;
    T1Ring<NB> ring;
    t1_prologue<0, NG, LA, NB>(ring, aa, ba);
    float pr[4];
    t1_group<0, NG, LA, NB, MODE>(ring, aa, ba, acc, pr);
    __syncthreads();
  }
  if (i0 + la < na && j0 + jb < nb) out[(long long)(i0 + la) * ldo + j0 + jb] = acc;
  if (clk && blockIdx.x == 0 && tid == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// ---------------------------------------------------------------- bc: the row through DPP broadcasts
// Block = W waves x 64 alphas; wave w owns rows i0 + RR w + r, the same for
// every lane.  Lane l holds A[i][x0 + 16 q + (l & 15)] (one VGPR per 16 cells
// and row, loaded a chunk ahead), and v_mul_f32_dpp row_newbcast:k hands cell
// 16 q + k to every lane of each 16-lane row inside the product: the row
// costs neither an LDS read nor an extra VALU op.  Lane l's alpha j0 + l comes
// from the block's LDS tile, one ds_read_b128 per 4 cells, LA groups ahead.
// (Needs -fno-slp-vectorize: paired into v_pk_mul_f32, the products keep
// the broadcasts as separate v_mov_b32_dpp.)
template <int K>
__device__ __forceinline__ float bcast16(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150 + K, 0xf,
                                                               0xf, true));
}
template <int NB>
struct BcRing {
  f4 b[NB];
};
template <int G, int NB>
__device__ __forceinline__ void bc_read(BcRing<NB>& r, uint32_t ba) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.b[G % NB]) : "v"(ba), "n"(16 * G));
}
template <int G, int LA, int NB>
__device__ __forceinline__ void bc_prologue(BcRing<NB>& r, uint32_t ba) {
  if constexpr (G < LA) {
    bc_read<G, NB>(r, ba);
    bc_prologue<G + 1, LA, NB>(r, ba);
  }
}
// wait for group G (issued so far: up to min(G - 1 + LA, NG - 1)), its products
template <int G, int NG, int LA, int NB, int RR, int NQ>
__device__ __forceinline__ void bc_products(BcRing<NB>& r, const float (&av)[RR][NQ], float (&p)[RR][4]) {
  constexpr int left = (NG - 1 - G) < (LA - 1) ? (NG - 1 - G) : (LA - 1);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(left) : "memory");
  asm volatile("" : "+v"(r.b[G % NB]));
  const f4 b = r.b[G % NB];
  constexpr int q = G / 4, k0 = (G % 4) * 4;
#pragma unroll
  for (int i = 0; i < RR; ++i) {
    p[i][0] = bcast16<k0>(av[i][q]) * b.x;
    p[i][1] = bcast16<k0 + 1>(av[i][q]) * b.y;
    p[i][2] = bcast16<k0 + 2>(av[i][q]) * b.z;
    p[i][3] = bcast16<k0 + 3>(av[i][q]) * b.w;
  }
}
template <int G, int NG, int LA, int NB, int RR, int NQ>
__device__ __forceinline__ void bc_group(BcRing<NB>& r, uint32_t ba, const float (&av)[RR][NQ], float (&acc)[RR],
                                         float (&pr)[RR][4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG) bc_read<G + LA, NB>(r, ba);
    if constexpr (G + 1 < NG) {
      float pn[RR][4];
      bc_products<G + 1, NG, LA, NB, RR, NQ>(r, av, pn);
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < RR; ++i) {
          acc[i] = acc[i] + pr[i][k];
          pr[i][k] = pn[i][k];
        }
      bc_group<G + 1, NG, LA, NB, RR, NQ>(r, ba, av, acc, pr);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < RR; ++i) acc[i] = acc[i] + pr[i][k];
    }
  }
}

template <int RR, int W, int CH, int LAV>
__global__ __launch_bounds__(64 * W) void k_bc(const float* __restrict__ Ag, int na, const float* __restrict__ Bg,
                                              int nb, int ld, int n, float* __restrict__ out, int ldo,
                                              unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int NT = 64 * W, C4 = CH / 4, ROW = CH + 4, NI = 64 * C4, L4 = (NI + NT - 1) / NT;
  constexpr int NQ = CH / 16, RB = W * RR;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int nrt = (na + RB - 1) / RB, ntiles = nrt * ((nb + 63) / 64);
  const int per = (gridDim.x + 7) / 8, t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= ntiles) return;
  const int i0 = (t % nrt) * RB, j0 = (t / nrt) * 64;
  constexpr int kOff = 0x7ffffff0, kNo = kOff / 4;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)Ag, 0, kOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Bg + (long long)j0 * ld), 0, kOff, 0x00020000);
  int ao[RR], bo[L4];
#pragma unroll
  for (int i = 0; i < RR; ++i) {
    const int row = i0 + w * RR + i;
    ao[i] = row < na ? row * ld + (l & 15) : kNo;
  }
#pragma unroll
  for (int k = 0; k < L4; ++k) {
    const int e = tid + NT * k, row = e / C4;
    bo[k] = e < NI && j0 + row < nb ? row * ld + (e % C4) * 4 : kNo;
  }
  f4 rg[L4];
  float an[RR][NQ], av[RR][NQ];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int c4 = ((tid + NT * k) % C4) * 4;
      rg[k] = __builtin_bit_cast(
          f4, __builtin_amdgcn_raw_buffer_load_b128(rsb, bo[k] != kNo && x0 + c4 < n ? (bo[k] + x0) * 4 : kOff, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < RR; ++i)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int x = x0 + 16 * q + (l & 15);
        an[i][q] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rsa, ao[i] != kNo && x < n ? (ao[i] + x0 + 16 * q) * 4 : kOff,
                                                        0, 0));
      }
  };
  const uint32_t ba = (uint32_t)(uintptr_t)(smem + l * ROW);
  float acc[RR];
#pragma unroll
  for (int i = 0; i < RR; ++i) acc[i] = 0.0f;
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += CH) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int e = tid + NT * k;
      if (e < NI) *(f4*)(smem + (e / C4) * ROW + (e % C4) * 4) = rg[k];
    }
#pragma unroll
    for (int i = 0; i < RR; ++i)
#pragma unroll
      for (int q = 0; q < NQ; ++q) av[i][q] = an[i][q];
    __syncthreads();
    if (x0 + CH < n) fetch(x0 + CH);
    constexpr int NG = CH / 4, LA = LAV, NB = LA + 1;
    BcRing<NB> ring;
    bc_prologue<0, LA, NB>(ring, ba);
    float pr[RR][4];
    bc_products<0, NG, LA, NB, RR, NQ>(ring, av, pr);
    bc_group<0, NG, LA, NB, RR, NQ>(ring, ba, av, acc, pr);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < RR; ++i) {
    const int row = i0 + w * RR + i, j = j0 + l;
    if (row < na && j < nb) out[(long long)row * ldo + j] = acc[i];
  }
  if (clk && blockIdx.x == 0 && tid == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// ---------------------------------------------------------------- bq: v1's 16 x 16 tiles, rows through DPP
// Block = 4 waves = 16 rows x 16 alphas.  Wave w, 16-lane row r: A row
// i0 + 4 w + r; lane k of that row: alpha j0 + k.  A row's cells come as one
// float4 per lane (lane k: cells 64 q + 4 k .. + 3, one buffer_load_dwordx4 per
// 64 cells, a chunk ahead) and reach the products through v_mul_f32_dpp
// row_newbcast:(g % 16): the rows cost no LDS traffic, and the block stages
// only its 16 alphas (one ds_read_b128 per 4 cells, broadcast to 4 lanes).
template <int G, int NG, int LA, int NB, int NQ>
__device__ __forceinline__ void bq_products(BcRing<NB>& r, const f4 (&av)[NQ], float (&p)[4]) {
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
template <int G, int NG, int LA, int NB, int NQ>
__device__ __forceinline__ void bq_group(BcRing<NB>& r, uint32_t ba, const f4 (&av)[NQ], float& acc, float (&pr)[4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG) bc_read<G + LA, NB>(r, ba);
    if constexpr (G + 1 < NG) {
      float pn[4];
      bq_products<G + 1, NG, LA, NB, NQ>(r, av, pn);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc = acc + pr[k];
        pr[k] = pn[k];
      }
      bq_group<G + 1, NG, LA, NB, NQ>(r, ba, av, acc, pr);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = acc + pr[k];
    }
  }
}

template <int CH, int LAV, int MODE = 0>
__global__ __launch_bounds__(256) void k_bq(const float* __restrict__ Ag, int na, const float* __restrict__ Bg,
                                           int nb, int ld, int n, float* __restrict__ out, int ldo,
                                           unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int NT = 256, C4 = CH / 4, ROW = CH + 4, NI = 16 * C4, L4 = NI / NT, NQ = CH / 64;
  static_assert(NI % NT == 0 && CH % 64 == 0, "whole float4 columns per thread, whole 64-cell blocks");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, rr = l >> 4, kk = l & 15;
  const int nrt = (na + 15) / 16, ntiles = nrt * ((nb + 15) / 16);
  const int per = (gridDim.x + 7) / 8, t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= ntiles) return;
  const int i0 = (t % nrt) * 16, j0 = (t / nrt) * 16;
  constexpr int kOff = 0x7ffffff0, kNo = kOff / 4;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)Ag, 0, kOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Bg + (long long)j0 * ld), 0, kOff, 0x00020000);
  const int row = i0 + 4 * w + rr;
  const int ao = row < na ? row * ld + 4 * kk : kNo;
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
    if (x0 + CH < n && MODE == 0) fetch(x0 + CH);
    constexpr int NG = CH / 4, LA = LAV, NB = LA + 1;
    BcRing<NB> ring;
    bc_prologue<0, LA, NB>(ring, ba);
    float pr[4];
    bq_products<0, NG, LA, NB, NQ>(ring, av, pr);
    bq_group<0, NG, LA, NB, NQ>(ring, ba, av, acc, pr);
    __syncthreads();
  }
  if (row < na && j0 + kk < nb) out[(long long)row * ldo + j0 + kk] = acc;
  if (clk && blockIdx.x == 0 && tid == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// ---------------------------------------------------------------- bv: bq without LDS
// bq's tiles and DPP rows, but each lane loads its own alpha's cells straight
// into registers (one buffer_load_dwordx4 per 4 cells, a 64-cell block ahead;
// the block's 4 waves read the same 16 alphas, L1 hits): no staging, no LDS,
// no barriers; the compiler counts the in-order vmcnt returns.
template <int NQB>
__device__ __forceinline__ void bv_block(const f4& a, const f4 (&al)[16], float& acc) {
  static_for<0, 16>([&](auto gc) {
    constexpr int g = decltype(gc)::value;
    const f4 b = al[g];
    const float p0 = bcast16<g>(a.x) * b.x, p1 = bcast16<g>(a.y) * b.y;
    const float p2 = bcast16<g>(a.z) * b.z, p3 = bcast16<g>(a.w) * b.w;
    acc = acc + p0;
    acc = acc + p1;
    acc = acc + p2;
    acc = acc + p3;
  });
}

__global__ __launch_bounds__(256) void k_bv(const float* __restrict__ Ag, int na, const float* __restrict__ Bg,
                                           int nb, int ld, int n, float* __restrict__ out, int ldo,
                                           unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, rr = l >> 4, kk = l & 15;
  const int nrt = (na + 15) / 16, ntiles = nrt * ((nb + 15) / 16);
  const int per = (ntiles + 7) / 8, kb = blockIdx.x / 8;
  if (kb >= per) return;
  const int t = (blockIdx.x % 8) * per + kb;
  if (t >= ntiles) return;
  const int i0 = (t % nrt) * 16, j0 = (t / nrt) * 16;
  constexpr int kOff = 0x7ffffff0, kNo = kOff / 4;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)Ag, 0, kOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)Bg, 0, kOff, 0x00020000);
  const int row = i0 + 4 * w + rr, alpha = j0 + kk;
  const int ao = row < na ? row * ld + 4 * kk : kNo;
  const int bo = alpha < nb ? alpha * ld : kNo;
  auto load = [&](int x0, f4& a, f4 (&al)[16]) {
    const bool ina = (ao != kNo) & (x0 + 4 * kk < n);
    a = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsa, ina ? (ao + x0) * 4 : kOff, 0, 0));
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const bool inb = (bo != kNo) & (x0 + 4 * g < n);
      al[g] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsb, inb ? (bo + x0 + 4 * g) * 4 : kOff,
                                                                           0, 0));
    }
  };
  float acc = 0.0f;
  f4 a0, a1, al0[16], al1[16];
  load(0, a0, al0);
  for (int x0 = 0; x0 < n; x0 += 128) {
    load(x0 + 64, a1, al1);  // (past n: reads +0.0)
    __builtin_amdgcn_sched_barrier(0);  // the next block's loads stay ahead of this block
    bv_block<0>(a0, al0, acc);
    if (x0 + 64 >= n) break;
    load(x0 + 128, a0, al0);
    __builtin_amdgcn_sched_barrier(0);
    bv_block<0>(a1, al1, acc);
  }
  if (row < na && alpha < nb) out[(long long)row * ldo + alpha] = acc;
  if (clk && blockIdx.x == 0 && tid == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// ---------------------------------------------------------------- bq2: two child rows per 16-lane row
// As bq, but each 16-lane row holds two child rows (two float4 sets) against
// its lanes' alphas: per cell two v_mul_f32_dpp and one v_pk_add_f32 for two
// chains, one alpha read per 4 cells for both.  Block = 4 waves = 32 rows x
// 16 alphas: 144 x 500 is 640 waves, every SIMD at most one.
template <int G, int NG, int LA, int NB, int NQ>
__device__ __forceinline__ void bq2_products(BcRing<NB>& r, const f4 (&av)[2][NQ], f2 (&p)[4]) {
  constexpr int left = (NG - 1 - G) < (LA - 1) ? (NG - 1 - G) : (LA - 1);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(left) : "memory");
  asm volatile("" : "+v"(r.b[G % NB]));
  const f4 b = r.b[G % NB];
  constexpr int q = G / 16, s = G % 16;
  p[0] = f2{bcast16<s>(av[0][q].x) * b.x, bcast16<s>(av[1][q].x) * b.x};
  p[1] = f2{bcast16<s>(av[0][q].y) * b.y, bcast16<s>(av[1][q].y) * b.y};
  p[2] = f2{bcast16<s>(av[0][q].z) * b.z, bcast16<s>(av[1][q].z) * b.z};
  p[3] = f2{bcast16<s>(av[0][q].w) * b.w, bcast16<s>(av[1][q].w) * b.w};
}
template <int G, int NG, int LA, int NB, int NQ>
__device__ __forceinline__ void bq2_group(BcRing<NB>& r, uint32_t ba, const f4 (&av)[2][NQ], f2& acc, f2 (&pr)[4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG) bc_read<G + LA, NB>(r, ba);
    if constexpr (G + 1 < NG) {
      f2 pn[4];
      bq2_products<G + 1, NG, LA, NB, NQ>(r, av, pn);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc = acc + pr[k];
        pr[k] = pn[k];
      }
      bq2_group<G + 1, NG, LA, NB, NQ>(r, ba, av, acc, pr);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = acc + pr[k];
    }
  }
}

template <int CH, int LAV>
__global__ __launch_bounds__(256) void k_bq2(const float* __restrict__ Ag, int na, const float* __restrict__ Bg,
                                            int nb, int ld, int n, float* __restrict__ out, int ldo,
                                            unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int NT = 256, C4 = CH / 4, ROW = CH + 4, NI = 16 * C4, L4 = NI / NT, NQ = CH / 64;
  static_assert(NI % NT == 0 && CH % 64 == 0, "whole float4 columns per thread, whole 64-cell blocks");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, rr = l >> 4, kk = l & 15;
  const int nrt = (na + 31) / 32, ntiles = nrt * ((nb + 15) / 16);
  const int per = (gridDim.x + 7) / 8, t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= ntiles) return;
  const int i0 = (t % nrt) * 32, j0 = (t / nrt) * 16;
  constexpr int kOff = 0x7ffffff0, kNo = kOff / 4;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)Ag, 0, kOff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Bg + (long long)j0 * ld), 0, kOff, 0x00020000);
  int rows[2], ao[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    rows[h] = i0 + 8 * w + 4 * h + rr;
    ao[h] = rows[h] < na ? rows[h] * ld + 4 * kk : kNo;
  }
  int bo[L4], bc4[L4];
#pragma unroll
  for (int k = 0; k < L4; ++k) {
    const int e = tid + NT * k, br = e / C4;
    bc4[k] = (e % C4) * 4;
    bo[k] = j0 + br < nb ? br * ld + bc4[k] : kNo;
  }
  f4 rg[L4], an[2][NQ], av[2][NQ];
  auto fetch = [&](int x0) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const bool in = (bo[k] != kNo) & (x0 + bc4[k] < n);
      rg[k] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsb, in ? (bo[k] + x0) * 4 : kOff, 0, 0));
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const bool in = (ao[h] != kNo) & (x0 + 64 * q + 4 * kk < n);
        an[h][q] = __builtin_bit_cast(
            f4, __builtin_amdgcn_raw_buffer_load_b128(rsa, in ? (ao[h] + x0 + 64 * q) * 4 : kOff, 0, 0));
      }
  };
  const uint32_t ba = (uint32_t)(uintptr_t)(smem + kk * ROW);
  f2 acc = f2{0.0f, 0.0f};
  fetch(0);
  for (int x0 = 0; x0 < n; x0 += CH) {
#pragma unroll
    for (int k = 0; k < L4; ++k) {
      const int e = tid + NT * k;
      *(f4*)(smem + (e / C4) * ROW + (e % C4) * 4) = rg[k];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < NQ; ++q) av[h][q] = an[h][q];
    __syncthreads();
    if (x0 + CH < n) fetch(x0 + CH);
    constexpr int NG = CH / 4, LA = LAV, NB = LA + 1;
    BcRing<NB> ring;
    bc_prologue<0, LA, NB>(ring, ba);
    f2 pr[4];
    bq2_products<0, NG, LA, NB, NQ>(ring, av, pr);
    bq2_group<0, NG, LA, NB, NQ>(ring, ba, av, acc, pr);
    __syncthreads();
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (rows[h] < na && j0 + kk < nb) out[(long long)rows[h] * ldo + j0 + kk] = acc[h];
  if (clk && blockIdx.x == 0 && tid == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// ---------------------------------------------------------------- mf: products on the matrix cores
// v_mfma_f32_4x4x1_16b_f32 with C = 0 returns 16 blocks of 4 x 4 outer
// products, each the IEEE product fl(a * b) (one rounding of the exact
// product; a -0 product comes back +0, which leaves a chain from +0
// unchanged).  Lane l = 4 b + t supplies A_b[t] and B_b[t] and receives
// D_b[0..3][t]: block b = (row group b >> 2, alpha group b & 3), A_b = rows
// K (b >> 2) + (t % K) (K = 2: rows r0, r1, r0, r1), B_b[t] = alpha 4 (b & 3) + t,
// so lane l's chains are rows K (b >> 2) + v (v < K) against alpha 4 (b & 3) + t,
// D[0..K) added in cell order by v_pk_add_f32.  One wave per block (4K rows x
// 16 alphas), its rows staged by 16-B LDS-DMA into a ring of NS chunks of 256
// cells (no VGPRs, no barriers: the wave reads only what it loaded).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
typedef float f4m __attribute__((ext_vector_type(4)));
template <int NB>
struct MfRing {
  f4 a[NB], b[NB];
};
template <int G, int NB>
__device__ __forceinline__ void mf_read(MfRing<NB>& r, uint32_t aa, uint32_t ba) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.a[G % NB]) : "v"(aa), "n"(16 * G));
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.b[G % NB]) : "v"(ba), "n"(16 * G));
}
template <int G, int LA, int NB>
__device__ __forceinline__ void mf_prologue(MfRing<NB>& r, uint32_t aa, uint32_t ba) {
  if constexpr (G < LA) {
    mf_read<G, NB>(r, aa, ba);
    mf_prologue<G + 1, LA, NB>(r, aa, ba);
  }
}
template <int G, int NG, int LA, int NB>
__device__ __forceinline__ void mf_products(MfRing<NB>& r, f4m (&d)[4]) {
  constexpr int left = (NG - 1 - G) < (LA - 1) ? (NG - 1 - G) : (LA - 1);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(2 * left) : "memory");
  asm volatile("" : "+v"(r.a[G % NB]), "+v"(r.b[G % NB]));
  const f4 a = r.a[G % NB], b = r.b[G % NB];
  const f4m z = {0.0f, 0.0f, 0.0f, 0.0f};
  d[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(a.x, b.x, z, 0, 0, 0);
  d[1] = __builtin_amdgcn_mfma_f32_4x4x1f32(a.y, b.y, z, 0, 0, 0);
  d[2] = __builtin_amdgcn_mfma_f32_4x4x1f32(a.z, b.z, z, 0, 0, 0);
  d[3] = __builtin_amdgcn_mfma_f32_4x4x1f32(a.w, b.w, z, 0, 0, 0);
}
template <int K>
__device__ __forceinline__ void mf_add(f2 (&acc)[K / 2], const f4m (&d)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    acc[0] = acc[0] + f2{d[c][0], d[c][1]};
    if constexpr (K == 4) acc[1] = acc[1] + f2{d[c][2], d[c][3]};
  }
}
template <int G, int NG, int LA, int NB, int K>
__device__ __forceinline__ void mf_group(MfRing<NB>& r, uint32_t aa, uint32_t ba, f2 (&acc)[K / 2], f4m (&pr)[4]) {
  if constexpr (G < NG) {
    if constexpr (G + LA < NG) mf_read<G + LA, NB>(r, aa, ba);
    if constexpr (G + 1 < NG) {
      f4m pn[4];
      mf_products<G + 1, NG, LA, NB>(r, pn);
      mf_add<K>(acc, pr);
#pragma unroll
      for (int c = 0; c < 4; ++c) pr[c] = pn[c];
      mf_group<G + 1, NG, LA, NB, K>(r, aa, ba, acc, pr);
    } else {
      mf_add<K>(acc, pr);
    }
  }
}

static float* g_zero = nullptr;
template <int K, int LAV, int NS>
__global__ __launch_bounds__(64) void k_mf(const float* __restrict__ Ag, int na, const float* __restrict__ Bg,
                                          int nb, int ld, int n, float* __restrict__ out, int ldo,
                                          unsigned long long* clk, const float* __restrict__ zero) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int CH = 256, RW = 4 * K, NR = RW + 16, ROWB = CH * 4 + 16, SLOT = NR * ROWB;
  extern __shared__ __attribute__((aligned(16))) char ring[];
  const int lane = threadIdx.x, b = lane >> 2, t = lane & 3;
  const int nrt = (na + RW - 1) / RW, ntiles = nrt * ((nb + 15) / 16);
  const int per = (gridDim.x + 7) / 8, tile = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (tile >= ntiles) return;
  const int i0 = (tile % nrt) * RW, j0 = (tile / nrt) * 16;
  const int nch = (n + CH - 1) / CH;
  auto issue = [&](int k, int s) {
    const int x = k * CH + 4 * lane;
    char* slot = ring + s * SLOT;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const bool ok = r < RW ? i0 + r < na : j0 + r - RW < nb;
      const float* row = r < RW ? Ag + (long long)(i0 + r) * ld : Bg + (long long)(j0 + r - RW) * ld;
      uintptr_t g = (uintptr_t)(ok && x < n ? row + x : zero + 4 * lane);
      asm("" : "+v"(g));
      __builtin_amdgcn_global_load_lds((glb_void_t*)g, (lds_void_t*)(slot + r * ROWB), 16, 0, 0);
    }
  };
  const uint32_t base = (uint32_t)(uintptr_t)ring;
  const uint32_t aoff = (uint32_t)((K * (b >> 2) + (t % K)) * ROWB), boff = (uint32_t)((RW + 4 * (b & 3) + t) * ROWB);
  f2 acc[K / 2];
#pragma unroll
  for (int v = 0; v < K / 2; ++v) acc[v] = f2{0.0f, 0.0f};
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nch) issue(s, s);
  for (int k = 0; k < nch; ++k) {
    const int s = k % NS;
    if (k + NS - 1 < nch) {
      issue(k + NS - 1, (k + NS - 1) % NS);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NR * (NS - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const uint32_t aa = base + s * SLOT + aoff, ba = base + s * SLOT + boff;
    constexpr int NG = CH / 4, LA = LAV, NB = LA + 1;
    MfRing<NB> rr;
    mf_prologue<0, LA, NB>(rr, aa, ba);
    f4m pr[4];
    mf_products<0, NG, LA, NB>(rr, pr);
    mf_group<0, NG, LA, NB, K>(rr, aa, ba, acc, pr);
  }
  const int j = j0 + 4 * (b & 3) + t;
#pragma unroll
  for (int v = 0; v < K; ++v) {
    const int i = i0 + K * (b >> 2) + v;
    if (i < na && j < nb) out[(long long)i * ldo + j] = acc[v / 2][v & 1];
  }
  if (clk && blockIdx.x == 0 && lane == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// ---------------------------------------------------------------- harness
static uint64_t sm_state = 0x243F6A8885A308D3ull;
static uint64_t splitmix() {
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double u01() { return (splitmix() >> 11) * (1.0 / 9007199254740992.0); }

typedef void (*Launch)(hipStream_t, const float*, int, const float*, int, int, int, float*, int);

template <int RR, int CA, int W, int CH>
static void launch_tile(hipStream_t st, const float* A, int na, const float* B, int nb, int ld, int n,
                        float* out, int ldo) {
  const size_t lds = (size_t)(W * RR + 64 * CA) * (CH + 4) * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tile<RR, CA, W, CH>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  hipLaunchKernelGGL((k_tile<RR, CA, W, CH>), dim3(cdiv(na, W * RR), cdiv(nb, 64 * CA)), dim3(64 * W),
                     lds, st, A, na, B, nb, ld, n, out, ldo);
}

template <bool XCD>
static void launch_v0(hipStream_t st, const float* A, int na, const float* B, int nb, int ld, int n,
                      float* out, int ldo) {
  const size_t lds = (size_t)32 * kRow * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_v0<XCD>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  if (XCD) {
    const int tiles = cdiv(na, 16) * cdiv(nb, 16);
    hipLaunchKernelGGL(k_v0<XCD>, dim3(cdiv(tiles, 8) * 8), dim3(256), lds, st, A, na, B, nb, ld, n, out, ldo);
  } else {
    hipLaunchKernelGGL(k_v0<XCD>, dim3(cdiv(na, 16), cdiv(nb, 16)), dim3(256), lds, st, A, na, B, nb, ld, n,
                       out, ldo);
  }
}

static unsigned long long* g_clk = nullptr;
template <int RP, int A, int CH, int MODE = 0>
static void launch_t3(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n,
                      float* out, int ldo) {
  const size_t lds = (size_t)(RP * (2 * CH + 4) + A * (CH + 4)) * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_t3<RP, A, CH, MODE>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  const int tiles = cdiv(na, 2 * RP) * cdiv(nb, A);
  hipLaunchKernelGGL((k_t3<RP, A, CH, MODE>), dim3(cdiv(tiles, 8) * 8), dim3((RP * A + 63) / 64 * 64), lds,
                     st, Ag, na, Bg, nb, ld, n, out, ldo, g_clk);
}

template <int RP, int A, int CH, int LAV = 4>
static void launch_t4(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n,
                      float* out, int ldo) {
  const size_t lds = (size_t)(RP * (2 * CH + 4) + A * (CH + 4)) * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_t4<RP, A, CH, LAV>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  const int tiles = cdiv(na, 2 * RP) * cdiv(nb, A);
  hipLaunchKernelGGL((k_t4<RP, A, CH, LAV>), dim3(cdiv(tiles, 8) * 8), dim3((RP * A + 63) / 64 * 64), lds, st,
                     Ag, na, Bg, nb, ld, n, out, ldo, g_clk);
}

template <int TA, int TB, int CH, int MODE = 0, int LAV = 4>
static void launch_v1(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n,
                      float* out, int ldo) {
  const size_t lds = (size_t)(TA + TB) * (CH + 4) * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_v1<TA, TB, CH, MODE, LAV>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  const int tiles = cdiv(na, TA) * cdiv(nb, TB);
  hipLaunchKernelGGL((k_v1<TA, TB, CH, MODE, LAV>), dim3(cdiv(tiles, 8) * 8), dim3(TA * TB), lds, st, Ag, na, Bg, nb, ld,
                     n, out, ldo, g_clk);
}

template <int RP, int A, int CH, int MODE = 0>
static void launch_t2(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n,
                      float* out, int ldo) {
  const size_t lds = (size_t)(2 * RP + A) * (CH + 4) * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_t2<RP, A, CH, MODE>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  const int tiles = cdiv(na, 2 * RP) * cdiv(nb, A);
  hipLaunchKernelGGL((k_t2<RP, A, CH, MODE>), dim3(cdiv(tiles, 8) * 8), dim3((RP * A + 63) / 64 * 64), lds, st,
                     Ag, na, Bg, nb, ld, n, out, ldo);
}

template <int RR, int W, int CH, int LAV>
static void launch_bc(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n, float* out,
                      int ldo) {
  const size_t lds = (size_t)64 * (CH + 4) * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_bc<RR, W, CH, LAV>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  const int tiles = cdiv(na, W * RR) * cdiv(nb, 64);
  hipLaunchKernelGGL((k_bc<RR, W, CH, LAV>), dim3(cdiv(tiles, 8) * 8), dim3(64 * W), lds, st, Ag, na, Bg, nb, ld,
                     n, out, ldo, g_clk);
}

template <int CH, int LAV, int MODE = 0>
static void launch_bq(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n, float* out,
                      int ldo) {
  const size_t lds = (size_t)16 * (CH + 4) * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_bq<CH, LAV, MODE>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  const int tiles = cdiv(na, 16) * cdiv(nb, 16);
  hipLaunchKernelGGL((k_bq<CH, LAV, MODE>), dim3(cdiv(tiles, 8) * 8), dim3(256), lds, st, Ag, na, Bg, nb, ld, n, out, ldo,
                     g_clk);
}

static void launch_bv(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n, float* out,
                      int ldo) {
  const int tiles = cdiv(na, 16) * cdiv(nb, 16);
  hipLaunchKernelGGL(k_bv, dim3(cdiv(tiles, 8) * 8), dim3(256), 0, st, Ag, na, Bg, nb, ld, n, out, ldo, g_clk);
}

template <int CH, int LAV>
static void launch_bq2(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n, float* out,
                       int ldo) {
  const size_t lds = (size_t)16 * (CH + 4) * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_bq2<CH, LAV>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  const int tiles = cdiv(na, 32) * cdiv(nb, 16);
  hipLaunchKernelGGL((k_bq2<CH, LAV>), dim3(cdiv(tiles, 8) * 8), dim3(256), lds, st, Ag, na, Bg, nb, ld, n, out,
                     ldo, g_clk);
}

template <int K, int LAV, int NS>
static void launch_mf(hipStream_t st, const float* Ag, int na, const float* Bg, int nb, int ld, int n, float* out,
                      int ldo) {
  const size_t lds = (size_t)NS * (4 * K + 16) * (256 * 4 + 16);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mf<K, LAV, NS>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  const int tiles = cdiv(na, 4 * K) * cdiv(nb, 16);
  hipLaunchKernelGGL((k_mf<K, LAV, NS>), dim3(cdiv(tiles, 8) * 8), dim3(64), lds, st, Ag, na, Bg, nb, ld, n, out,
                     ldo, g_clk, g_zero);
}

struct Variant {
  const char* name;
  Launch fn;
};

int main(int argc, char** argv) {
  const int na = argc > 1 ? atoi(argv[1]) : 144, nb = argc > 2 ? atoi(argv[2]) : 500,
            n = argc > 3 ? atoi(argv[3]) : 65536;
  if (n % kCH) {
    fprintf(stderr, "n must be a multiple of %d\n", kCH);
    return 1;
  }
  const int ld = n;
  std::vector<float> hA((size_t)na * ld), hB((size_t)nb * ld);
  // beliefs: nonnegative, a spread of magnitudes, a share of zeros; alphas:
  // negative values of a few tens
  for (auto& v : hA) {
    const double u = u01();
    v = u < 0.3 ? 0.0f : (float)(std::exp(-30.0 * u01()) * 1e-3);
  }
  for (size_t j = 0; j < (size_t)nb; ++j) {
    const double base = -5.0 - 35.0 * u01();
    for (int x = 0; x < n; ++x) hB[j * ld + x] = (float)(base * (1.0 + 0.1 * (u01() - 0.5)));
  }
  float *dA, *dB, *dO, *dR;
  CK(hipMalloc(&dA, hA.size() * 4));
  CK(hipMalloc(&dB, hB.size() * 4));
  CK(hipMalloc(&dO, (size_t)na * nb * 4));
  CK(hipMalloc(&dR, (size_t)na * nb * 4));
  CK(hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  CK(hipMalloc(&g_clk, 16));
  CK(hipMalloc(&g_zero, 4096));
  CK(hipMemset(g_zero, 0, 4096));
  const Variant vs[] = {
      {"v0 k_pair_seq 16x16, 1 chain/lane", launch_v0<false>},
      {"v1 16x16 LA4", launch_v1<16, 16, 512>},
      {"v1 16x16 LA6", launch_v1<16, 16, 512, 0, 6>},
      {"v1 16x16 LA7", launch_v1<16, 16, 512, 0, 7>},
      {"v1 16x16 LA7 no refetch (diag)", launch_v1<16, 16, 512, 1, 7>},
      {"v1 8x16 LA7", launch_v1<8, 16, 512, 0, 7>},
      {"t4 16 rows x 18 alphas (pk pairs)", launch_t4<8, 18, 512>},
      {"t4 16x18 LA5", launch_t4<8, 18, 512, 5>},
      {"t4 16x32 LA5", launch_t4<8, 32, 512, 5>},
      {"bc 4 rows x 64 alphas CH256 LA8", launch_bc<1, 4, 256, 8>},
      {"bc 8x64 (W8) CH256 LA8", launch_bc<1, 8, 256, 8>},
      {"bq 16x16 rows by DPP CH512 LA8", launch_bq<512, 8>},
      {"bq CH512 LA8 no refetch (diag)", launch_bq<512, 8, 1>},
      {"bq CH256 LA8", launch_bq<256, 8>},
      {"bq CH128 LA8", launch_bq<128, 8>},
      {"bv bq without LDS (alphas by buffer loads)", launch_bv},
      {"bq2 32x16, 2 rows per 16-lane row CH512 LA8", launch_bq2<512, 8>},
  };
  const int NV = sizeof(vs) / sizeof(vs[0]);
  std::vector<float> ref((size_t)na * nb), got((size_t)na * nb);
  // host check of v0 on a sample of chains
  vs[0].fn(st, dA, na, dB, nb, ld, n, dR, nb);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(ref.data(), dR, ref.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int s = 0; s < 64; ++s) {
    const int i = (int)(splitmix() % na), j = (int)(splitmix() % nb);
    volatile float acc = 0.0f;
    for (int x = 0; x < n; ++x) {
      volatile float p = hA[(size_t)i * ld + x] * hB[(size_t)j * ld + x];
      acc = acc + p;
    }
    uint32_t u0, u1;
    float a = acc, r = ref[(size_t)i * nb + j];
    memcpy(&u0, &a, 4);
    memcpy(&u1, &r, 4);
    if (u0 != u1) ++bad;
  }
  printf("shape %d x %d pairs, %d cells; v0 vs host sequential chain: %d of 64 sampled chains differ\n",
         na, nb, n, bad);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int v = 0; v < NV; ++v) {
    CK(hipMemset(dO, 0xff, (size_t)na * nb * 4));
    vs[v].fn(st, dA, na, dB, nb, ld, n, dO, nb);
    CK(hipStreamSynchronize(st));
    CK(hipGetLastError());
    CK(hipMemcpy(got.data(), dO, got.size() * 4, hipMemcpyDeviceToHost));
    const bool same = memcmp(got.data(), ref.data(), ref.size() * 4) == 0;
    float best = 1e30f, tot = 0.0f;
    const int reps = 5;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, st));
      vs[v].fn(st, dA, na, dB, nb, ld, n, dO, nb);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      tot += ms;
    }
    unsigned long long hc[2] = {0, 0};
    CK(hipMemcpy(hc, g_clk, 16, hipMemcpyDeviceToHost));
    CK(hipMemset(g_clk, 0, 16));
    printf("%-40s min %8.1f us  mean %8.1f us  bit-exact vs v0: %s", vs[v].name, best * 1e3,
           tot / reps * 1e3, same ? "yes" : "NO");
    if (hc[1]) printf("  block 0: %.2f cycles/cell, clock %.2f GHz", (double)hc[0] / n, hc[0] / (hc[1] * 10.0));
    printf("\n");
    fflush(stdout);
  }
  return bad ? 2 : 0;
}
