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
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/micro/pair_dots tools/micro/pair_dots.hip
//   tools/micro/pair_dots [na nb n]     (default 144 500 65536: 256^2, S = 500)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <cmath>
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

// ---------------------------------------------------------------- v0: the library shape
constexpr int kCH = 512, kRow = kCH + 4;

__global__ __launch_bounds__(256) void k_v0(const float* __restrict__ A, int na,
                                            const float* __restrict__ B, int nb, int ld, int n,
                                            float* __restrict__ out, int ldo) {
  constexpr int TA = 16, TB = 16, NT = 256;
  constexpr int LA4 = TA * 128 / NT, LB4 = TB * 128 / NT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sA = smem;
  float* sB = smem + TA * kRow;
  const int tid = threadIdx.x, la = tid % TA, jb = tid / TA;
  const int i0 = blockIdx.x * TA, j0 = blockIdx.y * TB;
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

static void launch_v0(hipStream_t st, const float* A, int na, const float* B, int nb, int ld, int n,
                      float* out, int ldo) {
  const size_t lds = (size_t)32 * kRow * sizeof(float);
  static bool once = false;
  if (!once) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_v0),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    once = true;
  }
  hipLaunchKernelGGL(k_v0, dim3(cdiv(na, 16), cdiv(nb, 16)), dim3(256), lds, st, A, na, B, nb, ld, n, out, ldo);
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
  const Variant vs[] = {
      {"v0 k_pair_seq 16x16, 1 chain/lane", launch_v0},
      {"tile RR2 CA1 W4 CH256 (144 blk)", launch_tile<2, 1, 4, 256>},
      {"tile RR2 CA1 W3 CH256 (192 blk)", launch_tile<2, 1, 3, 256>},
      {"tile RR2 CA1 W2 CH256 (288 blk)", launch_tile<2, 1, 2, 256>},
      {"tile RR1 CA2 W4 CH256", launch_tile<1, 2, 4, 256>},
      {"tile RR2 CA2 W4 CH128", launch_tile<2, 2, 4, 128>},
      {"tile RR4 CA1 W4 CH256", launch_tile<4, 1, 4, 256>},
      {"tile RR2 CA1 W4 CH512", launch_tile<2, 1, 4, 512>},
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
    printf("%-40s min %8.1f us  mean %8.1f us  bit-exact vs v0: %s\n", vs[v].name, best * 1e3,
           tot / reps * 1e3, same ? "yes" : "NO");
    fflush(stdout);
  }
  return bad ? 2 : 0;
}
