// Latency of a dependent fp32 add chain on gfx950 with one wave per SIMD
// (1024 blocks of 64 lanes: every SIMD of the 256 CUs holds one wave), the
// shape of the PBVI leaf dots' chains (one x-ordered chain per lane,
// DESIGN.md §3): cycles per chain element, read from s_memtime in block 0, for
//   add       acc = acc + x                 (the chain alone)
//   mul+add   acc = acc + fl(a * x)         (an independent product per element)
//   dpp+add   the product's first operand broadcast by row_newbcast
//   2 chains  two independent chains per lane, mul+add each
//   4 chains  four
//   vmul+vadd the products of 4 elements first, then their 4 adds
//   pk2       two chains as one packed pair: v_pk_mul_f32 + v_pk_add_f32
//   dpp pk2   as pk2, the shared operand broadcast first by v_mov_b32_dpp
//   lds1      mul+add, x from one ds_read_b128 per 4 elements (lane-distinct
//             rows, conflict-free), issued 4 groups ahead, counted waits
//   lds2      mul+add, both operands from LDS: two ds_read_b128 per 4 elements
//   lds1 dpp  as lds1, the other operand broadcast by row_newbcast
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -o tools/micro/valu_chain tools/micro/valu_chain.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <type_traits>

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                               \
    }                                                         \
  } while (0)

constexpr int kIters = 8192;

template <int K>
__device__ __forceinline__ float bcast16(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150 + K, 0xf,
                                                               0xf, true));
}

// operands that the compiler cannot fold: x_k = v * c_k, the c_k from the kernel's arguments
template <int MODE>
__global__ __launch_bounds__(64) void k_chain(float* out, unsigned long long* clk, float c0, float c1, float c2,
                                             float c3) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float v = threadIdx.x * 1e-3f + 1.0f;
  float x[4] = {v * c0, v * c1, v * c2, v * c3};
  float a[4] = {c3, c2, c1, c0};
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  f2v x2[4] = {f2v{x[0], x[1]}, f2v{x[1], x[2]}, f2v{x[2], x[3]}, f2v{x[3], x[0]}};
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(x[k]), "+v"(a[k]), "+v"(x2[k]));
    if constexpr (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[0] = acc[0] + x[k];
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[0] = acc[0] + a[k] * x[k];
    } else if constexpr (MODE == 2) {
      acc[0] = acc[0] + bcast16<0>(a[0]) * x[0];
      acc[0] = acc[0] + bcast16<1>(a[0]) * x[1];
      acc[0] = acc[0] + bcast16<2>(a[0]) * x[2];
      acc[0] = acc[0] + bcast16<3>(a[0]) * x[3];
    } else if constexpr (MODE == 3) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[0] = acc[0] + a[k] * x[k];
        acc[1] = acc[1] + a[3 - k] * x[k];
      }
    } else if constexpr (MODE == 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[0] = acc[0] + a[k] * x[k];
        acc[1] = acc[1] + a[3 - k] * x[k];
        acc[2] = acc[2] + a[k] * x[3 - k];
        acc[3] = acc[3] + a[(k + 1) & 3] * x[k];
      }
    } else if constexpr (MODE == 6 || MODE == 7) {
      f2v acc2 = f2v{acc[0], acc[1]};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float s = MODE == 7 ? (k == 0 ? bcast16<0>(a[0]) : k == 1 ? bcast16<1>(a[0]) : k == 2 ? bcast16<2>(a[0]) : bcast16<3>(a[0])) : a[k];
        acc2 = acc2 + f2v{s, s} * x2[k];
      }
      acc[0] = acc2.x;
      acc[1] = acc2.y;
    } else {
      float p[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] = a[k] * x[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(p[k]));
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[0] = acc[0] + p[k];
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = __builtin_amdgcn_s_memtime() - t0;
}

// LDS-fed chains: lane l reads row l of a 64 x 260-float tile (conflict-free
// ds_read_b128), NR reads per 4 elements, LA = 4 groups ahead
template <int NR, bool DPP>
__global__ __launch_bounds__(64) void k_lds_chain(float* out, unsigned long long* clk, float c0) {
  __shared__ __attribute__((aligned(16))) float tile[64 * 260];
  for (int i = threadIdx.x; i < 64 * 260; i += 64) tile[i] = (float)(i & 255) * c0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const uint32_t base = (uint32_t)(uintptr_t)(tile + threadIdx.x * 260);
  float a = c0 + threadIdx.x;
  float acc = 0.0f;
  for (int i = 0; i < kIters / 64; ++i) {
    // 64 groups of 4 elements over the row's 256 floats, 4 groups ahead
    f4v r[5][2];
    auto rd = [&](auto gc) {
      constexpr int g = decltype(gc)::value;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[g % 5][0]) : "v"(base), "n"(16 * g));
      if constexpr (NR == 2) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[g % 5][1]) : "v"(base), "n"(16 * ((g + 8) % 64)));
    };
    static_for<0, 4>(rd);
    static_for<0, 64>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      if constexpr (g + 4 < 64) rd(std::integral_constant<int, g + 4>{});
      constexpr int left = (63 - g) < 4 ? (63 - g) : 4;
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NR * left) : "memory");
      asm volatile("" : "+v"(r[g % 5][0]), "+v"(r[g % 5][1]));
      const f4v x = r[g % 5][0];
      const f4v y = NR == 2 ? r[g % 5][1] : f4v{a, a, a, a};
      if constexpr (DPP) {
        acc = acc + bcast16<0>(a) * x.x;
        acc = acc + bcast16<1>(a) * x.y;
        acc = acc + bcast16<2>(a) * x.z;
        acc = acc + bcast16<3>(a) * x.w;
      } else {
        acc = acc + y.x * x.x;
        acc = acc + y.y * x.y;
        acc = acc + y.z * x.z;
        acc = acc + y.w * x.w;
      }
    });
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = __builtin_amdgcn_s_memtime() - t0;
}

int main() {
  const int blocks = 1024;
  float* d;
  unsigned long long* clk;
  CK(hipMalloc(&d, (size_t)blocks * 64 * sizeof(float)));
  CK(hipMalloc(&clk, 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"add", "mul+add", "dpp mul+add", "2 chains mul+add", "4 chains mul+add",
                         "4 muls then 4 adds", "pk2 (2 chains packed)", "dpp pk2"};
  const int chains[] = {1, 1, 1, 2, 4, 1, 2, 2};
  for (int m = 0; m < 8; ++m) {
    float best = 1e30f;
    unsigned long long c = 0;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      switch (m) {
        case 0: hipLaunchKernelGGL(k_chain<0>, dim3(blocks), dim3(64), 0, 0, d, clk, 1.0f, 0.5f, 0.25f, 2.0f); break;
        case 1: hipLaunchKernelGGL(k_chain<1>, dim3(blocks), dim3(64), 0, 0, d, clk, 1.0f, 0.5f, 0.25f, 2.0f); break;
        case 2: hipLaunchKernelGGL(k_chain<2>, dim3(blocks), dim3(64), 0, 0, d, clk, 1.0f, 0.5f, 0.25f, 2.0f); break;
        case 3: hipLaunchKernelGGL(k_chain<3>, dim3(blocks), dim3(64), 0, 0, d, clk, 1.0f, 0.5f, 0.25f, 2.0f); break;
        case 4: hipLaunchKernelGGL(k_chain<4>, dim3(blocks), dim3(64), 0, 0, d, clk, 1.0f, 0.5f, 0.25f, 2.0f); break;
        case 6: hipLaunchKernelGGL(k_chain<6>, dim3(blocks), dim3(64), 0, 0, d, clk, 1.0f, 0.5f, 0.25f, 2.0f); break;
        case 7: hipLaunchKernelGGL(k_chain<7>, dim3(blocks), dim3(64), 0, 0, d, clk, 1.0f, 0.5f, 0.25f, 2.0f); break;
        default: hipLaunchKernelGGL(k_chain<5>, dim3(blocks), dim3(64), 0, 0, d, clk, 1.0f, 0.5f, 0.25f, 2.0f); break;
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      CK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost));
    }
    // s_memtime counts at the shader clock on gfx950? report both views
    const double elems = (double)kIters * 4;
    printf("%-22s %8.3f ms  %6.2f ns per element of a chain  (%.1f cycles at 2.4 GHz; s_memtime %.2f per element)\n",
           names[m], best, best * 1e6 / elems, best * 1e6 / elems * 2.4, (double)c / elems);
    (void)chains;
  }
  const char* lnames[] = {"lds1 mul+add", "lds2 mul+add", "lds1 dpp mul+add"};
  for (int m = 0; m < 3; ++m) {
    float best = 1e30f;
    unsigned long long c = 0;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      if (m == 0) hipLaunchKernelGGL((k_lds_chain<1, false>), dim3(blocks), dim3(64), 0, 0, d, clk, 0.5f);
      else if (m == 1) hipLaunchKernelGGL((k_lds_chain<2, false>), dim3(blocks), dim3(64), 0, 0, d, clk, 0.5f);
      else hipLaunchKernelGGL((k_lds_chain<1, true>), dim3(blocks), dim3(64), 0, 0, d, clk, 0.5f);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      CK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost));
    }
    const double elems = (double)(kIters / 64) * 256;
    printf("%-22s %8.3f ms  %6.2f ns per element of a chain  (%.1f cycles at 2.4 GHz; s_memtime %.2f per element)\n",
           lnames[m], best, best * 1e6 / elems, best * 1e6 / elems * 2.4, (double)c / elems);
  }
  return 0;
}
