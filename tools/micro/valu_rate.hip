// Issue rate of fp32 FMA forms on gfx950: v_fma_f32 against v_pk_fma_f32
// (two FMAs per lane), 8 independent accumulators per lane, 4 waves per SIMD
// (1024 blocks x 256 lanes... every CU busy), timed with HIP events: FMAs per
// second chip-wide and cycles per wave-instruction at the measured clock.
// The FIB sweep's inner chains are v_pk_fma_f32.
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/valu_rate tools/micro/valu_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e_ = (x);                                          \
    if (e_ != hipSuccess) {                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                   \
    }                                                             \
  } while (0)

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b) {
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = threadIdx.x * 1e-7f + k;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_fmaf(acc[k], a, b);
  }
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += acc[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk_fma(float* out, float a, float b) {
  f2 acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = f2{threadIdx.x * 1e-7f + k, threadIdx.x * 2e-7f + k};
  const f2 av = f2{a, a}, bv = f2{b, b};
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_elementwise_fma(acc[k], av, bv);
  }
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += acc[k].x + acc[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  const int blocks = 256 * 4;  // 4 waves per SIMD on 256 CUs (with 256-lane blocks)
  float* d;
  CK(hipMalloc(&d, (size_t)blocks * 256 * sizeof(float)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int form = 0; form < 2; ++form) {
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      if (form == 0) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f);
      else hipLaunchKernelGGL(k_pk_fma, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    const double fmas = (double)blocks * 256 * kIters * 8 * (form == 0 ? 1 : 2);
    const double instr_per_simd = (double)blocks * 4 /*waves*/ * kIters * 8 / 1024.0;
    printf("%-14s %8.3f ms  %7.1f TFLOP/s (2 per FMA)  %5.2f ns per wave-instruction per SIMD"
           " (%.1f cycles at 2.4 GHz)\n",
           form == 0 ? "v_fma_f32" : "v_pk_fma_f32", best, 2.0 * fmas / (best * 1e-3) / 1e12,
           best * 1e6 / instr_per_simd, best * 1e6 / instr_per_simd * 2.4);
  }
  return 0;
}
