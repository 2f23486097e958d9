// Streaming ceilings for the rollout step's traffic (2 B read + 2 B written
// per cell-copy): a grid-stride copy of N bytes with 8-B and 16-B lanes, and
// hipMemcpyDtoD, each timed with HIP events.  Then the alpha re-streaming a
// leaf pass fused into the last band step would add: the 9
// fp32 FIB planes of the 512^2 grid (9.4 MB, beyond one XCD's L2) read once
// per 2-copy chunk, 2048 times = 19.3 GB from L2 / MALL.  Build on the host:
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/copy_bw tools/micro/copy_bw.hip
// run on the GPU box: tools/micro/copy_bw [MiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                      \
    }                                                                \
  } while (0)

typedef unsigned int u2e __attribute__((ext_vector_type(2)));
typedef unsigned int u4e __attribute__((ext_vector_type(4)));

template <typename T>
__global__ __launch_bounds__(256) void k_copy(const T* __restrict__ a, T* __restrict__ b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(a[i], b + i);
}

// Unrolled one-shot copy: each thread moves U 16-B words, all U loads issued
// before the stores (U loads in flight per lane), the grid sized to the
// buffer (no grid-stride loop); NT: nontemporal stores, else plain.
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_u(const u4e* __restrict__ a, u4e* __restrict__ b,
                                                size_t n) {
  const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  u4e v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const size_t i = base + (size_t)k * 256;
    v[k] = i < n ? __builtin_nontemporal_load(a + i) : u4e{0, 0, 0, 0};
  }
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const size_t i = base + (size_t)k * 256;
    if (i < n) {
      if (NT) __builtin_nontemporal_store(v[k], b + i);
      else b[i] = v[k];
    }
  }
}

template <int U, bool NT>
static int run_u(const char* name, void* a, void* b, size_t bytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t n = bytes / 16;
  const int blocks = (int)((n + 256 * U - 1) / (256 * U));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((k_copy_u<U, NT>), dim3(blocks), dim3(256), 0, 0, (const u4e*)a, (u4e*)b, n);
  CK(hipEventRecord(e0));
  const int reps = 10;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_copy_u<U, NT>), dim3(blocks), dim3(256), 0, 0, (const u4e*)a, (u4e*)b, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  printf("%-24s blocks %6d  %8.3f ms  %6.2f TB/s (read+write)\n", name, blocks, ms,
         2.0 * bytes / (ms * 1e-3) / 1e12);
  return 0;
}

// read-only stream (the leaf pass's belief traffic): every word xor-folded
// into a per-lane register, stored only if it equals a value zeros never give
template <typename T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ a, size_t n, unsigned* sink) {
  unsigned acc = 0u;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const T v = __builtin_nontemporal_load(a + i);
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc ^= v[k];
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// block (t, r): tile t's 9 x 512 floats of the planes (plane stride ps),
// summed (so the loads are kept); the same tile for every r, so the working
// set is the planes' 9.4 MB and the reads come from L2 / MALL
__global__ __launch_bounds__(256) void k_restream(const float* __restrict__ F, size_t ps,
                                                  float* __restrict__ sink) {
  const size_t x = (size_t)blockIdx.x * 512 + threadIdx.x * 2;
  float acc = 0.0f;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const float2 v = *reinterpret_cast<const float2*>(F + q * ps + x);
    acc += v.x + v.y;
  }
  if (acc == 12345.0f) sink[blockIdx.y] = acc;  // never: keeps the loads
}


template <typename T>
static int run(const char* name, void* a, void* b, size_t bytes, int blocks) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t n = bytes / sizeof(T);
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_copy<T>, dim3(blocks), dim3(256), 0, 0, (const T*)a, (T*)b, n);
  CK(hipEventRecord(e0));
  const int reps = 10;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k_copy<T>, dim3(blocks), dim3(256), 0, 0, (const T*)a, (T*)b, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  printf("%-24s blocks %6d  %8.3f ms  %6.2f TB/s (read+write)\n", name, blocks, ms,
         2.0 * bytes / (ms * 1e-3) / 1e12);
  return 0;
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 2048;
  const size_t bytes = mib << 20;
  void *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  for (int blocks : {2048, 8192, 32768}) {
    if (run<u2e>("copy 8B/lane", a, b, bytes, blocks)) return 1;
    if (run<u4e>("copy 16B/lane", a, b, bytes, blocks)) return 1;
  }
  // one-shot unrolled copies (the guide's float4 copy: 6.29 TB/s)
  if (run_u<1, false>("copy16 U1 plain", a, b, bytes)) return 1;
  if (run_u<4, false>("copy16 U4 plain", a, b, bytes)) return 1;
  if (run_u<8, false>("copy16 U8 plain", a, b, bytes)) return 1;
  if (run_u<1, true>("copy16 U1 nt", a, b, bytes)) return 1;
  if (run_u<4, true>("copy16 U4 nt", a, b, bytes)) return 1;
  if (run_u<8, true>("copy16 U8 nt", a, b, bytes)) return 1;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0;
  for (int blocks : {2048, 8192, 32768}) {
    const size_t n = bytes / 16;
    hipLaunchKernelGGL(k_read<u4e>, dim3(blocks), dim3(256), 0, 0, (const u4e*)a, n, (unsigned*)b);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 10; ++r)
      hipLaunchKernelGGL(k_read<u4e>, dim3(blocks), dim3(256), 0, 0, (const u4e*)a, n, (unsigned*)b);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    printf("%-24s blocks %6d  %8.3f ms  %6.2f TB/s (read only)\n", "read 16B/lane", blocks, ms,
           bytes / (ms * 1e-3) / 1e12);
  }
  CK(hipMemcpyDtoD(b, a, bytes));
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) CK(hipMemcpyDtoD(b, a, bytes));
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  printf("%-24s %8.3f ms  %6.2f TB/s (read+write)\n", "hipMemcpyDtoD", ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
  // the fused leaf pass's alpha re-streaming: 9 planes of 512^2 floats, read
  // once per 2-copy chunk of 4096 copies
  {
    const size_t cells = 512 * 512, ps = cells;
    float *F, *sink;
    CK(hipMalloc(&F, 9 * cells * sizeof(float)));
    CK(hipMalloc(&sink, 4096 * sizeof(float)));
    CK(hipMemset(F, 0, 9 * cells * sizeof(float)));
    const int reps = 2048;
    const dim3 grid((unsigned)(cells / 512), reps);
    hipLaunchKernelGGL(k_restream, grid, dim3(256), 0, 0, (const float*)F, ps, sink);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r)
      hipLaunchKernelGGL(k_restream, grid, dim3(256), 0, 0, (const float*)F, ps, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    const double gb = 9.0 * cells * 4 * reps / 1e9;
    printf("%-24s %8.3f ms  %6.2f TB/s (%.1f GB of 9.4 MB re-read %d times)\n",
           "alpha re-stream", ms, gb / (ms * 1e-3) / 1e3, gb, reps);
  }
  return 0;
}
