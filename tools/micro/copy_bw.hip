// Streaming ceilings for the rollout step's traffic (2 B read + 2 B written
// per cell-copy): a grid-stride copy of N bytes with 8-B and 16-B lanes, and
// hipMemcpyDtoD, each timed with HIP events.  Build on the host:
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/copy_bw tools/micro/copy_bw.hip
// run on the GPU box: tools/micro/copy_bw [MiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u2e __attribute__((ext_vector_type(2)));
typedef unsigned int u4e __attribute__((ext_vector_type(4)));

template <typename T>
__global__ __launch_bounds__(256) void k_copy(const T* __restrict__ a, T* __restrict__ b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(a[i], b + i);
}

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                      \
    }                                                                \
  } while (0)

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
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMemcpyDtoD(b, a, bytes));
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) CK(hipMemcpyDtoD(b, a, bytes));
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  printf("%-24s %8.3f ms  %6.2f TB/s (read+write)\n", "hipMemcpyDtoD", ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
  return 0;
}
