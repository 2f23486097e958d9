// Host cost of hipLaunchKernel against the kernel-argument size (a
// ResidentRun carries its trajectory in ~2.3 KB of kernargs): mean host time
// per launch of an empty kernel, and the event span of 1000 back-to-back
// launches, for 64 B .. 3 KB arguments.
// hipcc --offload-arch=gfx950 -O2 kernarg_cost.hip -o kernarg_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

template <int B>
struct Arg {
  unsigned char v[B];
};

template <int B>
__global__ void k_empty(Arg<B> a, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.v[B - 1] == 7) out[0] = 1;
}

template <int B>
void run(hipStream_t s, int* out) {
  Arg<B> a{};
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_empty<B>, dim3(1), dim3(64), 0, s, a, out);
  (void)hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int n = 1000;
  (void)hipEventRecord(e0, s);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty<B>, dim3(1), dim3(64), 0, s, a, out);
  auto t1 = std::chrono::steady_clock::now();
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // one launch from idle: host time of the call
  double lone = 0;
  for (int i = 0; i < 20; ++i) {
    (void)hipStreamSynchronize(s);
    auto a0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_empty<B>, dim3(1), dim3(64), 0, s, a, out);
    auto a1 = std::chrono::steady_clock::now();
    lone += std::chrono::duration<double, std::micro>(a1 - a0).count();
  }
  (void)hipStreamSynchronize(s);
  printf("kernarg %5d B: host %.2f us/launch (back-to-back), %.2f us (from idle), GPU span %.2f us/launch\n",
         B, std::chrono::duration<double, std::micro>(t1 - t0).count() / n, lone / 20,
         ms * 1e3 / n);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

int main() {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  int* out;
  (void)hipMalloc(&out, 4);
  run<64>(s, out);
  run<256>(s, out);
  run<1024>(s, out);
  run<2304>(s, out);
  run<3072>(s, out);
  (void)hipFree(out);
  (void)hipStreamDestroy(s);
  return 0;
}
