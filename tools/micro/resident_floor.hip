// The dispatch floor of a k_loop_resident-shaped launch: 256 workgroups of
// 1024 lanes, 136 KB of dynamic LDS, ~128 VGPRs, doing nothing -- back-to-back
// event-timed launches, against a 256-lane launch of the same grid.  The
// difference between a short resident launch and its steps is compared with
// this floor.
// hipcc --offload-arch=gfx950 -O2 resident_floor.hip -o resident_floor
#include <hip/hip_runtime.h>

#include <cstdio>

template <int T>
__global__ __launch_bounds__(T) void k_floor(float* out, int n) {
  extern __shared__ float lds[];
  float v[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] = (float)(threadIdx.x + i);
  // keep the registers live (the VGPR budget shapes wave launch)
  asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
               "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]),
               "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15]));
  asm volatile("" : "+v"(v[16]), "+v"(v[17]), "+v"(v[18]), "+v"(v[19]), "+v"(v[20]),
               "+v"(v[21]), "+v"(v[22]), "+v"(v[23]), "+v"(v[24]), "+v"(v[25]), "+v"(v[26]),
               "+v"(v[27]), "+v"(v[28]), "+v"(v[29]), "+v"(v[30]), "+v"(v[31]));
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 32; ++i) s += v[i];
  if (n < 0) {  // never: the LDS is allocated but not touched
    lds[threadIdx.x] = s;
    out[threadIdx.x] = lds[threadIdx.x ^ 1];
  }
}

template <int T>
void run(hipStream_t s, float* out, size_t lds, const char* name) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_floor<T>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_floor<T>, dim3(256), dim3(T), lds, s, out, 1);
  (void)hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int n = 200;
  (void)hipEventRecord(e0, s);
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_floor<T>, dim3(256), dim3(T), lds, s, out, 1);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("%s: %.2f us per back-to-back launch\n", name, ms * 1e3 / n);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

int main() {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  float* out;
  (void)hipMalloc(&out, 4096 * sizeof(float));
  run<1024>(s, out, 136 * 1024, "256 x 1024 lanes, 136 KB LDS");
  run<1024>(s, out, 0, "256 x 1024 lanes, no LDS");
  run<256>(s, out, 0, "256 x 256 lanes, no LDS");
  (void)hipFree(out);
  (void)hipStreamDestroy(s);
  return 0;
}
