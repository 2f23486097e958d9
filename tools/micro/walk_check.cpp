// k_chain_walk2 (PP2_CHAIN_WALK=2) against k_chain_walk (the default) through the
// library's own launchers: random dot / child / cdf chains of several lengths,
// results compared bit for bit (and against a host sequential chain for DOT).
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/walk_check tools/micro/walk_check.cpp \
//     -Lpath_planning_2d_amd -lpp2_hip -Wl,-rpath,'$ORIGIN/../../path_planning_2d_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

namespace pp2 {
hipError_t launch_pair_seq_small(hipStream_t st, int op, const float* A, int na, const float* B, int nb, int ld,
                                 int n, float* out, int ldo, const int* alist, const int* acount);
hipError_t launch_row_cdf_seq(hipStream_t st, const float* row, int n, float* cdf, float* sum);
}

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
  } while (0)

int main() {
  const int ns[] = {100, 511, 512, 513, 1000, 4000, 8192};
  int bad = 0;
  for (int n : ns) {
    const int na = 5, nb = 3, ld = (n + 63) / 64 * 64;
    std::vector<float> hA((size_t)na * ld, 0.0f), hB((size_t)nb * ld, 0.0f);
    srand(n);
    for (int i = 0; i < na; ++i)
      for (int x = 0; x < n; ++x) hA[(size_t)i * ld + x] = (rand() % 1000) * 1e-4f;
    for (int j = 0; j < nb; ++j)
      for (int x = 0; x < n; ++x) hB[(size_t)j * ld + x] = -(rand() % 1000) * 3e-3f;
    float *dA, *dB, *dO, *dC, *dS;
    CK(hipMalloc(&dA, hA.size() * 4));
    CK(hipMalloc(&dB, hB.size() * 4));
    CK(hipMalloc(&dO, na * nb * 4));
    CK(hipMalloc(&dC, ld * 4));
    CK(hipMalloc(&dS, 4));
    CK(hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> r[2][3];
    for (int m = 0; m < 2; ++m) {
      setenv("PP2_CHAIN_WALK", m ? "1" : "2", 1);
      for (int op = 0; op < 2; ++op) {  // PAIR_DOT = ?, PAIR_CHILD = ?  (values from the header: 1 dot, 2 child)
        CK(hipMemset(dO, 0xff, na * nb * 4));
        CK(pp2::launch_pair_seq_small(0, op == 0 ? 1 : 2, dA, na, dB, nb, ld, n, dO, nb, nullptr, nullptr));
        CK(hipDeviceSynchronize());
        r[m][op].resize(na * nb);
        CK(hipMemcpy(r[m][op].data(), dO, na * nb * 4, hipMemcpyDeviceToHost));
      }
      CK(hipMemset(dC, 0xff, ld * 4));
      CK(pp2::launch_row_cdf_seq(0, dA, n, dC, dS));
      CK(hipDeviceSynchronize());
      r[m][2].resize(n + 1);
      CK(hipMemcpy(r[m][2].data(), dC, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r[m][2].data() + n, dS, 4, hipMemcpyDeviceToHost));
    }
    // host DOT chains
    int hd = 0;
    for (int i = 0; i < na; ++i)
      for (int j = 0; j < nb; ++j) {
        volatile float acc = 0.0f;
        for (int x = 0; x < n; ++x) {
          volatile float p = hA[(size_t)i * ld + x] * hB[(size_t)j * ld + x];
          acc = acc + p;
        }
        float g = r[0][0][i * nb + j], a = acc;
        if (memcmp(&g, &a, 4)) ++hd;
      }
    // host cdf of row 0
    int hc = 0;
    {
      volatile float acc = 0.0f;
      for (int x = 0; x < n; ++x) {
        acc = acc + hA[x];
        float g = r[0][2][x], a = acc;
        if (memcmp(&g, &a, 4)) ++hc;
      }
      float g = r[0][2][n], a = acc;
      if (memcmp(&g, &a, 4)) ++hc;
    }
    printf("n %5d cdf: walk2 vs host running sums: %d of %d differ\n", n, hc, n + 1);
    bad += hc;
    for (int op = 0; op < 3; ++op) {
      const bool same = memcmp(r[0][op].data(), r[1][op].data(), r[0][op].size() * 4) == 0;
      printf("n %5d %s: walk2 vs walk %s", n, op == 0 ? "dot  " : op == 1 ? "child" : "cdf  ", same ? "equal" : "DIFFER");
      if (!same) {
        int first = -1, cnt = 0;
        for (size_t e = 0; e < r[0][op].size(); ++e)
          if (memcmp(&r[0][op][e], &r[1][op][e], 4)) {
            if (first < 0) first = (int)e;
            ++cnt;
          }
        printf(" (%d entries, first %d: %g vs %g)", cnt, first, r[0][op][first], r[1][op][first]);
      }
      printf("\n");
      if (!same) ++bad;
    }
    printf("n %5d dot: walk2 vs host chain: %d of %d differ\n", n, hd, na * nb);
    bad += hd;
    CK(hipFree(dA)); CK(hipFree(dB)); CK(hipFree(dO)); CK(hipFree(dC)); CK(hipFree(dS));
  }
  return bad ? 1 : 0;
}
