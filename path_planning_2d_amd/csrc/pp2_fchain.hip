// pp2_fchain.hip -- the reference-order planner's grid-wide fp32 sums on the
// device, exact and parallel (the scheme of pp2_fchain.h).  Built WITHOUT
// denormal flushing: these sums restate the reference's x86 HOST arithmetic
// (IEEE, no FMA).  The child beliefs they sum are device arithmetic
// (cudaBayesBeliefUpdate under --use_fast_math): their one product per cell
// is flushed here explicitly, as the oracle's ftzf does.
//
//   k_fchain<BASE, K>  one workgroup per group of K chains (K = 0: one chain
//                      of the base terms themselves) over x = 0 .. n-1:
//                      std::accumulate (search_tree_cuda.cu:225-229),
//                      std::inner_product (:168-173, evaluateFibCpu
//                      fast_informed_bound_cuda.cu:278-297) and, for a row,
//                      the running sums (forwardSampling's cdf, :176-183)
//   k_store_children   child = fl(pred_a * L_z) / sum (the QNode constructor's
//                      renormalisation :225-229) into the kept nodes' rows
#include <hip/hip_runtime.h>
#include <float.h>

#define PP2_FC_HD __host__ __device__
#include "pp2_fchain.h"
#include "pp2_pbvi_internal.h"

namespace pp2 {
namespace {

using namespace fchain;

constexpr int kFcThreads = 1024, kFcWaves = kFcThreads / 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  return v;
}

__device__ __forceinline__ float wave_incl_scan(float v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  return v;
}

__device__ __forceinline__ float lane_value(float v, int q) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), q));
}

// The device's flush of a product (FTZ build of the reference kernel).
__device__ __forceinline__ float ftz(float v) {
  return fabsf(v) < FLT_MIN ? copysignf(0.0f, v) : v;
}

// Term sources of one group.
template <int BASE>
struct Base {
  const float* __restrict__ pr;  // FC_ROW: the row; else the prediction row of action a
  const float* __restrict__ lr;  // the likelihood row of observation z
  float s;                       // FC_CHILD_NORM: the child's mass

  __device__ __forceinline__ float operator()(int x) const {
    if (BASE == FC_ROW) return pr[x];
    const float c = ftz(pr[x] * ftz(lr[x]));  // p *= L[16 idx + z] (point_based_value_iteration_cuda.cu:130)
    return BASE == FC_CHILD_NORM ? c / s : c;  // b[x] /= sum (search_tree_cuda.cu:228-229)
  }
};

enum : uint32_t { kPos = 1u, kNeg = 2u, kBad = 4u };
enum : int { kChunkTable = 0, kChunkSeq = 1 };

template <int BASE, int K>
__global__ __launch_bounds__(kFcThreads) void k_fchain(FcArgs a) {
  constexpr int KC = K > 0 ? K : 1;
  constexpr bool kCdfCapable = BASE == FC_ROW && K == 0;
  __shared__ float sP[KC][kFcMaxChunks];     // approximate running sum before each chunk
  __shared__ uint32_t sT[KC][kFcMaxChunks];  // chunk table entries
  __shared__ int sSE[kCdfCapable ? kFcMaxChunks : 1];  // cdf: chunk start state (E + 128 | mode << 16)
  __shared__ int sSK[kCdfCapable ? kFcMaxChunks : 1];  //      and k
  __shared__ float sWt[KC][kFcWaves];
  __shared__ uint32_t sFlags[KC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = a.n, ld = a.ld;
  const int cg = a.g0 + blockIdx.x;  // group (child c = z * 9 + a) index
  Base<BASE> base;
  if (BASE == FC_ROW) {
    base.pr = a.row + (long long)blockIdx.x * a.row_stride;
    base.lr = nullptr;
    base.s = 1.0f;
  } else {
    base.pr = a.pred + (long long)(cg % 9) * ld;
    base.lr = a.lrows + (long long)(cg / 9) * ld;
    base.s = BASE == FC_CHILD_NORM ? a.sums[cg] : 1.0f;
  }
  const float* __restrict__ part = a.partners;
  const bool cdf = kCdfCapable && a.cdf != nullptr;
  const int m = fc_lane_elems(n);
  const int chunk = 64 * m;
  const int nch = (n + chunk - 1) / chunk;
  if (threadIdx.x < KC) sFlags[threadIdx.x] = 0u;
  __syncthreads();

  // ---- pass 1: approximate chunk sums of |t|, and the chains' sign flags
  uint32_t fl[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) fl[i] = 0u;
  for (int j = w; j < nch; j += kFcWaves) {
    float acc[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) acc[i] = 0.0f;
    for (int p = 0; p < m; ++p) {
      const int x = j * chunk + p * 64 + lane;
      if (x < n) {
        const float v = base(x);
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          const float t = K > 0 ? v * part[(long long)i * ld + x] : v;
          acc[i] += fabsf(t);
          fl[i] |= !isfinite(t) ? kBad : t > 0.0f ? kPos : t < 0.0f ? kNeg : 0u;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const float sum = wave_sum(acc[i]);
      if (lane == 0) sP[i][j] = sum;
    }
  }
#pragma unroll
  for (int i = 0; i < KC; ++i) {
    const uint32_t f = (__ballot((fl[i] & kPos) != 0u) ? kPos : 0u) |
                       (__ballot((fl[i] & kNeg) != 0u) ? kNeg : 0u) |
                       (__ballot((fl[i] & kBad) != 0u) ? kBad : 0u);
    if (lane == 0 && f) atomicOr(&sFlags[i], f);
  }
  __syncthreads();

  // ---- exclusive prefix of the chunk sums (thread t <-> chunk t)
  {
    const int t = threadIdx.x;
    float own[KC], incl[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      own[i] = t < nch ? sP[i][t] : 0.0f;
      incl[i] = wave_incl_scan(own[i], lane);
      if (lane == 63) sWt[i][w] = incl[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      float b0 = 0.0f;
      for (int q = 0; q < w; ++q) b0 += sWt[i][q];
      if (t < nch) sP[i][t] = b0 + (incl[i] - own[i]);
    }
  }
  __syncthreads();

  // ---- pass 2: chunk tables in the domain of the approximate running sum
  for (int j = w; j < nch; j += kFcWaves) {
    int E[KC];
    float d[KC];
    bool tie[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      E[i] = domain_of(sP[i][j]);
      d[i] = 0.0f;
      tie[i] = false;
    }
    for (int p = 0; p < m; ++p) {
      const int x = j * chunk + p * 64 + lane;
      if (x < n) {
        const float v = base(x);
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          const float t = K > 0 ? v * part[(long long)i * ld + x] : v;
          bool tx;
          d[i] += units_of(fabsf(t), E[i], &tx);
          tie[i] = tie[i] || tx;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const float ds = wave_sum(d[i]);  // exact below 2^24; else no entry
      const bool anytie = __ballot(tie[i]) != 0ull;
      if (lane == 0) sT[i][j] = make_entry(E[i], ds, anytie);
    }
  }
  __syncthreads();

  // term x of chain i, as the reference forms it
  auto term = [&](int i, int x) -> float {
    if (x >= n) return 0.0f;
    const float v = base(x);
    return K > 0 ? v * part[(long long)i * ld + x] : v;
  };
  // chunk j added term by term to s (|t| when `absd`), in x order
  auto seq_chunk = [&](int i, int j, float s, bool absd) -> float {
    for (int p = 0; p < m; ++p) {
      float t = term(i, j * chunk + p * 64 + lane);
      if (absd) t = fabsf(t);
#pragma unroll
      for (int q = 0; q < 64; ++q) s = s + lane_value(t, q);
    }
    return s;
  };

  // ---- driver: wave i walks chain i
  if (w < KC) {
    const int i = w;
    const uint32_t f = sFlags[i];
    const bool seq_all = (f & kBad) || ((f & kPos) && (f & kNeg));
    const bool neg = (f & kNeg) && !(f & kPos);
    float res;
    if (seq_all) {
      float s = 0.0f;
      for (int j = 0; j < nch; ++j) s = seq_chunk(i, j, s, false);
      res = s;
    } else {
      int E = kEMin, k = 0, j = 0;
      while (j < nch) {
        const int jj = j + lane;
        const uint32_t e = jj < nch ? sT[i][jj] : kNoEntry;
        const bool valid = e != kNoEntry && entry_domain(e) == E;
        const int dl = valid ? entry_units(e) : 0;
        const int incl = wave_incl_scan(dl, lane);
        const bool ok = valid && k + incl <= kK24;
        const uint64_t bad = ~__ballot(ok);
        const int fc = bad == 0ull ? 64 : __builtin_ctzll(bad);
        if (cdf && lane < fc) {
          sSE[jj] = (E + 128) | (kChunkTable << 16);
          sSK[jj] = k + incl - dl;
        }
        if (fc > 0) {
          k += __shfl(incl, fc - 1);
          normalise(&E, &k);
        }
        j += fc;
        if (j < nch && fc < 64) {  // a crossing, a tie or a table of another domain
          if (cdf && lane == 0) {
            sSE[j] = (E + 128) | (kChunkSeq << 16);
            sSK[j] = k;
          }
          const float s = seq_chunk(i, j, value_of(E, k), true);
          state_of(s, &E, &k);
          ++j;
        }
      }
      const float r = value_of(E, k);
      res = neg ? (r == 0.0f ? 0.0f : -r) : r;
    }
    if (lane == 0) a.out[(long long)cg * a.ldo + i] = res;
    if (cdf && seq_all) {  // the running sums term by term (mixed or non-finite belief)
      float s = 0.0f;
      for (int x0 = 0; x0 < n; x0 += 64) {
        const float t = term(0, x0 + lane);
        float mine = 0.0f;
#pragma unroll
        for (int q = 0; q < 64; ++q) {
          s = s + lane_value(t, q);
          if (lane == q) mine = s;
        }
        if (x0 + lane < n) a.cdf[x0 + lane] = mine;
      }
    }
  }

  // ---- cdf: every running sum from its chunk's start state
  if (cdf) {
    __syncthreads();
    const uint32_t f = sFlags[0];
    if ((f & kBad) || ((f & kPos) && (f & kNeg))) return;
    const bool neg = (f & kNeg) && !(f & kPos);
    auto out_of = [&](float r) { return neg ? (r == 0.0f ? 0.0f : -r) : r; };
    for (int j = w; j < nch; j += kFcWaves) {
      const int E = (sSE[j] & 0xffff) - 128, mode = sSE[j] >> 16, k = sSK[j];
      if (mode == kChunkSeq) {
        float s = value_of(E, k);
        for (int p = 0; p < m; ++p) {
          const int x = j * chunk + p * 64 + lane;
          const float t = fabsf(term(0, x));
          float mine = 0.0f;
#pragma unroll
          for (int q = 0; q < 64; ++q) {
            s = s + lane_value(t, q);
            if (lane == q) mine = s;
          }
          if (x < n) a.cdf[x] = out_of(mine);
        }
      } else {
        // lane owns m consecutive cells; the chunk's table applied, so no
        // term ties and the state stays in domain E: exact integer prefix
        const int x0 = j * chunk + lane * m;
        int own = 0;
        for (int q = 0; q < m; ++q) {
          bool tx;
          own += (int)units_of(fabsf(term(0, x0 + q)), E, &tx);
        }
        const int excl = wave_incl_scan(own, lane) - own;
        int kx = k + excl;
        for (int q = 0; q < m; ++q) {
          const int x = x0 + q;
          bool tx;
          kx += (int)units_of(fabsf(term(0, x)), E, &tx);
          if (x < n) a.cdf[x] = out_of(value_of(E, kx));
        }
      }
    }
  }
}

// dst_r[x] = fl(pred_a[x] * L_z[x]) / sums[c_r], c_r = z * 9 + a.
__global__ __launch_bounds__(256) void k_store_children(FcStoreList L, const float* __restrict__ pred,
                                                        const float* __restrict__ lrows,
                                                        const float* __restrict__ sums, int n,
                                                        int ld) {
  const int r = blockIdx.y;
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= n) return;
  const int c = L.child[r];
  const float v = ftz(pred[(long long)(c % 9) * ld + x] * ftz(lrows[(long long)(c / 9) * ld + x]));
  L.dst[r][x] = v / sums[c];
}

}  // namespace

hipError_t launch_fchain(hipStream_t st, int base, int K, int groups, const FcArgs& a) {
  if (groups <= 0) return hipSuccess;
  if (a.n < 0 || a.n > kFcMaxCells || (K != 0 && K != 9) || !a.out)
    return hipErrorInvalidValue;
  if (base != FC_ROW && (!a.pred || !a.lrows || a.g0 < 0 || a.g0 + groups > 144))
    return hipErrorInvalidValue;
  if (base == FC_CHILD_NORM && !a.sums) return hipErrorInvalidValue;
  if (K != 0 && !a.partners) return hipErrorInvalidValue;
  if (a.cdf && (base != FC_ROW || K != 0)) return hipErrorInvalidValue;
  const dim3 grid(groups), block(kFcThreads);
  if (base == FC_ROW && K == 0) hipLaunchKernelGGL((k_fchain<FC_ROW, 0>), grid, block, 0, st, a);
  else if (base == FC_ROW) hipLaunchKernelGGL((k_fchain<FC_ROW, 9>), grid, block, 0, st, a);
  else if (base == FC_CHILD && K == 0) hipLaunchKernelGGL((k_fchain<FC_CHILD, 0>), grid, block, 0, st, a);
  else if (base == FC_CHILD_NORM && K == 9)
    hipLaunchKernelGGL((k_fchain<FC_CHILD_NORM, 9>), grid, block, 0, st, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_store_children(hipStream_t st, const FcStoreList& L, const float* pred,
                                 const float* lrows, const float* sums, int n, int ld) {
  if (L.n <= 0 || n <= 0) return hipSuccess;
  if (L.n > 144) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_store_children, dim3((n + 255) / 256, L.n), dim3(256), 0, st, L, pred, lrows,
                     sums, n, ld);
  return hipGetLastError();
}

}  // namespace pp2

// Diagnostic entry point for tests/test_gpu_fchain.py (not part of pp2.h):
// the FC_ROW chains of one host row x[n] on device 0 -- K = 0: out[0] =
// accumulate(x) and, with cdf, every running sum; K = 9: out[i] =
// inner_product(x, partners[i]) (partners: 9 rows of n).  Synchronous.
extern "C" int pp2_debug_fchain_row(int n, const float* x, const float* partners, int K,
                                    float* out, float* cdf) {
  if (n < 0 || !x || !out || (K != 0 && K != 9) || (K == 9 && !partners) || (cdf && K != 0))
    return 1;
  const size_t ld = ((size_t)n + 63) / 64 * 64 + 64;
  float *dx = nullptr, *dp = nullptr, *dout = nullptr, *dcdf = nullptr;
  int st = 0;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && st == 0) st = 2;
    return st == 0;
  };
  if (ok(hipMalloc(&dx, ld * sizeof(float))) && ok(hipMalloc(&dout, 16 * sizeof(float))) &&
      ok(hipMemset(dx, 0, ld * sizeof(float))) &&
      ok(hipMemcpy(dx, x, (size_t)n * sizeof(float), hipMemcpyHostToDevice)) &&
      (K == 0 || (ok(hipMalloc(&dp, 9 * ld * sizeof(float))) &&
                  ok(hipMemset(dp, 0, 9 * ld * sizeof(float))) &&
                  ok(hipMemcpy2D(dp, ld * sizeof(float), partners, (size_t)n * sizeof(float),
                                 (size_t)n * sizeof(float), 9, hipMemcpyHostToDevice)))) &&
      (!cdf || ok(hipMalloc(&dcdf, ld * sizeof(float))))) {
    pp2::FcArgs a;
    a.n = n;
    a.ld = (int)ld;
    a.row = dx;
    a.partners = dp;
    a.out = dout;
    a.ldo = K == 9 ? 9 : 1;
    a.cdf = dcdf;
    if (ok(pp2::launch_fchain(nullptr, pp2::FC_ROW, K, 1, a)) && ok(hipDeviceSynchronize()) &&
        ok(hipMemcpy(out, dout, (K == 9 ? 9 : 1) * sizeof(float), hipMemcpyDeviceToHost)) && cdf)
      ok(hipMemcpy(cdf, dcdf, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
  }
  for (float* p : {dx, dp, dout, dcdf})
    if (p) (void)hipFree(p);
  return st;
}
