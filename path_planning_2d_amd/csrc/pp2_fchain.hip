// pp2_fchain.hip -- the reference-order planner's grid-wide fp32 sums on the
// device, exact and parallel (the scheme of pp2_fchain.h).  Built WITHOUT
// denormal flushing: these sums restate the reference's x86 HOST arithmetic
// (IEEE, no FMA).  The child beliefs they sum are device arithmetic
// (cudaBayesBeliefUpdate under --use_fast_math): their one product per cell
// is flushed here explicitly, as the oracle's ftzf does.
//
// A set of chains (G groups x K partners, or K = 0: one chain of the base
// terms per group) runs as three launches:
//   k_fc_sums    per 256-cell chunk and chain: the approximate sum of |t|
//                (any order; it only picks each chunk's binade), sign flags
//   k_fc_tables  per chunk and chain: the approximate running sum before the
//                chunk, its binade E, and the chunk's increment in E
//   k_fc_drive   one wave per chain: the exact state walked over the chunk
//                entries 64 at a time; the chunks whose entry does not apply
//                (binade crossings, ties, a neighbouring E) term by term with
//                add_exact -- a prefix scan up to the first term that does
//                not apply, its fp32 add, again -- from terms prefetched into
//                LDS where the tables predicted the fallback
// and, for a row's running sums (forwardSampling's cdf), k_fc_cdf: every
// chunk from its exact start state, term by term as above.
//
// Reference sums (search_tree_cuda.cu): std::accumulate of a child belief
// (:225-229), std::inner_product for the QNode reward (:168-173),
// evaluateFibCpu (fast_informed_bound_cuda.cu:278-297), and the sampling cdf
// (:176-183); k_tree_sample restates forwardSampling's draws (:311-366).
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <utility>

#define PP2_FC_HD __host__ __device__
#include "pp2_fchain.h"
#include "pp2_pbvi_internal.h"

namespace pp2 {
namespace {

using namespace fchain;

typedef float f4a __attribute__((ext_vector_type(4)));

constexpr int kFcChunk = 256;     // cells per chunk: 4 per lane
constexpr int kFcWin = 1024;      // chunk entries per driver window (LDS)
constexpr int kFcStash = 8;       // predicted fallback chunks prefetched per window

// Wave scans and sums on DPP row shifts (no LDS crossbar round trips): the
// inclusive scan of each 16-lane row, then the rows' totals by readlane.
__device__ __forceinline__ int row_shr(int v, int ctrl) {
  switch (ctrl) {
    case 1: return __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    case 2: return __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    case 4: return __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    default: return __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  }
}
__device__ __forceinline__ int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float rdl(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// (the rows' totals carried by DPP row_bcast:15 -- lane 15 of each row into
// the next, rows 1 and 3 -- then row_bcast:31 into rows 2 and 3: no scalar
// round trips)
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
  (void)lane;
  v += row_shr(v, 1);
  v += row_shr(v, 2);
  v += row_shr(v, 4);
  v += row_shr(v, 8);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}

// Segment records of the walker (k_fc_walk): a chunk's increments summed from
// its segment's head, saturated at 2^25, and its domain keys (hi 16 bits: the
// largest entry domain; lo 16 bits: 255 - the smallest domain of an entry
// adding something), both as running values from the head -- segmented wave
// scans on DPP (row shifts, then row_bcast:15 / :31).
constexpr uint32_t kSegSat = 1u << 25;

__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
  return max(a & 0xffff0000u, b & 0xffff0000u) | max(a & 0xffffu, b & 0xffffu);
}
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dppu(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ void seg_step(uint32_t& f, uint32_t& s, uint32_t& k) {
  const uint32_t pf = dppu<CTRL, RM>(f), ps = dppu<CTRL, RM>(s), pk = dppu<CTRL, RM>(k);
  const bool head = f != 0u;
  s = head ? s : min(ps + s, kSegSat);
  k = head ? k : pk_max(pk, k);
  f |= pf;
}
// inclusive segmented scan over the lanes (f: a head in or before the lane)
__device__ __forceinline__ void wave_seg_scan(uint32_t& f, uint32_t& s, uint32_t& k) {
  seg_step<0x111, 0xf>(f, s, k);
  seg_step<0x112, 0xf>(f, s, k);
  seg_step<0x114, 0xf>(f, s, k);
  seg_step<0x118, 0xf>(f, s, k);
  seg_step<0x142, 0xa>(f, s, k);
  seg_step<0x143, 0xc>(f, s, k);
}

// the wave's total (uniform): any association will do for these sums
// (approximate running sums, or integer-valued floats below 2^24)
__device__ __forceinline__ float wave_sum(float v) {
  int b = __builtin_bit_cast(int, v);
#pragma unroll
  for (int c = 1; c < 16; c <<= 1) {
    const int o = row_shr(b, c);
    b = __builtin_bit_cast(int, __builtin_bit_cast(float, b) + __builtin_bit_cast(float, o));
  }
  const float f = __builtin_bit_cast(float, b);
  return (rdl(f, 15) + rdl(f, 31)) + (rdl(f, 47) + rdl(f, 63));
}

// the wave's maximum of non-negative float bits (uniform)
__device__ __forceinline__ uint32_t wave_max_bits(uint32_t v) {
#pragma unroll
  for (int c = 1; c < 16; c <<= 1) v = max(v, (uint32_t)row_shr((int)v, c));
  return max(max((uint32_t)rdl((int)v, 15), (uint32_t)rdl((int)v, 31)),
             max((uint32_t)rdl((int)v, 47), (uint32_t)rdl((int)v, 63)));
}

// The lowest domain where every |t| <= the float of bits mx is below half an
// ulp (mx < 2^(E-24)): a chunk adding nothing there adds nothing above either.
__device__ __forceinline__ int zero_domain(uint32_t mx) {
  if (mx == 0u) return kEMin;
  const int et = (int)(mx >> 23);
  const int e = et == 0 ? -127 : et - 127;  // (subnormal: below 2^-126)
  return max(e + 25, kEMin);
}

// inclusive float scan of a wave (any association: approximate running sums)
__device__ __forceinline__ float wave_incl_scan_f(float v, int lane) {
  int b = __builtin_bit_cast(int, v);
#pragma unroll
  for (int c = 1; c < 16; c <<= 1)
    b = __builtin_bit_cast(int, __builtin_bit_cast(float, b) +
                                    __builtin_bit_cast(float, row_shr(b, c)));
  const float f = __builtin_bit_cast(float, b);
  const float r0 = rdl(f, 15), r1 = rdl(f, 31), r2 = rdl(f, 47);
  const int row = lane >> 4;
  return f + (row >= 1 ? r0 : 0.0f) + (row >= 2 ? r1 : 0.0f) + (row >= 3 ? r2 : 0.0f);
}

// The device's flush of a product (FTZ build of the reference kernel).
__device__ __forceinline__ float ftz(float v) {
  return fabsf(v) < FLT_MIN ? copysignf(0.0f, v) : v;
}

enum : uint32_t { kPos = 1u, kNeg = 2u, kBad = 4u };
enum : uint32_t { kPredicted = 1u };  // tab[].y: the driver will likely fall back here

// group g's id, and whether it is active (false: neither is any later g --
// the kernels walk their groups in grid strides and stop there).  FC_LIST:
// id = g, the index of the chain's (row, partner) entry in plist.
__device__ __forceinline__ bool group_id(const FcArgs& a, int g, int* id) {
  if (g >= a.ngroups) return false;
  if (a.gcount && g >= *a.gcount) return false;
  *id = a.glist ? a.glist[g] : a.g0 + g;
  return true;
}

// The base terms of one group, and the chain terms.
template <int BASE, int K>
struct Terms {
  const float* __restrict__ pr;  // FC_ROW: the row; FC_CHILD: the prediction row of action a
  const float* __restrict__ lr;  // FC_CHILD: the likelihood row of observation z
  const float* __restrict__ part;
  int n, ld;
  float m;  // FC_KEPT: the child's mass (set by the kernel)

  __device__ __forceinline__ void init(const FcArgs& a, int id) {
    n = a.n;
    ld = a.ld;
    part = a.partners;
    m = 1.0f;
    if (BASE == FC_KEPT) {
      pr = a.pred + (long long)(id % 9) * ld;
      lr = a.lrows + (long long)(id / 9) * ld;
    } else if (BASE == FC_ROW) {
      pr = a.row + (long long)id * a.row_stride;
      lr = nullptr;
    } else if (BASE == FC_LIST) {  // row plist[id].x times partner plist[id].y
      const int2 e = a.plist[id];
      pr = a.row + (long long)e.x * a.row_stride;
      lr = a.partners + (long long)e.y * ld;
    } else {
      pr = a.pred + (long long)(id % 9) * ld;
      lr = a.lrows + (long long)(id / 9) * ld;
    }
  }
  // p *= L[16 idx + z] (point_based_value_iteration_cuda.cu:130), flushed;
  // FC_LIST: inner_product's host product b[x] * alpha[x] (IEEE)
  __device__ __forceinline__ float base(int x) const {
    if (BASE == FC_ROW) return pr[x];
    if (BASE == FC_LIST) return pr[x] * lr[x];
    if (BASE == FC_KEPT) return ftz(pr[x] * ftz(lr[x])) / m;  // (search_tree_cuda.cu:228-229)
    return ftz(pr[x] * ftz(lr[x]));
  }
  __device__ __forceinline__ float term(float v, int i, int x) const {
    return K > 0 ? v * part[(long long)i * ld + x] : v;
  }
  // every chain's partner values of the 4 cells x0 .. x0+3 (0 past n), all
  // loads issued before any is used (K = 9: one round trip, not nine)
  __device__ __forceinline__ void partner_quads(int x0, float (&w)[K > 0 ? K : 1][4]) const {
    constexpr int KC = K > 0 ? K : 1;
    if (K == 0) return;
    if (x0 + 4 <= n) {
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        const f4a q = *reinterpret_cast<const f4a*>(part + (long long)i * ld + x0);
#pragma unroll
        for (int c = 0; c < 4; ++c) w[i][c] = q[c];
      }
    } else {
#pragma unroll
      for (int i = 0; i < KC; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) w[i][c] = x0 + c < n ? part[(long long)i * ld + x0 + c] : 0.0f;
    }
  }
  // chain i's terms from the base values and the partner quads
  __device__ __forceinline__ void terms_with(const float (&v)[4], const float (&w)[K > 0 ? K : 1][4],
                                             int i, float (&t)[4]) const {
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = K > 0 ? v[q] * w[i][q] : v[q];
  }
  // chain i's terms of the 4 cells x0 .. x0+3 from their base values v (0
  // past n: v is)
  __device__ __forceinline__ void terms_of(const float (&v)[4], int i, int x0,
                                          float (&t)[4]) const {
    if (K == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = v[q];
    } else if (x0 + 4 <= n) {
      const f4a w = *reinterpret_cast<const f4a*>(part + (long long)i * ld + x0);
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = v[q] * w[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = x0 + q < n ? v[q] * part[(long long)i * ld + x0 + q] : 0.0f;
    }
  }
  // the 4 terms of chain i at x0 .. x0+3 (x0 % 4 == 0; 0 past n); i < 0:
  // the base values
  __device__ __forceinline__ void terms4(int i, int x0, float (&t)[4]) const {
    if (x0 + 4 <= n) {
      const f4a p = *reinterpret_cast<const f4a*>(pr + x0);
      f4a v = p;
      if (BASE == FC_CHILD) {
        const f4a l = *reinterpret_cast<const f4a*>(lr + x0);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ftz(p[q] * ftz(l[q]));
      } else if (BASE == FC_KEPT) {
        const f4a l = *reinterpret_cast<const f4a*>(lr + x0);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ftz(p[q] * ftz(l[q])) / m;
      } else if (BASE == FC_LIST) {
        const f4a l = *reinterpret_cast<const f4a*>(lr + x0);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = p[q] * l[q];
      }
      if (K > 0 && i >= 0) {
        const f4a w = *reinterpret_cast<const f4a*>(part + (long long)i * ld + x0);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = v[q] * w[q];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = v[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        t[q] = x0 + q < n ? (i >= 0 ? term(base(x0 + q), i, x0 + q) : base(x0 + q)) : 0.0f;
    }
  }
};

// FC_KEPT: the child's mass -- exact (mass) or, for the sums, approximate
// (the children set's chunk sums; any value will do there: it only scales
// the chunk sums the binades are predicted from)
__device__ __forceinline__ float kept_mass(const FcArgs& a, int id, int nch, int lane) {
  if (a.kept_unit) return 1.0f;
  if (a.mass) return a.mass[id];
  const float* m = a.msum + (long long)id * nch;
  float acc = 0.0f;
  int c = lane;
  for (; c + 192 < nch; c += 256) {  // (four loads in flight)
    const float m0 = m[c], m1 = m[c + 64], m2 = m[c + 128], m3 = m[c + 192];
    acc += (m0 + m1) + (m2 + m3);
  }
  for (; c < nch; c += 64) acc += m[c];
  return wave_sum(acc);
}

// ---------------------------------------------------------------- pass 1
template <int BASE, int K>
__global__ __launch_bounds__(256) void k_fc_sums(FcArgs a) {
  constexpr int KC = K > 0 ? K : 1;
  __shared__ uint32_t sFlags[KC];
  const int seg = blockIdx.x;
  for (int g = blockIdx.y;; g += gridDim.y) {  // (block-uniform)
  int id;
  if (!group_id(a, g, &id)) return;
  Terms<BASE, K> T;
  T.init(a, id);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = fc_chunks(a.n), nseg = fc_segments(a.n);
  const int gc = a.by_id ? id : g;  // (the scratch chains' index)
  if (BASE == FC_KEPT) T.m = kept_mass(a, id, nch, lane);
  if (threadIdx.x < KC) sFlags[threadIdx.x] = 0u;
  __syncthreads();
  uint32_t fl[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) fl[i] = 0u;
  const int j = seg * kFcSegChunks + w;
  if (j < nch) {
    const int x0 = j * kFcChunk + 4 * lane;
    float v[4], wq[KC][4];
    T.terms4(-1, x0, v);  // the base terms
    T.partner_quads(x0, wq);
    // kept_unit: the terms here are fl(w alpha), the chain's fl(fl(w / m)
    // alpha) (0 < w <= m); the signs come from w and alpha, which an
    // underflow of either product cannot hide
    const bool unit = BASE == FC_KEPT && a.kept_unit;
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      float acc = 0.0f, tt[4];
      T.terms_with(v, wq, i, tt);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float t = tt[q];
        acc += fabsf(t);
        const float sg = unit ? (v[q] != 0.0f ? wq[i][q] : 0.0f) : t;
        fl[i] |= !isfinite(t) ? kBad : sg > 0.0f ? kPos : sg < 0.0f ? kNeg : 0u;
      }
      const float sum = wave_sum(acc);
      if (lane == 0) a.csum[(long long)(gc * KC + i) * nch + j] = sum;
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
  if (threadIdx.x < KC)
    a.cflag[(long long)(gc * KC + threadIdx.x) * nseg + seg] = sFlags[threadIdx.x];
  __syncthreads();  // (sFlags of the next group)
  }
}

// ---------------------------------------------------------------- crossing plans
// A predicted chunk (kPredicted: the approximate running sum crosses a
// binade in it, or no entry) is where a walker leaves its entries for exact
// rounds.  Most such chunks hold one to three binade crossings and nothing
// else; their walk is then known up to the crossing terms' exact adds: the
// tables kernel predicts the crossing terms from the approximate running sum
// (sP + the chunk's fp32 prefix of |t|) and records
//   E0, the domain it assumed at the chunk start,
//   d_0, the increments in E0 of the terms before the first crossing,
//   for each crossing s = 1 .. nc: the term t*_s, its domain after, D_s, and
//   d_s, the increments in D_s of the terms up to the next crossing,
// valid only with no tie among the non-crossing terms and every d_s < 2^24.
// A walker arriving in state (E, k) follows it as the scalar chain
//   E == E0, k + d_0 <= 2^24; then per crossing s = fl(value_of(E, k) + t*_s)
//   (the reference's own add), state_of(s) in domain D_s, k + d_s <= 2^24
// and falls back to exact rounds on any failed check -- so the plan only
// decides the speed.  (A term before a crossing applies iff no tie and the
// sum stays <= 2^24, which the checks guarantee for the whole run.)
// Record: two uint4 per chunk, w0 = valid | nc << 1 | (E0 + 128) << 8 |
// (D_1 - E0) << 16 | (D_2 - E0) << 20 | (D_3 - E0) << 24, w1 = d_0,
// then (t*_s bits, d_s) for s = 1 .. 3.
constexpr int kPlanMax = 3;

__device__ __forceinline__ void chunk_plan(const float (&tt)[4], float sp, int E, int lane,
                                           uint4* out) {
  // the approximate running sum after each term (DPP float scan), its domain
  float c[4], acc = 0.0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    acc += fabsf(tt[q]);
    c[q] = acc;
  }
  int fb = __builtin_bit_cast(int, acc);
#pragma unroll
  for (int sh = 1; sh < 16; sh <<= 1)
    fb = __builtin_bit_cast(int, __builtin_bit_cast(float, fb) +
                                     __builtin_bit_cast(float, row_shr(fb, sh)));
  fb = __builtin_bit_cast(int, __builtin_bit_cast(float, fb) +
                                   __builtin_bit_cast(float, (int)dppu<0x142, 0xa>((uint32_t)fb)));
  fb = __builtin_bit_cast(int, __builtin_bit_cast(float, fb) +
                                   __builtin_bit_cast(float, (int)dppu<0x143, 0xc>((uint32_t)fb)));
  const float ex = __builtin_bit_cast(float, fb) - acc;
  int D[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) D[q] = domain_of(sp + (ex + c[q]));
  int prev = (int)dppu<0x138, 0xf>((uint32_t)D[3]);  // (wave_shr:1: the lane before's last)
  prev = lane == 0 ? E : prev;
  bool cr[4];
  int ncl = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    cr[q] = D[q] > prev;
    prev = D[q];
    ncl += cr[q];
  }
  const int nci = wave_incl_scan(ncl, lane);
  const int nc = rdl(nci, 63);
  uint32_t w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  if (nc >= 1 && nc <= kPlanMax) {
    // the non-crossing terms' increments in their domains, their running
    // sum over the chunk (a crossing term adds none: it is an fp32 add)
    int u[4], pu[4], acu = 0, ci[4], cnt = nci - ncl;
    bool tie = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bool tx = false;
      const float uf = cr[q] ? 0.0f : units_of(fabsf(tt[q]), D[q], &tx);
      tie = tie || tx;
      u[q] = (int)fminf(uf, (float)kK24);  // (no scan overflow: >= 2^24 fails)
      acu += u[q];
      pu[q] = acu;
      cnt += cr[q];
      ci[q] = cnt;
    }
    // (a lane adding 2^24 or more holds a run that cannot apply: no plan; so
    // the scan below stays under 2^30)
    bool valid = __ballot(tie || acu > kK24) == 0ull;
    const int pincl = wave_incl_scan(min(acu, kK24), lane), pex = pincl - min(acu, kK24);
    // P_s: the running increment at crossing s; d_s = P_{s+1} - P_s (P_0 = 0,
    // P_{nc+1} = the chunk's total)
    int Pprev = 0;
    w[0] = 1u | ((uint32_t)nc << 1) | ((uint32_t)(E + 128) << 8);
#pragma unroll
    for (int sg = 1; sg <= kPlanMax; ++sg) {
      if (sg <= nc) {
        uint32_t tv = 0u;
        int dv = 0, pv = 0;
        bool has = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool me = cr[q] && ci[q] == sg;
          tv = me ? bits_of(fabsf(tt[q])) : tv;
          dv = me ? D[q] : dv;
          pv = me ? pex + pu[q] : pv;
          has = has || me;
        }
        const uint64_t m = __ballot(has);
        const int L = m ? __builtin_ctzll(m) : 0;
        const int off = rdl(dv, L) - E, P = rdl(pv, L);
        valid = valid && m != 0ull && off >= 1 && off <= 15 && P - Pprev < kK24;
        w[0] |= (uint32_t)(off & 15) << (12 + 4 * sg);
        w[2 * sg - 1] = (uint32_t)(P - Pprev);
        w[2 * sg] = (uint32_t)rdl((int)tv, L);
        Pprev = P;
      }
    }
    const int tot = rdl(pincl, 63);
    valid = valid && tot - Pprev < kK24;
#pragma unroll
    for (int sg = 1; sg <= kPlanMax; ++sg)  // (d_nc: selects, no dynamic index)
      w[2 * sg + 1] = sg == nc ? (uint32_t)(tot - Pprev) : w[2 * sg + 1];
    if (!valid) w[0] = 0u;
  }
  if (lane == 0) {
    out[0] = make_uint4(w[0], w[1], w[2], w[3]);
    out[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

// ---------------------------------------------------------------- pass 2
// One chunk's table entries (and crossing plans, and FC_KEPT's normalised
// cells) from its base values v and the approximate running sums before it,
// sP[i] of chain i: k_fc_tables' and k_fc_sumtab's common part.
// One chain's entry (and crossing plan, PLANS) of chunk j: its terms tt and
// the approximate running sum sp before the chunk; chain = the scratch chain.
// (Branch-free but for the plan: the K = 9 loop's chains interleave.)
template <bool PLANS = true>
__device__ __forceinline__ void chain_chunk_entry(const FcArgs& a, const float (&tt)[4], float sp,
                                                  int j, long long chain, int lane, int nch) {
  const int E = domain_of(sp);
  float d = 0.0f;
  bool tie = false;
  uint32_t mx = 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bool tx;
    d += units_of(fabsf(tt[q]), E, &tx);
    tie = tie || tx;
    mx = max(mx, bits_of(tt[q]) & 0x7fffffffu);
  }
  const float ds = wave_sum(d);  // exact below 2^24; else no entry
  const bool anytie = __ballot(tie) != 0ull;
  // a chunk adding nothing is tabled for the lowest domain where it adds
  // nothing (entry_applies: every domain above too)
  const int Ez = ds == 0.0f ? zero_domain(wave_max_bits(mx)) : E;
  const uint32_t e = make_entry(min(E, Ez), ds, anytie);
  // predicted fallback: no entry, or the chunk's sum likely crosses
  // into the next binade (from the approximate running sum)
  // (a chunk adding nothing crosses nothing)
  const bool pred = e == kNoEntry ||
                    (ds > 0.0f && ldexpf(sp, 23 - E) + ds >= (float)kK24 * (1.0f - 0x1p-12f));
  if (lane == 0) a.tab[chain * nch + j] = make_uint2(e, pred ? kPredicted : 0u);
  if (PLANS && pred && a.plan) {
    const unsigned long long p0 = a.stats ? __builtin_amdgcn_s_memtime() : 0ull;
    chunk_plan(tt, sp, E, lane, a.plan + 2 * (chain * nch + j));
    if (a.stats && lane == 0) {  // (plans: count, s_memtime cycles)
      atomicAdd(a.stats + 22, 1);
      atomicAdd(a.stats + 23, (int)(__builtin_amdgcn_s_memtime() - p0));
    }
  }
}

// FC_KEPT: the kept child's normalised cells of a chunk (k_store_kept's
// job): its dense row for the drive, and its node row
__device__ __forceinline__ void store_kept_cells(const FcArgs& a, const float (&v)[4], int x0, int id) {
  float* kr = a.kept_rows + (long long)id * a.ld;
  float* nr = a.rowptr ? a.rowptr[id] : nullptr;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (x0 + q < a.n) {
      kr[x0 + q] = v[q];
      if (nr) nr[x0 + q] = v[q];
    }
  }
}

// One chunk's table entries (and crossing plans, and FC_KEPT's normalised
// cells) from its base values v and the approximate running sums before it,
// sP[i] of chain i: k_fc_tables' and k_fc_sumtab's common part.
template <int BASE, int K>
__device__ __forceinline__ void chunk_entries(const FcArgs& a, const Terms<BASE, K>& T,
                                              const float (&v)[4], int x0, int j, int gc, int id,
                                              const float* sP, int sPstride, int lane, int nch,
                                              const float (*wq0)[4] = nullptr) {
  constexpr int KC = K > 0 ? K : 1;
  if (BASE == FC_KEPT && a.kept_rows) store_kept_cells(a, v, x0, id);
  float wq[KC][4];
  if (wq0) {
#pragma unroll
    for (int i = 0; i < KC; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) wq[i][q] = wq0[i][q];
  } else {
    T.partner_quads(x0, wq);
  }
  const uint32_t cm = K > 0 && a.cmask ? a.cmask[id] : 0xffffu;
  if (K > 0 && BASE == FC_KEPT && a.plan) {
    // (the kept children's FIB sets with PP2_FC_PLAN9=1: crossing plans for
    // the candidate chains)
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      if (!((cm >> i) & 1u)) continue;
      float tt[4];
      T.terms_with(v, wq, i, tt);
      chain_chunk_entry<true>(a, tt, sP[i * sPstride], j, (long long)gc * KC + i, lane, nch);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < KC; ++i) {
    if (!((cm >> i) & 1u)) continue;  // (uniform: not a candidate)
    float tt[4];
    T.terms_with(v, wq, i, tt);
    // (K = 9: no crossing plans, launch_set; compiled out so the chains'
    // code interleaves)
    chain_chunk_entry<K == 0>(a, tt, sP[i * sPstride], j, (long long)gc * KC + i, lane, nch);
  }
}

// ---------------------------------------------------------------- K = 9: a wave per chain
// The sums and tables of K = 9 sets with a wave per chain (576-thread
// workgroups: 9 waves over the segment's 4 chunks): a wave's dependent
// sequence is 4 chunks of one chain, not 9 chains of one chunk -- the
// tables of a one-group set are latency, not throughput (12 us for the 9
// rewards), and a chunk's 9 crossing plans spread over 9 waves.
template <int BASE>
__global__ __launch_bounds__(576) void k_fc_sums9(FcArgs a) {
  __shared__ __attribute__((aligned(16))) float sV[kFcSegChunks][kFcChunk];  // base values
  const int seg = blockIdx.x;
  const int lane = threadIdx.x & 63, i = threadIdx.x >> 6;
  for (int g = blockIdx.y;; g += gridDim.y) {  // (block-uniform)
    int id;
    if (!group_id(a, g, &id)) return;
    Terms<BASE, 9> T;
    T.init(a, id);
    const int nch = fc_chunks(a.n), nseg = fc_segments(a.n);
    const int gc = a.by_id ? id : g;
    const long long chain = (long long)gc * 9 + i;
    const int j0 = seg * kFcSegChunks;
    // the segment's base values, once: waves 0 .. 3 a chunk each (FC_KEPT:
    // the normalisation's division done once, not per chain)
    if (i < kFcSegChunks) {
      if (BASE == FC_KEPT) T.m = kept_mass(a, id, nch, lane);
      const int j = j0 + i, x0 = j * kFcChunk + 4 * lane;
      float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (j < nch) T.terms4(-1, x0, v);
      *reinterpret_cast<f4a*>(&sV[i][4 * lane]) = f4a{v[0], v[1], v[2], v[3]};
    }
    __syncthreads();
    uint32_t fl = 0u;
#pragma unroll
    for (int c = 0; c < kFcSegChunks; ++c) {
      const int j = j0 + c;
      if (j >= nch) break;
      const int x0 = j * kFcChunk + 4 * lane;
      const f4a vv = *reinterpret_cast<const f4a*>(&sV[c][4 * lane]);
      const float v[4] = {vv[0], vv[1], vv[2], vv[3]};
      float tt[4], acc = 0.0f;
      T.terms_of(v, i, x0, tt);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc += fabsf(tt[q]);
        fl |= !isfinite(tt[q]) ? kBad : tt[q] > 0.0f ? kPos : tt[q] < 0.0f ? kNeg : 0u;
      }
      const float sum = wave_sum(acc);
      if (lane == 0) a.csum[chain * nch + j] = sum;
    }
    const uint32_t f = (__ballot((fl & kPos) != 0u) ? kPos : 0u) |
                       (__ballot((fl & kNeg) != 0u) ? kNeg : 0u) |
                       (__ballot((fl & kBad) != 0u) ? kBad : 0u);
    if (lane == 0) a.cflag[chain * nseg + seg] = f;
    __syncthreads();  // (sV of the next group)
  }
}

template <int BASE>
__global__ __launch_bounds__(576) void k_fc_tables9(FcArgs a) {
  __shared__ __attribute__((aligned(16))) float sV[kFcSegChunks][kFcChunk];  // base values
  const int seg = blockIdx.x;
  const int lane = threadIdx.x & 63, i = threadIdx.x >> 6;
  for (int g = blockIdx.y;; g += gridDim.y) {  // (block-uniform)
    int id;
    if (!group_id(a, g, &id)) return;
    Terms<BASE, 9> T;
    T.init(a, id);
    const int nch = fc_chunks(a.n);
    const int gc = a.by_id ? id : g;
    const long long chain = (long long)gc * 9 + i;
    const float* cs = a.csum + chain * nch;
    const int j0 = seg * kFcSegChunks;
    // the approximate running sum before the segment; the segment's own
    // chunk sums (lanes 0 .. 3) -- loads first
    float acc = 0.0f;
    for (int t = lane; t < j0; t += 64) acc += cs[t];
    const float own = lane < kFcSegChunks && j0 + lane < nch ? cs[j0 + lane] : 0.0f;
    // the segment's base values, once: waves 0 .. 3 a chunk each (FC_KEPT:
    // the normalised cells, stored to their rows here too)
    if (i < kFcSegChunks) {
      if (BASE == FC_KEPT) T.m = a.mass[id];
      const int j = j0 + i, x0 = j * kFcChunk + 4 * lane;
      float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (j < nch) {
        T.terms4(-1, x0, v);
        if (BASE == FC_KEPT && a.kept_rows) store_kept_cells(a, v, x0, id);
      }
      *reinterpret_cast<f4a*>(&sV[i][4 * lane]) = f4a{v[0], v[1], v[2], v[3]};
    }
    const float sc9 = BASE == FC_KEPT && a.kept_unit ? 1.0f / a.mass[id] : 1.0f;
    float run = wave_sum(acc) * sc9;
    // (not a candidate, launch_fib_cands: the wave only stages base values)
    const bool skip = a.cmask && !((a.cmask[id] >> i) & 1u);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kFcSegChunks; ++c) {
      const int j = j0 + c;
      if (j >= nch || skip) break;
      const int x0 = j * kFcChunk + 4 * lane;
      const f4a vv = *reinterpret_cast<const f4a*>(&sV[c][4 * lane]);
      const float v[4] = {vv[0], vv[1], vv[2], vv[3]};
      float tt[4];
      T.terms_of(v, i, x0, tt);
      chain_chunk_entry(a, tt, run, j, chain, lane, nch);
      run += rdl(own, c) * sc9;
    }
    __syncthreads();  // (sV of the next group)
  }
}

template <int BASE, int K>
__global__ __launch_bounds__(256) void k_fc_tables(FcArgs a) {
  constexpr int KC = K > 0 ? K : 1;
  __shared__ float sPart[KC][4];
  __shared__ float sP[KC][kFcSegChunks];
  const int seg = blockIdx.x;
  // FC_KEPT: every group (kept child) has the same partner rows, so a
  // workgroup looping over several stages its segment's partner quads in
  // LDS once (in registers across the loop they spill)
  __shared__ __attribute__((aligned(16))) float sWq[BASE == FC_KEPT ? KC : 1][kFcSegChunks][kFcChunk];
  if (BASE == FC_KEPT) {
    Terms<BASE, K> T0;
    T0.init(a, 0);
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    float w0[KC][4];
    T0.partner_quads((seg * kFcSegChunks + wv) * kFcChunk + 4 * ln, w0);
#pragma unroll
    for (int i = 0; i < KC; ++i)
      *reinterpret_cast<f4a*>(&sWq[i][wv][4 * ln]) = f4a{w0[i][0], w0[i][1], w0[i][2], w0[i][3]};
  }
  for (int g = blockIdx.y;; g += gridDim.y) {  // (block-uniform)
  int id;
  if (!group_id(a, g, &id)) return;
  Terms<BASE, K> T;
  T.init(a, id);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = fc_chunks(a.n);
  const int j0 = seg * kFcSegChunks;
  const int gc = a.by_id ? id : g;  // (the scratch chains' index)
  if (BASE == FC_KEPT) T.m = a.mass[id];
  // the approximate running sum before this segment, and inside it (every
  // chain's loads issued before the first is used: one round trip)
  {
    const float* cs0 = a.csum + (long long)(gc * KC) * nch;
    float acc[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) acc[i] = (int)threadIdx.x < j0 ? cs0[(long long)i * nch + threadIdx.x] : 0.0f;
    for (int t = threadIdx.x + 256; t < j0; t += 256)
#pragma unroll
      for (int i = 0; i < KC; ++i) acc[i] += cs0[(long long)i * nch + t];
    // the segment's own chunk sums: thread i * 4 + c (i < KC, c < 4)
    const int oi = threadIdx.x >> 2, oc = threadIdx.x & 3;
    const float own = oi < KC && j0 + oc < nch ? cs0[(long long)oi * nch + j0 + oc] : 0.0f;
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const float s2 = wave_sum(acc[i]);
      if (lane == 0) sPart[i][w] = s2;
    }
    if (oi < KC) sP[oi][oc] = own;  // (the chunk sums, turned into running sums below)
  }
  __syncthreads();
  if (threadIdx.x < KC) {
    const int i = threadIdx.x;
    // (kept_unit: the sums were of the unnormalised cells)
    const float sc = BASE == FC_KEPT && a.kept_unit ? 1.0f / T.m : 1.0f;
    float run = ((sPart[i][0] + sPart[i][1]) + (sPart[i][2] + sPart[i][3])) * sc;
#pragma unroll
    for (int c = 0; c < kFcSegChunks; ++c) {
      const float cs = sP[i][c] * sc;
      sP[i][c] = run;
      run += cs;
    }
  }
  __syncthreads();
  if (j0 + w < nch) {
    const int jl = w, j = j0 + jl;
    const int x0 = j * kFcChunk + 4 * lane;
    float v[4];
    T.terms4(-1, x0, v);
    if constexpr (BASE == FC_KEPT) {
      float wq[KC][4];
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        const f4a q = *reinterpret_cast<const f4a*>(&sWq[i][jl][4 * lane]);
#pragma unroll
        for (int c = 0; c < 4; ++c) wq[i][c] = q[c];
      }
      chunk_entries<BASE, K>(a, T, v, x0, j, gc, id, &sP[0][jl], kFcSegChunks, lane, nch, wq);
    } else {
      chunk_entries<BASE, K>(a, T, v, x0, j, gc, id, &sP[0][jl], kFcSegChunks, lane, nch);
    }
  }
  __syncthreads();  // (sPart / sP of the next group)
  }
}

// ---------------------------------------------------------------- sums + tables
// k_fc_sums and k_fc_tables as one launch: each workgroup (segment seg of
// group g, a chunk per wave) forms its chunk sums, publishes their total --
// one 64-bit agent-scope store of (launch tag, float bits) per chain and
// segment -- and takes the approximate running sum before its segment from
// the totals its predecessors publish (lanes poll one each), then tables its
// chunks.  Dependencies point to lower segments of the same group only, and
// workgroups dispatch in increasing order, so the earliest unfinished
// workgroup can always proceed.  Saves the second launch, its dependency
// wait, the terms' second pass and k_fc_tables' O(segments) prefix loads.
template <int BASE, int K>
__global__ __launch_bounds__(256) void k_fc_sumtab(FcArgs a) {
  constexpr int KC = K > 0 ? K : 1;
  __shared__ uint32_t sFlags[KC];
  __shared__ float sCS[KC][kFcSegChunks];
  __shared__ float sPre[KC];
  __shared__ float sP[KC][kFcSegChunks];
  const int seg = blockIdx.x;
  for (int g = blockIdx.y;; g += gridDim.y) {  // (block-uniform)
  int id;
  if (!group_id(a, g, &id)) return;
  Terms<BASE, K> T;
  T.init(a, id);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = fc_chunks(a.n), nseg = fc_segments(a.n);
  const int gc = a.by_id ? id : g;  // (the scratch chains' index)
  if (BASE == FC_KEPT) T.m = kept_mass(a, id, nch, lane);
  if (threadIdx.x < KC) sFlags[threadIdx.x] = 0u;
  __syncthreads();
  // 1. the chunk sums (k_fc_sums)
  const int j = seg * kFcSegChunks + w;
  const int x0 = j * kFcChunk + 4 * lane;
  float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t fl[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) fl[i] = 0u;
  if (j < nch) T.terms4(-1, x0, v);
#pragma unroll
  for (int i = 0; i < KC; ++i) {
    float acc = 0.0f, tt[4];
    T.terms_of(v, i, x0, tt);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float t = tt[q];
      acc += fabsf(t);
      fl[i] |= !isfinite(t) ? kBad : t > 0.0f ? kPos : t < 0.0f ? kNeg : 0u;
    }
    const float sum = wave_sum(acc);  // (0 past the chunks)
    if (lane == 0) {
      sCS[i][w] = sum;
      if (j < nch) a.csum[(long long)(gc * KC + i) * nch + j] = sum;
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
  // 2. publish the segment's totals; the running sum before the segment
  if (threadIdx.x < KC) {
    const int i = threadIdx.x;
    a.cflag[(long long)(gc * KC + i) * nseg + seg] = sFlags[i];
    const float tot = (sCS[i][0] + sCS[i][1]) + (sCS[i][2] + sCS[i][3]);
    __hip_atomic_store(a.agg + (long long)(gc * KC + i) * nseg + seg,
                       ((unsigned long long)a.epoch << 32) | bits_of(tot), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int i = w; i < KC; i += 4) {  // (wave w: chains w, w + 4, ...)
    const unsigned long long* ag = a.agg + (long long)(gc * KC + i) * nseg;
    float pv = 0.0f;
    for (int s2 = lane; s2 < seg; s2 += 64) {
      unsigned long long x;
      for (;;) {
        x = __hip_atomic_load(ag + s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(x >> 32) == a.epoch) break;
        __builtin_amdgcn_s_sleep(1);
      }
      pv += __builtin_bit_cast(float, (uint32_t)x);
    }
    const float pre = wave_sum(pv);
    if (lane == 0) sPre[i] = pre;
  }
  __syncthreads();
  if (threadIdx.x < KC) {
    const int i = threadIdx.x;
    float run = sPre[i];
    for (int c = 0; c < kFcSegChunks; ++c) {
      sP[i][c] = run;
      run += sCS[i][c];
    }
  }
  __syncthreads();
  // 3. the entries (k_fc_tables)
  if (j < nch) chunk_entries<BASE, K>(a, T, v, x0, j, gc, id, &sP[0][w], kFcSegChunks, lane, nch);
  __syncthreads();  // (LDS of the next group)
  }
}

// ---------------------------------------------------------------- exact chunk
// Chunk of a non-negative chain (|t|) from the exact state (E, k): lane l
// holds terms 4l .. 4l+3.  Each round applies the increments of the terms
// from `done` on up to the first that does not apply (a tie, or past
// 2^(E+1)), adds that one in fp32, and goes on after it (add_exact, in
// parallel).  With cv, every running value (cv[q] of term 4l + q).
// (Ties could go by the parity of the state before them, tie_increment, a
// segmented XOR scan a round: measured in the 256^2 plan step, its chains'
// events are binade crossings, and the longer round cost more than the
// ties it saved.)
//
// A round is ~130 instructions of one wave (~850 cycles in the plan step,
// beside the other stream's kernels); the chain itself is 256 dependent adds
// (~8000 cycles there: ~31 a term).  So a chunk of many events (the climb of
// a chain through binades, runs of ties: 6 .. 14 in a belief's first nonzero
// chunks) runs as rounds up to max_rounds and then, with sT (the wave's
// 256-float LDS buffer), as the fp32 chain for the rest -- every lane the
// same adds over broadcast LDS reads, terms before `done` read as +0.0
// (s + 0 = s for s >= +0); cv from the value at each lane's first term,
// recorded on the way, and the lane's own 4 adds again.
__device__ __forceinline__ void chunk_exact(const float (&t)[4], int lane, int* pE, int* pk,
                                            float (*cv)[4], int* rounds = nullptr,
                                            float* sT = nullptr, int max_rounds = 1 << 30) {
  int E = *pE, k = *pk, done = 0;
  for (int rd = 0;; ++rd) {
    if (sT && rd >= max_rounds) {
      // the rest as the chain itself
      *reinterpret_cast<f4a*>(&sT[4 * lane]) = f4a{t[0], t[1], t[2], t[3]};
      float s = value_of(E, k), s0 = s;
#pragma unroll 1
      for (int xb = done & ~63; xb < kFcChunk; xb += 64) {
#pragma unroll
        for (int gq = 0; gq < 16; ++gq) {
          const int x = xb + 4 * gq;
          if (cv && lane == x / 4) s0 = s;  // (lane x/4's first term comes next)
          const f4a w = *reinterpret_cast<const f4a*>(&sT[x]);
#pragma unroll
          for (int q = 0; q < 4; ++q) s = s + (x + q >= done ? w[q] : 0.0f);
        }
      }
      if (cv) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (4 * lane + q >= done) {
            s0 = s0 + t[q];
            (*cv)[q] = s0;
          }
        }
      }
      state_of(rdl(s, 0), &E, &k);
      break;
    }
    if (rounds) ++*rounds;
    int r[4];
    bool tie[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bool tx;
      const float rf = units_of(t[q], E, &tx);
      const bool act = 4 * lane + q >= done;
      r[q] = act ? (int)rf : 0;
      tie[q] = act && tx;
    }
    int tot = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) tot += r[q];
    tot = min(tot, kK24 + 1);  // no scan overflow; anything above 2^24 fails anyway
    const int incl = wave_incl_scan(tot, lane);
    // the lane's terms in order: each applies (k grows by its increment)
    // until the first that does not (a tie, or past 2^24) -- selects, no
    // branches (a divergent if per term tripled the round's instructions)
    int kk = k + incl - tot, bad = 4, kb = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool act = bad == 4 && 4 * lane + q >= done;
      const bool stop = act && (tie[q] || kk + r[q] > kK24);
      const bool ok = act && !stop;
      bad = stop ? q : bad;
      kb = stop ? kk : kb;
      kk = ok ? kk + r[q] : kk;
      if (cv) (*cv)[q] = ok ? value_of(E, kk) : (*cv)[q];
    }
    const uint64_t bm = __ballot(bad < 4);
    if (bm == 0ull) {
      k += rdl(incl, 63);
      break;
    }
    const int lb = __builtin_ctzll(bm);
    // (the failing term picked per lane by masks -- no branches on the
    // scalar unit, and no dynamic index the compiler would put in scratch)
    const uint32_t tqb =
        (bits_of(t[0]) & (0u - (uint32_t)(bad == 0))) | (bits_of(t[1]) & (0u - (uint32_t)(bad == 1))) |
        (bits_of(t[2]) & (0u - (uint32_t)(bad == 2))) | (bits_of(t[3]) & (0u - (uint32_t)(bad == 3)));
    const float tq = __builtin_bit_cast(float, tqb);
    const int qb = rdl(bad, lb), kbef = rdl(kb, lb);
    const float tb = rdl(tq, lb);
    const float s = value_of(E, kbef) + tb;  // the reference's own add
    state_of(s, &E, &k);
    if (cv) {
#pragma unroll
      for (int q = 0; q < 4; ++q) (*cv)[q] = lane == lb && q == qb ? s : (*cv)[q];
    }
    // (values of later terms computed in this round were provisional: the
    // next round recomputes them)
    done = 4 * lb + qb + 1;
    if (done >= kFcChunk) break;
  }
  *pE = E;
  *pk = k;
}

// ---------------------------------------------------------------- driver
template <int BASE, int K>
__global__ __launch_bounds__(64) void k_fc_drive(FcArgs a) {
  constexpr int KC = K > 0 ? K : 1;
  __shared__ uint2 sE[kFcWin];
  __shared__ __attribute__((aligned(16))) float sStash[kFcStash][kFcChunk];
  __shared__ int sStashId[kFcStash];
  for (int ch = blockIdx.x;; ch += gridDim.x) {  // (one wave: uniform)
  const int g = ch / KC, i = ch % KC;
  int id;
  if (!group_id(a, g, &id)) return;
  if (K > 0 && a.cmask && !((a.cmask[id] >> i) & 1u)) continue;  // (not a candidate)
  Terms<BASE, K> T;
  T.init(a, id);
  const int lane = threadIdx.x;
  const int n = a.n, nch = fc_chunks(n), nseg = fc_segments(n);
  const int cx = a.by_id ? id * KC + i : ch;  // (the scratch chain)
  const uint2* tab = a.tab + (long long)cx * nch;
  const bool cdf = BASE == FC_ROW && K == 0 && a.cdf != nullptr;
  const unsigned long long tk0 = a.stats ? __builtin_amdgcn_s_memrealtime() : 0ull;
  unsigned long long tk1 = 0ull, tk2 = 0ull;
  uint32_t f = 0u;
  for (int s = lane; s < nseg; s += 64) f |= a.cflag[(long long)cx * nseg + s];
  f = (__ballot((f & kPos) != 0u) ? kPos : 0u) | (__ballot((f & kNeg) != 0u) ? kNeg : 0u) |
      (__ballot((f & kBad) != 0u) ? kBad : 0u);
  if (a.stats) tk1 = __builtin_amdgcn_s_memrealtime();
  const bool seq_all = (f & kBad) || ((f & kPos) && (f & kNeg));
  const bool neg = (f & kNeg) && !(f & kPos);
  if (cdf && lane == 0) a.cst[nch] = make_int2((int)f, 0);
  float res;
  if (seq_all) {
    // mixed signs or a non-finite term: the reference's chain itself
    float s = 0.0f;
    for (int j = 0; j < nch; ++j) {
      float t[4];
      T.terms4(i, j * kFcChunk + 4 * lane, t);
      float cv[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      for (int l = 0; l < 64; ++l) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          s = s + rdl(t[q], l);
          if (lane == l) cv[q] = s;
        }
      }
      if (cdf) {
        const int x0 = j * kFcChunk + 4 * lane;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (x0 + q < n) a.cdf[x0 + q] = cv[q];
      }
    }
    res = s;
  } else {
    int E = kEMin, k = 0, j = 0, wbase = -kFcWin, nstash = 0;
    int n_it = 0, n_fb = 0, n_rounds = 0, n_hit = 0;
    {
      // chunk 0 from the exact zero state as the chain itself, one fp32 add
      // per term: its running sum climbs through many binades (about log2
      // of its term count), each an exact round of ~1000 cycles, where the
      // sequential chain costs ~10 cycles a term
      float t[4];
      T.terms4(i, 4 * lane, t);
      float s = 0.0f;
#pragma unroll
      for (int l = 0; l < 64; ++l)
#pragma unroll
        for (int q = 0; q < 4; ++q) s = s + rdl(fabsf(t[q]), l);
      if (cdf && lane == 0) a.cst[0] = make_int2(kEMin, 0);
      state_of(s, &E, &k);
      normalise(&E, &k);
      j = 1;
    }
    while (j < nch) {
      ++n_it;
      if (j >= wbase + kFcWin) {  // the next window of entries, and its predicted fallbacks
        wbase = j;
        for (int c = lane; c < kFcWin; c += 64)
          sE[c] = wbase + c < nch ? tab[wbase + c] : make_uint2(kNoEntry, 0u);
        __syncthreads();
        nstash = 0;
        for (int c0 = 0; c0 < kFcWin && nstash < kFcStash && wbase + c0 < nch; c0 += 64) {
          const bool pr = wbase + c0 + lane < nch && (sE[c0 + lane].y & kPredicted);
          uint64_t m = __ballot(pr);
          while (m && nstash < kFcStash) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            if (lane == 0) sStashId[nstash] = wbase + c0 + l;
            ++nstash;
          }
        }
        __syncthreads();
        // all of the window's stash loads in flight together
        float st[kFcStash][4];
#pragma unroll
        for (int s2 = 0; s2 < kFcStash; ++s2)
          if (s2 < nstash) T.terms4(i, sStashId[s2] * kFcChunk + 4 * lane, st[s2]);
#pragma unroll
        for (int s2 = 0; s2 < kFcStash; ++s2)
          if (s2 < nstash)
            *reinterpret_cast<f4a*>(&sStash[s2][4 * lane]) =
                f4a{fabsf(st[s2][0]), fabsf(st[s2][1]), fabsf(st[s2][2]), fabsf(st[s2][3])};
        __syncthreads();
        if (a.stats && tk2 == 0ull) tk2 = __builtin_amdgcn_s_memrealtime();
      }
      const int jj = j + lane;
      const uint2 e = jj < nch && jj < wbase + kFcWin ? sE[jj - wbase] : make_uint2(kNoEntry, 0u);
      const bool valid = entry_applies(e.x, E);
      const int dl = valid ? entry_units(e.x) : 0;
      const int incl = wave_incl_scan(dl, lane);
      const bool ok = valid && k + incl <= kK24;
      const uint64_t badm = ~__ballot(ok);
      const int fc = badm == 0ull ? 64 : __builtin_ctzll(badm);
      if (cdf && lane < fc) a.cst[jj] = make_int2(E, k + incl - dl);
      if (fc > 0) {
        k += rdl(incl, fc - 1);
        normalise(&E, &k);
      }
      j += fc;
      if (j < nch && fc < 64 && j < wbase + kFcWin) {
        // chunk j term by term: from the stash, or loaded now
        if (cdf && lane == 0) a.cst[j] = make_int2(E, k);
        int slot = -1;
        for (int s2 = 0; s2 < nstash; ++s2)
          if (sStashId[s2] == j) slot = s2;
        float t[4];
        ++n_fb;
        if (slot >= 0) {
          ++n_hit;
          const f4a v = *reinterpret_cast<const f4a*>(&sStash[slot][4 * lane]);
#pragma unroll
          for (int q = 0; q < 4; ++q) t[q] = v[q];
        } else {
          T.terms4(i, j * kFcChunk + 4 * lane, t);
#pragma unroll
          for (int q = 0; q < 4; ++q) t[q] = fabsf(t[q]);
        }
        chunk_exact(t, lane, &E, &k, nullptr, &n_rounds);
        normalise(&E, &k);
        ++j;
      }
    }
    if (a.stats && lane == 0) {
      const unsigned long long tk3 = __builtin_amdgcn_s_memrealtime();
      atomicAdd(a.stats + 0, n_it);
      atomicAdd(a.stats + 1, n_fb);
      atomicAdd(a.stats + 2, n_rounds);
      atomicAdd(a.stats + 3, n_hit);
      // 100 MHz ticks: flags, first window + stash, the walk; chains
      atomicAdd(a.stats + 4, (int)(tk1 - tk0));
      atomicAdd(a.stats + 5, (int)(tk2 - tk1));
      atomicAdd(a.stats + 6, (int)(tk3 - tk2));
      atomicAdd(a.stats + 7, 1);
    }
    const float r = value_of(E, k);
    res = neg ? (r == 0.0f ? 0.0f : -r) : r;
  }
  if (lane == 0) {
    if (BASE == FC_LIST) {  // out[row * ldo + partner]
      const int2 e = a.plist[id];
      a.out[(long long)e.x * a.ldo + e.y] = res;
    } else {
      a.out[(long long)id * a.ldo + i] = res;
    }
  }
  __syncthreads();  // (the window / stash of the next chain)
  }
}

// ---------------------------------------------------------------- walker (round 6)
// k_fc_walk (below): k_fc_drive's job for chains of at most kWkEntries
// chunks (n <= 262144).  The first chunk runs as the fp32 chain itself (it
// climbs through many binades, an exact round each otherwise), every later
// exact chunk as exact rounds, the chain itself after eight (chunk_exact).
// (build knobs for same-box A/B builds, tools/ab_planner.sh: the walker's
// issue priority, the exact rounds before an exact chunk's chain tail)
#ifndef PP2_WALK_PRIO
#define PP2_WALK_PRIO 1
#endif
#ifndef PP2_CDF_TAIL  // (k_fc_cdf's exact rounds before the serial tail; A/B builds)
#define PP2_CDF_TAIL 8
#endif
#ifndef PP2_WALK_TAIL
#define PP2_WALK_TAIL 8
#endif
constexpr int kWkEntries = 1024;  // chunk entries in LDS
constexpr int kWkStash = 16;      // predicted fallback chunks staged in LDS
constexpr int kWkPlan = 128;      // predicted chunks whose crossing plans are staged in LDS
typedef __attribute__((address_space(3))) void fc_lds_void;
typedef __attribute__((address_space(1))) void fc_glb_void;

// the operand rows of chain (g, i): the base row and, for the products, the
// second factor (FC_CHILD: L_z; K = 9: the partner; FC_LIST: the alpha)
template <int BASE, int K>
struct WalkRows {
  const float* p0;
  const float* p1;  // nullptr: terms are p0 itself
  __device__ __forceinline__ void init(const FcArgs& a, int id, int i) {
    if (BASE == FC_ROW) {
      p0 = a.row + (long long)id * a.row_stride;
      p1 = K > 0 ? a.partners + (long long)i * a.ld : nullptr;
    } else if (BASE == FC_LIST) {
      const int2 e = a.plist[id];
      p0 = a.row + (long long)e.x * a.row_stride;
      p1 = a.partners + (long long)e.y * a.ld;
    } else {
      p0 = a.pred + (long long)(id % 9) * a.ld;
      p1 = a.lrows + (long long)(id / 9) * a.ld;
    }
  }
  // the term of operands (u, v): Terms' per-cell operation
  __device__ __forceinline__ float term(float u, float v) const {
    if (BASE == FC_CHILD) return ftz(u * ftz(v));
    return p1 ? u * v : u;
  }
};

constexpr int kSegSlow = 1 << 20;  // sSeg[].x: the segment was walked chunk by chunk

// k_fc_drive's job for chains of at most kWkEntries chunks, as a walk over
// SEGMENTS.  The tables mark the chunks a chain will likely not take from its
// entry (kPredicted: no entry, or the approximate running sum crosses a
// binade in it) -- the breaks.  Between two breaks lies a segment whose
// entries all apply at once when the state's domain is the one they were
// tabled for; one pass over the entries (4 per lane, segmented scans)
// records each segment's saturated increment and domain range, so the walk
// itself is a scalar loop: per segment one check and one add (a mispredicted
// segment walks its chunks as before), per break one exact chunk from the
// operand rows the same pass staged into LDS.  A walker is one wave running
// a chain of dependent instructions; what it saves is steps (a walk step over
// 256 entries was ~1000 cycles, a segment is tens).  With cdf the chunk start
// states go to cst: the breaks' as they are walked, every segment chunk's
// after the walk from its segment's start state and running increment.  Same
// outputs as k_fc_drive: tests/test_gpu_fchain.py runs both.
template <int BASE, int K>
__global__ __launch_bounds__(64) void k_fc_walk(FcArgs a) {
  constexpr int KC = K > 0 ? K : 1;
  __shared__ uint32_t sE[kWkEntries];
  __shared__ uint32_t sInc[kWkEntries];  // increments from the segment head (saturated)
  __shared__ uint32_t sKey[kWkEntries];  // domain keys from the segment head
  __shared__ short sOrd[kWkEntries];     // breaks before the chunk; a break: -(ordinal + 1)
  __shared__ short sBrk[kWkEntries];     // the breaks' chunks in order
  __shared__ int2 sSeg[kWkEntries + 1];  // (cdf) each segment's start state
  __shared__ __attribute__((aligned(16))) float sRaw[2][kWkStash][kFcChunk];
  __shared__ __attribute__((aligned(16))) float sT[kFcChunk];  // (chunk_exact's chain tails)
  __shared__ __attribute__((aligned(16))) uint32_t sPlan[kWkPlan][8];  // the first breaks' plans
  // (a walker is latency: first in its SIMD's issue arbitration, ahead of
  // the bandwidth kernels of the other stream sharing it)
  if (PP2_WALK_PRIO) __builtin_amdgcn_s_setprio(3);
  for (int ch = blockIdx.x;; ch += gridDim.x) {  // (one wave: uniform)
  const int g = ch / KC, i = ch % KC;
  int id;
  if (!group_id(a, g, &id)) return;
  if (K > 0 && a.cmask && !((a.cmask[id] >> i) & 1u)) continue;  // (not a candidate)
  WalkRows<BASE, K> R;
  R.init(a, id, i);
  const int lane = threadIdx.x;
  const int n = a.n, nch = fc_chunks(n), nseg = fc_segments(n);
  const int cx = a.by_id ? id * KC + i : ch;  // (the scratch chain)
  const uint2* tab = a.tab + (long long)cx * nch;
  const bool cdf = BASE == FC_ROW && K == 0 && a.cdf != nullptr;
  const unsigned long long tk0 = a.stats ? __builtin_amdgcn_s_memrealtime() : 0ull;
  unsigned long long tk1 = 0ull, tk2 = 0ull;
  int n_it = 0, n_fb = 0, n_rounds = 0, n_hit = 0, n_slow = 0, n_plan = 0;
  // 1. flags; entries, breaks and segment records (4 chunks a lane); the
  //    first kWkStash breaks' operand rows into LDS
  uint32_t f = 0u;
  for (int s = lane; s < nseg; s += 64) f |= a.cflag[(long long)cx * nseg + s];
  int nb = 0;
  uint32_t cs = 0u, ck = 0u;  // the records of the last chunk so far
#pragma unroll 1
  for (int c0 = 0; c0 < nch; c0 += 4 * 64) {
    uint2 t[4];
    bool br[4];
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + 4 * lane + q;
      t[q] = c < nch ? tab[c] : make_uint2(0u, 0u);
      br[q] = c < nch && ((t[q].y & kPredicted) || t[q].x == kNoEntry);
      cnt += br[q];
    }
    const int incl = wave_incl_scan(cnt, lane);
    int o = nb + incl - cnt;
    nb += rdl(incl, 63);
    uint32_t lf = 0u, ls = 0u, lk = 0u, vs[4], vk[4];
    bool vf[4];
    int oq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + 4 * lane + q;
      const uint32_t e = t[q].x;
      const uint32_t d = br[q] ? 0u : (uint32_t)entry_units(e);
      const uint32_t key = br[q] ? 0u : ((e >> 24) << 16) | (d > 0u ? 255u - (e >> 24) : 0u);
      const bool head = br[q] || c == 0;
      ls = head ? d : min(ls + d, kSegSat);
      lk = head ? key : pk_max(lk, key);
      lf |= head;
      vs[q] = ls;
      vk[q] = lk;
      vf[q] = lf != 0u;
      oq[q] = o;
      o += br[q];
      if (c < nch) {
        sE[c] = e;
        sOrd[c] = (short)(br[q] ? -(oq[q] + 1) : oq[q]);
        if (br[q]) sBrk[oq[q]] = (short)c;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint64_t m = __ballot(br[q] && oq[q] < (a.plan ? kWkPlan : kWkStash));
#pragma unroll 1
      while (m) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        const int s2 = rdl(oq[q], l);
        if (s2 < kWkStash) {
          long long x = (long long)(c0 + 4 * l + q) * kFcChunk + 4 * lane;
          x = x < a.ld ? x : 0;  // (cells past the row stride: read at 0, masked at use)
          __builtin_amdgcn_global_load_lds((fc_glb_void*)(R.p0 + x), (fc_lds_void*)&sRaw[0][s2][0],
                                           16, 0, 0);
          if (R.p1)
            __builtin_amdgcn_global_load_lds((fc_glb_void*)(R.p1 + x), (fc_lds_void*)&sRaw[1][s2][0],
                                             16, 0, 0);
        }
        if (a.plan && lane < 2)  // (the chunk's crossing plan: 2 x 16 B)
          __builtin_amdgcn_global_load_lds(
              (fc_glb_void*)(a.plan + 2 * ((long long)cx * nch + c0 + 4 * l + q) + lane),
              (fc_lds_void*)&sPlan[s2][0], 16, 0, 0);
      }
    }
    // the lanes' records: the carry into lane 0, the segmented scan, each
    // chunk's from the lane before (lane 0: the carry)
    uint32_t wf = lf, ws = ls, wk = lk;
    if (lane == 0 && !lf) {
      ws = min(cs + ws, kSegSat);
      wk = pk_max(ck, wk);
    }
    wave_seg_scan(wf, ws, wk);
    uint32_t es = dppu<0x138, 0xf>(ws), ek = dppu<0x138, 0xf>(wk);  // (wave_shr:1)
    es = lane == 0 ? cs : es;
    ek = lane == 0 ? ck : ek;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + 4 * lane + q;
      if (!vf[q]) {
        vs[q] = min(es + vs[q], kSegSat);
        vk[q] = pk_max(ek, vk[q]);
      }
      if (c < nch) {
        sInc[c] = vs[q];
        sKey[c] = vk[q];
      }
    }
    cs = (uint32_t)rdl((int)vs[3], 63);
    ck = (uint32_t)rdl((int)vk[3], 63);
  }
  f = (__ballot((f & kPos) != 0u) ? kPos : 0u) | (__ballot((f & kNeg) != 0u) ? kNeg : 0u) |
      (__ballot((f & kBad) != 0u) ? kBad : 0u);
  if (cdf && lane == 0) a.cst[nch] = make_int2((int)f, 0);
  const bool seq_all = (f & kBad) || ((f & kPos) && (f & kNeg));
  const bool neg = (f & kNeg) && !(f & kPos);
  if (a.stats) tk1 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the LDS-DMA has landed)
  __syncthreads();
  if (a.stats) tk2 = __builtin_amdgcn_s_memrealtime();
  float res;
  if (seq_all) {
    // mixed signs or a non-finite term: the reference's chain itself (rare:
    // a rolled loop, one term per iteration)
    float s = 0.0f;
#pragma unroll 1
    for (int x = 0; x < n; ++x) {
      const float t = R.term(R.p0[x], R.p1 ? R.p1[x] : 0.0f);
      s = s + t;
      if (cdf && lane == 0) a.cdf[x] = s;
    }
    res = s;
  } else {
    int E = kEMin, k = 0;
    unsigned long long c_step = 0ull, c_fetch = 0ull, c_exact = 0ull, c_zero = 0ull, c0 = 0ull;
    // operands of chunk j (stash slot sl, or from the rows)
    auto operands = [&](int j, int sl, f4a* u, f4a* v) {
      *v = f4a{0.0f, 0.0f, 0.0f, 0.0f};
      if (sl >= 0) {
        *u = *reinterpret_cast<const f4a*>(&sRaw[0][sl][4 * lane]);
        if (R.p1) *v = *reinterpret_cast<const f4a*>(&sRaw[1][sl][4 * lane]);
      } else {
        const int x0 = j * kFcChunk + 4 * lane;
        const int xs = x0 < a.ld ? x0 : 0;  // (masked at use)
        *u = *reinterpret_cast<const f4a*>(R.p0 + xs);
        if (R.p1) *v = *reinterpret_cast<const f4a*>(R.p1 + xs);
      }
    };
    // chunk j from the state: by its crossing plan (plan words pw, lane l
    // holding word l; plan: whether it has one), else term by term from
    // operands u, v of the lane's 4 cells (stash slot sl; sl < 0: loaded
    // from the rows here)
    auto exact_chunk = [&](int j, int sl, f4a u, f4a v, uint32_t pw, bool plan) {
      if (cdf && lane == 0) a.cst[j] = make_int2(E, k);
      ++n_fb;
      n_hit += sl >= 0;
      const int x0 = j * kFcChunk + 4 * lane;
      const uint32_t w0 = plan ? (uint32_t)rdl((int)pw, 0) : 0u;
      if (w0 & 1u) {
        // d_0 in E0, then per crossing the reference's own add and the
        // increments of the run after it
        const int nc = (int)((w0 >> 1) & 3u);
        int Ep = E, kp = k + rdl((int)pw, 1);
        bool ok = E == (int)((w0 >> 8) & 255u) - 128 && kp <= kK24;
#pragma unroll
        for (int sg = 1; sg <= kPlanMax; ++sg) {
          if (ok && sg <= nc) {
            const float sv = value_of(Ep, kp) + rdl(__builtin_bit_cast(float, pw), 2 * sg);
            state_of(__builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                                                   __builtin_bit_cast(int, sv))),
                     &Ep, &kp);
            kp += rdl((int)pw, 2 * sg + 1);
            ok = Ep == E + (int)((w0 >> (12 + 4 * sg)) & 15u) && kp <= kK24;
          }
        }
        if (ok) {
          E = Ep;
          k = kp;
          normalise(&E, &k);
          ++n_plan;
          if (a.stats) {
            const unsigned long long c1 = __builtin_amdgcn_s_memtime();
            c_fetch += c1 - c0;
            c0 = c1;
          }
          return;
        }
      }
      if (sl < 0) operands(j, -1, &u, &v);
      float t[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = x0 + q < n ? fabsf(R.term(u[q], v[q])) : 0.0f;
      if (a.stats) {
        const float tt = t[0] + t[1] + t[2] + t[3];  // (the fetch has landed)
        asm volatile("" ::"v"(tt));
        const unsigned long long c1 = __builtin_amdgcn_s_memtime();
        c_fetch += c1 - c0;
        c0 = c1;
      }
      // (from zero, the chunk climbs through many binades: the chain itself
      // at once; else exact rounds, the chain itself after eight)
      chunk_exact(t, lane, &E, &k, nullptr, &n_rounds, sT, j == 0 ? 0 : PP2_WALK_TAIL);
      normalise(&E, &k);
      if (a.stats) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime();
        (j == 0 ? c_zero : c_exact) += c1 - c0;
        c0 = c1;
      }
    };
    // a mispredicted segment [j, end): walk steps over its entries (256 a
    // step, 4 a lane, branch-free), each failing chunk exactly
    auto walk_steps = [&](int j, int end) {
#pragma unroll 1
      while (j < end) {
        ++n_it;
        uint32_t ev[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) ev[q] = sE[min(j + 4 * lane + q, nch - 1)];
        const uint32_t ebias = (uint32_t)(E + 128);
        int dq[4], tot = 0;
        bool vq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          vq[q] = (j + 4 * lane + q < end) & (ev[q] != kNoEntry) &
                  (((ev[q] >> 24) == ebias) | (((ev[q] & 0xffffffu) == 0u) & ((ev[q] >> 24) < ebias)));
          dq[q] = vq[q] ? (int)(ev[q] & 0xffffffu) : 0;
          tot += dq[q];
        }
        tot = min(tot, kK24 + 1);
        const int excl = wave_incl_scan(tot, lane) - tot;
        int run = k + excl, fq = 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool stop = fq == 4 && (!vq[q] || run + dq[q] > kK24);
          fq = stop ? q : fq;
          run = fq == 4 ? run + dq[q] : run;
        }
        const uint64_t failm = __ballot(fq < 4);
        const int L = failm ? __builtin_ctzll(failm) : 64;
        if (cdf && lane <= L) {
          int r2 = k + excl;
          const int lim = lane < L ? 4 : fq;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = j + 4 * lane + q;
            if (q < lim && m < end) a.cst[m] = make_int2(E, r2);
            r2 += dq[q];
          }
        }
        const int fc = L < 64 ? 4 * L + rdl(fq, L) : 256;
        k = rdl(run, L < 64 ? L : 63);
        normalise(&E, &k);
        j += fc;
        // (a stop at the exact top of a binade: the normalised state may take
        // chunk j's entry after all -- the next step does)
        const uint32_t ej = j < end ? sE[j] : kNoEntry;
        if (j < end && L < 64 && !(entry_applies(ej, E) && k + entry_units(ej) <= kK24)) {
          exact_chunk(j, -1, f4a{0.0f, 0.0f, 0.0f, 0.0f}, f4a{0.0f, 0.0f, 0.0f, 0.0f}, 0u, false);
          ++j;
        }
      }
    };
    // the first 64 segments' records in registers (lane l: segment l's end,
    // increment and keys; an empty segment's are neutral)
    int rb = nch;
    uint32_t rS = 0u, rK = 0u;
    if (lane <= nb) {
      rb = lane < nb ? (int)sBrk[lane] : nch;
      const int ra = lane == 0 ? 0 : (int)sBrk[lane - 1] + 1;
      if (ra < rb) {
        rS = sInc[rb - 1];
        rK = sKey[rb - 1];
      }
    }
    // (break 0's operands and plan words, staged one break ahead)
    f4a nu = {0.0f, 0.0f, 0.0f, 0.0f}, nv = nu;
    if (nb > 0 && kWkStash > 0) operands(0, 0, &nu, &nv);
    const int npl = a.plan ? min(nb, kWkPlan) : 0;
    uint32_t npw = npl > 0 ? sPlan[0][lane & 7] : 0u;
    if (a.stats) c0 = __builtin_amdgcn_s_memtime();
    // 2. the walk: segment i (from break i - 1 to break i), then break i
    int a0 = 0;
#pragma unroll 1
    for (int bi = 0;; ++bi) {
      normalise(&E, &k);
      int b;
      uint32_t S, ky;
      if (bi < 64) {
        b = rdl(rb, bi);
        S = (uint32_t)rdl((int)rS, bi);
        ky = (uint32_t)rdl((int)rK, bi);
      } else {
        b = bi < nb ? (int)sBrk[bi] : nch;
        S = a0 < b ? sInc[b - 1] : 0u;
        ky = a0 < b ? sKey[b - 1] : 0u;
      }
      if (a0 < b) {
        const int eb = E + 128;
        const bool fast =
            (int)(ky >> 16) <= eb && 255 - (int)(ky & 0xffffu) >= eb && (int)S <= kK24 - k;
        if (fast) {
          if (cdf && lane == 0) sSeg[bi] = make_int2(E, k);
          k += (int)S;
        } else {
          if (cdf && lane == 0) sSeg[bi] = make_int2(kSegSlow, 0);
          ++n_slow;
          walk_steps(a0, b);
        }
      }
      if (a.stats) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime();
        c_step += c1 - c0;
        c0 = c1;
      }
      if (bi >= nb) break;
      normalise(&E, &k);
      const int sl = bi < kWkStash ? bi : -1;
      const f4a u = nu, v = nv;
      const uint32_t pw = npw;
      // (the next break's, ahead)
      if (bi + 1 < nb && bi + 1 < kWkStash) operands(0, bi + 1, &nu, &nv);
      if (bi + 1 < npl) npw = sPlan[bi + 1][lane & 7];
      exact_chunk(b, sl, u, v, pw, bi < npl);
      a0 = b + 1;
    }
    // 3. (cdf) every segment chunk's start state
    if (cdf) {
#pragma unroll 1
      for (int m = lane; m < nch; m += 64) {
        const int o = sOrd[m];
        if (o < 0) continue;  // (a break: walked above)
        const int2 st = sSeg[o];
        if (st.x == kSegSlow) continue;
        a.cst[m] = make_int2(st.x, st.y + (int)(sInc[m] - (uint32_t)entry_units(sE[m])));
      }
    }
    if (a.stats && lane == 0) {  // (s_memtime cycles: segments, fetches, exact rounds, chunk 0)
      atomicAdd(a.stats + 8, nb);
      atomicAdd(a.stats + 9, n_slow);
      atomicAdd(a.stats + 10, n_plan);
      atomicAdd(a.stats + 11, (int)c_step);
      atomicAdd(a.stats + 12, (int)c_fetch);
      atomicAdd(a.stats + 13, (int)c_exact);
      atomicAdd(a.stats + 14, (int)c_zero);
    }
    const float r = value_of(E, k);
    res = neg ? (r == 0.0f ? 0.0f : -r) : r;
  }
  if (a.stats && lane == 0) {
    const unsigned long long tk3 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(a.stats + 0, n_it);
    atomicAdd(a.stats + 1, n_fb);
    atomicAdd(a.stats + 2, n_rounds);
    atomicAdd(a.stats + 3, n_hit);
    // 100 MHz ticks: flags + entries + the stash issued, the stash landed, the walk; chains
    atomicAdd(a.stats + 4, (int)(tk1 - tk0));
    atomicAdd(a.stats + 5, (int)(tk2 - tk1));
    atomicAdd(a.stats + 6, (int)(tk3 - tk2));
    atomicAdd(a.stats + 7, 1);
    // (the longest chain, 100 MHz ticks, and -- racy, a diagnostic -- its
    // breaks, exact rounds, mispredicted segments, stash hits, entries)
    const int dur = (int)(tk3 - tk0);
    if (atomicMax(a.stats + 15, dur) < dur) {
      a.stats[16] = n_fb;
      a.stats[17] = n_rounds;
      a.stats[18] = n_it;
      a.stats[19] = n_hit;
      a.stats[20] = nch;
      a.stats[21] = id;
    }
  }
  if (lane == 0) {
    if (BASE == FC_LIST) {  // out[row * ldo + partner]
      const int2 e = a.plist[id];
      a.out[(long long)e.x * a.ldo + e.y] = res;
    } else {
      a.out[(long long)id * a.ldo + i] = res;
    }
  }
  __syncthreads();  // (the LDS of the next chain)
  }
}

// ---------------------------------------------------------------- running sums
// One wave per chunk: every running sum of the row from the chunk's exact
// start state (k_fc_drive's a.cst), term by term (chunk_exact).
__global__ __launch_bounds__(256) void k_fc_cdf(FcArgs a) {
  __shared__ __attribute__((aligned(16))) float sT[4][kFcChunk];  // (chunk_exact's chain tails)
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int n = a.n, nch = fc_chunks(n);
  if (j >= nch) return;
  const uint32_t f = (uint32_t)a.cst[nch].x;
  if ((f & kBad) || ((f & kPos) && (f & kNeg))) return;  // the driver wrote them itself
  const bool neg = (f & kNeg) && !(f & kPos);
  Terms<FC_ROW, 0> T;
  T.init(a, a.g0);
  float t[4];
  const int x0 = j * kFcChunk + 4 * lane;
  T.terms4(0, x0, t);
#pragma unroll
  for (int q = 0; q < 4; ++q) t[q] = fabsf(t[q]);
  int E = a.cst[j].x, k = a.cst[j].y;
  float cv[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  chunk_exact(t, lane, &E, &k, &cv, nullptr, sT[threadIdx.x >> 6], PP2_CDF_TAIL);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float v = neg ? (cv[q] == 0.0f ? 0.0f : -cv[q]) : cv[q];
    if (x0 + q < n) a.cdf[x0 + q] = v;
  }
  // the last running sum of every 16 cells (k_tree_sample's first search;
  // past n the sums stay at the row's total)
  if (a.sub && (lane & 3) == 3 && (x0 + 3) / 16 < (n + 15) / 16)
    a.sub[(x0 + 3) / 16] = neg ? (cv[3] == 0.0f ? 0.0f : -cv[3]) : cv[3];
}

// ---------------------------------------------------------------- sampling
// QNode::forwardSampling for the 9 actions of an expansion
// (search_tree_cuda.cu:176-196, :311-366): draw j of action a takes the
// state from the belief's cdf with the host's rand() value r[a N + j]
// (find_if: the first running sum >= r), the next state from the cumulative
// T row with curand uniform u1[j], the observation from the cumulative L row
// with u2[j] (host-order fp32 cumulative sums).  Then the observations'
// counts per action, counts[a * 16 + z], and the kept children c = z * 9 + a
// in std::set order (klist, *kcount).
constexpr int kSampleSub = 4096;  // 16-cell running-sum ends held in LDS (n <= 65536)
__global__ __launch_bounds__(1024) void k_tree_sample(SampleArgs s, FcRowTable rows) {
  __shared__ int cnt[144];
  if (s.rows_out && threadIdx.x < 144) s.rows_out[threadIdx.x] = rows.p[threadIdx.x];
  __shared__ float sSub[kSampleSub];
  for (int i = threadIdx.x; i < 144; i += blockDim.x) cnt[i] = 0;
  const int N = s.N, n = s.n, W = s.g.width;
  const int nsub = (n + 15) / 16;
  // a non-decreasing cdf (no negative or non-finite cell: the chain-set
  // flags) with its 16-cell ends: first the 16 cells, in LDS, then the cell
  const uint32_t f = s.sub ? (uint32_t)s.cst[(n + kFcChunk - 1) / kFcChunk].x : 0u;
  const bool two = s.sub && nsub <= kSampleSub && !(f & kNeg) && !(f & kBad);
  if (two)
    for (int i = threadIdx.x; i < nsub; i += blockDim.x) sSub[i] = s.sub[i];
  __syncthreads();
  for (int jt = threadIdx.x; jt < 9 * N; jt += blockDim.x) {
    const int act = jt / N, j = jt - act * N;
    const float r = s.r[jt];
    int s1 = n;  // the first x with cdf[x] >= r (n: none)
    if (two) {
      int l2 = 0, h2 = nsub;
      while (l2 < h2) {
        const int mid = (l2 + h2) >> 1;
        if (sSub[mid] < r) l2 = mid + 1;
        else h2 = mid;
      }
      if (l2 < nsub) {
        float cv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) cv[q] = 16 * l2 + q < n ? s.cdf[16 * l2 + q] : INFINITY;
#pragma unroll
        for (int q = 15; q >= 0; --q)
          if (cv[q] >= r) s1 = 16 * l2 + q;
      }
    } else {
      int lo = 0, hi = n;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s.cdf[mid] < r) lo = mid + 1;
        else hi = mid;
      }
      s1 = lo;
    }
    if (s1 >= n) {  // the reference runs off its arrays: the last cell with mass
      s1 = n - 1;
      while (s1 > 0 && s.cdf[s1] == s.cdf[s1 - 1]) --s1;
    }
    const int y1 = s1 / W, x1 = s1 - y1 * W;
    float td = 0.0f;
    uint32_t s2i = 0;
    bool found = false;
    for (int q = 0; q < 9; ++q) {
      const float tv = s.T.p[(long long)y1 * s.T.rs + (long long)(9 * act + q) * s.T.ps + x1];
      td = q == 0 ? tv : td + tv;
      if (!found && s.u1[j] <= td) {
        s2i = (uint32_t)q;
        found = true;
      }
    }
    uint32_t s2 = (uint32_t)s1 + (s2i / 3 - 1) * (uint32_t)W + (s2i % 3 - 1);
    if (s2 >= (uint32_t)n) s2 = (uint32_t)s1;  // (never with a row-stochastic T)
    const int y2 = (int)(s2 / (uint32_t)W), x2 = (int)(s2 - (uint32_t)y2 * (uint32_t)W);
    float ld = 0.0f;
    int o = 0;
    found = false;
    for (int q = 0; q < 16; ++q) {
      const float lv = s.L.p[(long long)y2 * s.L.rs + (long long)q * s.L.ps + x2];
      ld = q == 0 ? lv : ld + lv;
      if (!found && s.u2[j] <= ld) {
        o = q;
        found = true;
      }
    }
    atomicAdd(&cnt[act * 16 + o], 1);
  }
  __syncthreads();
  // the kept children z * 9 + act in std::set order (act-major, z inner): a
  // compaction of cnt[act * 16 + z] > 0 over its 144 entries (3 waves)
  __shared__ int wtot[3];
  const int i = threadIdx.x, lane = i & 63, wv = i >> 6;
  const bool kept = i < 144 && cnt[i] > 0;
  const uint64_t m = __ballot(kept);
  const int pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (wv < 3 && lane == 0) wtot[wv] = __popcll(m);
  __syncthreads();
  if (i < 144) {
    const int off = (wv >= 1 ? wtot[0] : 0) + (wv >= 2 ? wtot[1] : 0);
    if (kept) s.klist[off + pre] = (i & 15) * 9 + (i >> 4);
    s.counts[i] = cnt[i];
    if (i == 0) *s.kcount = wtot[0] + wtot[1] + wtot[2];
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
  L.dst[r][x] = v / sums[c];  // b[x] /= sum (search_tree_cuda.cu:228-229)
}

// k_store_children over the kept children of the device list (klist,
// *kcount): child c into dst + c * ld.
__global__ __launch_bounds__(256) void k_store_kept(const int* __restrict__ klist,
                                                    const int* __restrict__ kcount,
                                                    const float* __restrict__ pred,
                                                    const float* __restrict__ lrows,
                                                    const float* __restrict__ sums,
                                                    float* __restrict__ dst, int n, int ld,
                                                    FcRowTable rows) {
  const int r = blockIdx.y;
  if (r >= *kcount) return;
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= n) return;
  const int c = klist[r];
  const float v = ftz(pred[(long long)(c % 9) * ld + x] * ftz(lrows[(long long)(c / 9) * ld + x]));
  const float b = v / sums[c];  // b[x] /= sum (search_tree_cuda.cu:228-229)
  dst[(long long)c * ld + x] = b;
  if (rows.use) rows.p[c][x] = b;
}

// The kept children's FIB candidates (launch_fib_cands).  The sums pass
// formed chain i's chunk sums A_j of |t'|, t' = fl(fl(w / m') alpha) with the
// approximate mass m' (kept_mass from msum); the chain's terms are
// t = fl(fl(w / m) alpha) with the exact mass m, so the chunk sums C_j of |t|
// are within A_j m' / m (1 +- 2^-15) -- the sums' rounding, < 2^-18, and 4
// roundings per term -- plus an absolute n 2^-100 for subnormal results
// (|alpha| < 2^40).  When no term is positive or non-finite, the reference's
// x-ordered fp32 chain R is <= 0, and each of its n adds rounds by at most u
// (= 2^-24) times its partial sum, itself at most (1 + n u / (1 - n u)) times
// the prefix of |t| through the add's chunk: | |R| - T | <= u (1 + ...) 256
// sum_j (nch - j) C_j (T = sum |t|).  A chain whose lowest |R| exceeds
// another's highest has the lower dot, never evaluateFibCpu's first maximum:
// out = -inf, and it is neither tabled nor walked.
__global__ __launch_bounds__(64) void k_fib_cands(FcArgs a, uint16_t* __restrict__ cmask) {
  const int lane = threadIdx.x;
  for (int g = blockIdx.x;; g += gridDim.x) {
    int id;
    if (!group_id(a, g, &id)) return;
    const int nch = fc_chunks(a.n), nseg = fc_segments(a.n);
    FcArgs ap = a;
    ap.mass = nullptr;  // (the sums pass's m'; kept_unit: 1)
    const double mp = kept_mass(ap, id, nch, lane), m = a.mass[id];
    const double nu = (double)a.n * 0x1p-24, rel = nu / (1.0 - nu);
    // (subnormal results: the chain's terms, and the sums pass's rescaled by
    // m' / m -- with kept_unit m' = 1 and m can be small)
    const double absl = (double)a.n * (0x1p-100 + 0x1p-148 * (mp / m));
    const bool mok = mp > 0.0 && m > 0.0 && isfinite(mp) && isfinite(m) && nu < 0.5;
    double lo[9], hi[9];
    bool bounded[9];
    // (every chain's loads issued before any sum: one round trip per 64 chunks)
    float acc[9], wacc[9];  // sum A_j, sum (nch - j) A_j
    uint32_t f[9];
    const float* cs = a.csum + (long long)id * 9 * nch;
    const uint32_t* cf = a.cflag + (long long)id * 9 * nseg;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      acc[i] = wacc[i] = 0.0f;
      f[i] = 0u;
    }
    for (int c = lane; c < nch; c += 64)
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const float x = cs[(long long)i * nch + c];
        acc[i] += x;
        wacc[i] = __builtin_fmaf((float)(nch - c), x, wacc[i]);
      }
    for (int c = lane; c < nseg; c += 64)
#pragma unroll
      for (int i = 0; i < 9; ++i) f[i] |= cf[(long long)i * nseg + c];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const double A = mok ? (double)wave_sum(acc[i]) * (mp / m) : INFINITY;
      const double W = mok ? (double)wave_sum(wacc[i]) * (mp / m) * (1.0 + 0x1p-15) : INFINITY;
      const double err = 0x1p-24 * (1.0 + rel) * 256.0 * W + absl;
      lo[i] = A * (1.0 - 0x1p-15) - err;
      hi[i] = A * (1.0 + 0x1p-15) + err;
      bounded[i] = __ballot((f[i] & (kPos | kBad)) != 0u) == 0ull && hi[i] < 0x1p126;
    }
    // the smallest upper bound of |R| over the bounded chains
    double hi_min = INFINITY;
#pragma unroll
    for (int i = 0; i < 9; ++i)
      if (bounded[i]) hi_min = fmin(hi_min, hi[i]);
    uint32_t cm = 0u;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const bool cand = !bounded[i] || lo[i] <= hi_min;
      cm |= cand ? 1u << i : 0u;
      if (!cand && lane == 0) a.out[(long long)id * a.ldo + i] = -INFINITY;
    }
    if (lane == 0) cmask[id] = (uint16_t)cm;
  }
}

// The kept children's dense rows (src + c * ld) into their node rows
// rows.p[c] -- beside the FIB walk that reads the dense ones.
__global__ __launch_bounds__(256) void k_copy_kept(const int* __restrict__ klist,
                                                   const int* __restrict__ kcount,
                                                   const float* __restrict__ src, int n, int ld,
                                                   FcRowTable rows) {
  const int r = blockIdx.y;
  if (r >= *kcount) return;
  const int c = klist[r];
  const int x = 4 * (blockIdx.x * 256 + threadIdx.x);
  if (x >= n) return;
  const float* s = src + (long long)c * ld + x;
  float* d = rows.p[c] + x;
  if (x + 4 <= n) {
    *reinterpret_cast<f4a*>(d) = *reinterpret_cast<const f4a*>(s);
  } else {
    for (int q = 0; x + q < n; ++q) d[q] = s[q];
  }
}

// ================================================================ fused chain sets
// (round 6) A chain set as ONE launch: one workgroup of 1024 threads per
// chain of n <= 1024 C cells (C = 16, 32 or 64 terms per thread; 256^2 takes
// C = 64), the chain's |terms| held in registers from the first pass to the
// last --
//   A  thread t forms the C consecutive terms of chunk t (cells [C t, C t +
//      C)), keeps |t|, its approximate chunk sum and the sign flags;
//   B  a workgroup scan of the approximate sums: the approximate running sum
//      before each chunk;
//   C  each chunk's table entry (binade E of that running sum, the chunk's
//      integer increment d in E) and whether the walk will likely fall back
//      there -- those chunks' |terms| go to an LDS stash;
//   D  wave 0 walks the entries 64 at a time with the exact state (E, k) and
//      adds each fallback chunk term by term, one fp32 add per term (the
//      reference's own chain), from the stash or from the terms formed again;
// and, for the expanded belief (k_fx_cdf_sample), every running sum from its
// chunk's exact start state, then forwardSampling's 9 x N draws on them.  The
// three launches of a k_fc_* set (sums, tables, drive: ~70-80 us on the 256^2
// plan step's critical path, profiles/r05 kernel_stats_plan_*) become one.
constexpr int kFxThreads = 1024;
constexpr int kFxStash = 32;  // predicted fallback chunks whose |terms| wave 0 reads from LDS
constexpr uint32_t kFxZero = 0xfffffffeu;  // entry of a chunk of zero terms: applies in any binade

// diagnostics: workgroup thread 0 stamps the 100 MHz clock at phase k
__device__ __forceinline__ void fx_stamp(const FxArgs& a, int k) {
  if (a.stamps && threadIdx.x == 0)
    a.stamps[8 * (long long)blockIdx.x + k] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ bool fx_group(const FxArgs& a, int g, int* id) {
  if (g >= a.ngroups) return false;
  if (a.gcount && g >= *a.gcount) return false;
  *id = a.glist ? a.glist[g] : a.g0 + g;
  return true;
}

// The terms of one chain (group id, partner i):
//   FX_ROW    row[id][x] (K = 9: * partners[i][x], the host's product)
//   FX_CHILD  fl_ftz(pred[id % 9][x] * fl_ftz(L[id / 9][x])) -- the
//             unnormalised child (cudaBayesBeliefUpdate's last product)
//   FX_KEPT   the normalised child b[x] = that / sums[id] (search_tree_cuda.cu:
//             228-229), times partners[i][x] (evaluateFibCpu's product)
// the same per-cell operations as k_fc_* (Terms) and k_store_kept.
template <int SRC, int K>
struct FxTerms {
  const float* __restrict__ pr;
  const float* __restrict__ lr;
  const float* __restrict__ al;
  float mass;
  int n;

  __device__ __forceinline__ void init(const FxArgs& a, int id, int i) {
    n = a.n;
    al = K > 0 ? a.partners + (long long)i * a.ld : nullptr;
    if (SRC == FX_ROW) {
      pr = a.row + (long long)id * a.row_stride;
      lr = nullptr;
      mass = 1.0f;
    } else {
      pr = a.pred + (long long)(id % 9) * a.ld;
      lr = a.lrows + (long long)(id / 9) * a.ld;
      mass = SRC == FX_KEPT ? a.sums[id] : 1.0f;
    }
  }
  // the base value (FX_KEPT: the normalised child) of one cell
  __device__ __forceinline__ float base1(float p, float l) const {
    if (SRC == FX_ROW) return p;
    const float v = ftz(p * ftz(l));
    return SRC == FX_KEPT ? v / mass : v;
  }
  __device__ __forceinline__ float term1(float b, float w) const { return K > 0 ? b * w : b; }
  // the term of cell x (0 at or past n): the walker's reload
  __device__ __forceinline__ float at(int x) const {
    if (x >= n) return 0.0f;
    return term1(base1(pr[x], SRC == FX_ROW ? 0.0f : lr[x]), K > 0 ? al[x] : 0.0f);
  }
  // 4 cells from x0 (x0 + 4 <= the row stride): the bases (FX_KEPT's stored
  // rows) and the terms, 0 past n
  __device__ __forceinline__ void at4(int x0, float (&b)[4], float (&t)[4]) const {
    const f4a p = *reinterpret_cast<const f4a*>(pr + x0);
    f4a l = {0.0f, 0.0f, 0.0f, 0.0f}, w = {0.0f, 0.0f, 0.0f, 0.0f};
    if (SRC != FX_ROW) l = *reinterpret_cast<const f4a*>(lr + x0);
    if (K > 0) w = *reinterpret_cast<const f4a*>(al + x0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      b[q] = x0 + q < n ? base1(p[q], l[q]) : 0.0f;
      t[q] = x0 + q < n ? term1(b[q], w[q]) : 0.0f;
    }
  }
};

// Shared state of one chain's workgroup.  A chunk is kFxC = 64 consecutive
// cells; the workgroup's 16 waves take 64 chunks each.  In the passes over the
// terms a chunk is one 16-lane row of a wave (4 cells per lane): a wave's
// 16-B loads then cover 1 KB of consecutive cells, 4 chunks per instruction.
constexpr int kFxC = 64;
struct FxShared {
  uint32_t e[kFxThreads];   // chunk entries (kNoEntry: none)
  float cb[kFxThreads];     // the approximate chunk sum (A), then the running sum before it (B)
  int slot[kFxThreads];     // the chunk's stash slot, or -1
  float start[kFxThreads];  // the chunk's exact start value (running sums)
  __attribute__((aligned(16))) float st[kFxStash][kFxC];
  float wsum[16];
  uint32_t flag;
  int nst;
  float res;
};

// broadcast lane i of each 16-lane row to the row (DPP row_newbcast, gfx950)
template <int I>
__device__ __forceinline__ float row_bcast(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0x150 + I, 0xf, 0xf, false));
}
// the 16-lane row's total in its lane 15 (any association; float, or int below 2^31)
__device__ __forceinline__ float row_total_f(float v) {
  int b = __builtin_bit_cast(int, v);
#pragma unroll
  for (int c = 1; c < 16; c <<= 1)
    b = __builtin_bit_cast(int, __builtin_bit_cast(float, b) +
                                    __builtin_bit_cast(float, row_shr(b, c)));
  return __builtin_bit_cast(float, b);
}
__device__ __forceinline__ int row_total_i(int v) {
#pragma unroll
  for (int c = 1; c < 16; c <<= 1) v += row_shr(v, c);
  return v;
}

// Phases A-D of one chain (every thread of the workgroup calls it; returns
// with the workgroup synchronised, the result in S.res and, with RUN, every
// chunk's exact start value in S.start); *pf the chain's sign flags.  The
// passes form the terms again from the (L2-resident) rows instead of holding
// them: the loops stay loops (a fully unrolled kernel runs once through ~20
// KB of code), and the registers stay few.
template <int SRC, int K, bool RUN>
__device__ __forceinline__ void fx_walk(const FxArgs& a, const FxTerms<SRC, K>& T, FxShared& S,
                                        uint32_t* pf, int id, int i) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rw = lane >> 4, c16 = lane & 15;
  const int n = a.n, nch = (n + kFxC - 1) / kFxC;
  fx_stamp(a, 0);
  if (tid == 0) {
    S.flag = 0u;
    S.nst = 0;
  }
  // A: flags and approximate chunk sums, 4 chunks per wave instruction (FX_KEPT,
  // partner 0: the normalised child stored on the way)
  uint32_t fl = 0u;
  {
    float* __restrict__ store = nullptr;
    float* __restrict__ store2 = nullptr;
    if (SRC == FX_KEPT && i == 0) {
      store = a.rows_out ? a.rows_out + (long long)id * a.ld : nullptr;
      store2 = a.use_dst ? a.dst[id] : nullptr;
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int j = 64 * w + 4 * g + rw, x = kFxC * j + 4 * c16;
      float b[4] = {0.0f, 0.0f, 0.0f, 0.0f}, t[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (x < n) T.at4(x, b, t);
      if (SRC == FX_KEPT && x < n) {
        if (store) *reinterpret_cast<f4a*>(store + x) = f4a{b[0], b[1], b[2], b[3]};
        if (store2) *reinterpret_cast<f4a*>(store2 + x) = f4a{b[0], b[1], b[2], b[3]};
      }
      float s4 = 0.0f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        fl |= !isfinite(t[q]) ? kBad : t[q] > 0.0f ? kPos : t[q] < 0.0f ? kNeg : 0u;
        s4 += fabsf(t[q]);
      }
      s4 = row_total_f(s4);
      if (c16 == 15) S.cb[j] = s4;
    }
  }
  {
    const uint32_t f = (__ballot((fl & kPos) != 0u) ? kPos : 0u) |
                       (__ballot((fl & kNeg) != 0u) ? kNeg : 0u) |
                       (__ballot((fl & kBad) != 0u) ? kBad : 0u);
    __syncthreads();  // (S.flag, S.nst initialised; S.cb written)
    fx_stamp(a, 1);
    if (lane == 0 && f) atomicOr(&S.flag, f);
  }
  // B: the approximate running sum before each chunk (thread t: chunk t)
  {
    const float cs = S.cb[tid];
    const float incl = wave_incl_scan_f(cs, lane);
    if (lane == 63) S.wsum[w] = incl;
    __syncthreads();
    float before = incl - cs;
    for (int v = 0; v < w; ++v) before += S.wsum[v];
    S.cb[tid] = before;
  }
  __syncthreads();
  fx_stamp(a, 2);
  const uint32_t f = S.flag;
  *pf = f;
  const bool seq_all = (f & kBad) || ((f & kPos) && (f & kNeg));
  // C: each chunk's entry; the predicted fallbacks' |terms| into the stash
  if (!seq_all) {
    float bef[16];  // (the 16 chunks' running sums read together)
#pragma unroll
    for (int g = 0; g < 16; ++g) bef[g] = S.cb[64 * w + 4 * g + rw];
#pragma unroll 4
    for (int g = 0; g < 16; ++g) {
      const int j = 64 * w + 4 * g + rw, x = kFxC * j + 4 * c16;
      if (64 * w + 4 * g >= nch) break;  // (wave-uniform)
      float b[4] = {0.0f, 0.0f, 0.0f, 0.0f}, t[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (x < n) T.at4(x, b, t);
      const float before = bef[g];
      const int E = domain_of(before);
      int d = 0;
      bool tie = false;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bool tx;
        const float r = units_of(fabsf(t[q]), E, &tx);
        d += (int)fminf(r, (float)(kK24 + 1));
        tie = tie || tx;
      }
      d = row_total_i(d);  // (<= 64 (2^24 + 1) < 2^31)
      const bool rtie = ((__ballot(tie) >> (16 * rw)) & 0xffffull) != 0ull;
      // a chunk of +0 terms (|t|: every term +-0) leaves any state as it is
      const bool zero = __ballot(t[0] != 0.0f || t[1] != 0.0f || t[2] != 0.0f || t[3] != 0.0f) >>
                            (16 * rw) & 0xffffull ? false : true;
      uint32_t e = kNoEntry;
      if (!rtie && d < kK24 && E <= 127) e = ((uint32_t)(E + 128) << 24) | (uint32_t)d;
      const float pu = ldexpf(before, 23 - E);  // the running sum in units of E
      const bool pred = j < nch && (j == 0 || (!zero && (e == kNoEntry ||
                        pu + (float)d >= (float)kK24 * (1.0f - 0x1p-12f) ||
                        pu < (float)(1 << 23) * (1.0f + 0x1p-10f))));
      if (zero) e = kFxZero;
      if (c16 == 15 && j < nch) S.e[j] = e;
      // (d, E, before are the row's in its lane 15: pred is read there)
      const uint64_t pm = __ballot(c16 == 15 && pred);
      if (pm) {  // a predicted fallback in this wave's 4 chunks: stash its |terms|
        int sl = -1;
        if (c16 == 15 && pred) {
          sl = atomicAdd(&S.nst, 1);
          if (sl >= kFxStash) sl = -1;
        }
        sl = __shfl(sl, lane | 15);
        if (sl >= 0)
          *reinterpret_cast<f4a*>(&S.st[sl][4 * c16]) =
              f4a{fabsf(t[0]), fabsf(t[1]), fabsf(t[2]), fabsf(t[3])};
        if (c16 == 15 && j < nch) S.slot[j] = sl;
      } else if (c16 == 15 && j < nch) {
        S.slot[j] = -1;
      }
    }
  }
  __syncthreads();
  fx_stamp(a, 3);
  // D: wave 0 walks the entries, 4 per lane (256 per step)
  if (w == 0) {
    float res;
    if (seq_all) {
      // mixed signs or a non-finite term: the reference's chain itself, the
      // next chunk's terms loaded while this one's are added
      float s = 0.0f;
      float tn = T.at(lane);
      for (int j = 0; j < nch; ++j) {
        const float tl = tn;
        if (j + 1 < nch) tn = T.at(kFxC * (j + 1) + lane);
        if (RUN && lane == 0) S.start[j] = s;
#pragma unroll 8
        for (int q = 0; q < kFxC; ++q) s = s + rdl(tl, q);
      }
      res = s;
    } else {
      const bool neg = (f & kNeg) && !(f & kPos);
      int E = kEMin, k = 0, j = 0;
      unsigned n_it = 0, n_fb = 0, n_miss = 0;
      unsigned long long cy_step = 0, cy_fb = 0;  // (diagnostics: shader clocks)
      while (j < nch) {
        ++n_it;
        const unsigned long long c0 = a.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
        // (branch-free: the 4 LDS reads go out together, one wait)
        uint32_t ev[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) ev[q] = S.e[min(j + 4 * lane + q, nch - 1)];
        int dq[4];
        bool vq[4];
        int tot = 0;
        const uint32_t ebias = (uint32_t)(E + 128);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t e = ev[q];
          const bool in = j + 4 * lane + q < nch;
          const bool z = e == kFxZero;
          vq[q] = in & (z | ((e != kNoEntry) & (((e >> 24) == ebias) |
                                                (((e & 0xffffffu) == 0u) & ((e >> 24) < ebias)))));
          dq[q] = (vq[q] & !z) ? (int)(e & 0xffffffu) : 0;
          tot += dq[q];
        }
        tot = min(tot, kK24 + 1);  // (anything above 2^24 fails anyway; no scan overflow)
        const int excl = wave_incl_scan(tot, lane) - tot;
        // the lane's entries in order: each applies until the first that does
        // not (its binade is not the state's, or past 2^(E+1))
        int run = k + excl, fq = 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool stop = fq == 4 && (!vq[q] || run + dq[q] > kK24);
          fq = stop ? q : fq;
          run = fq == 4 ? run + dq[q] : run;
        }
        const uint64_t failm = __ballot(fq < 4);
        const int L = failm ? __builtin_ctzll(failm) : 64;
        if (RUN && lane <= L) {
          int r2 = k + excl;
          const int lim = lane < L ? 4 : fq;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = j + 4 * lane + q;
            if (q < lim && m < nch) S.start[m] = value_of(E, r2);
            r2 += dq[q];
          }
        }
        const int fc = L < 64 ? 4 * L + rdl(fq, L) : 256;
        k = rdl(run, L < 64 ? L : 63);
        normalise(&E, &k);
        j += fc;
        const unsigned long long c1 = a.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
        cy_step += c1 - c0;
        if (j < nch && L < 64) {
          // chunk j term by term, one fp32 add per term: lane 0 runs the
          // chain on VGPR operands (~7 cycles an add; through readlane /
          // SGPR operands it was ~45), from the stash or the terms formed again
          const int sl = S.slot[j];
          ++n_fb;
          n_miss += sl < 0;
          float s = value_of(E, k);
          if (RUN && lane == 0) S.start[j] = s;
          if (lane == 0) {
#pragma unroll
            for (int h = 0; h < kFxC / 16; ++h) {
              float v[16];
              if (sl >= 0) {
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                  const f4a u = *reinterpret_cast<const f4a*>(&S.st[sl][16 * h + 4 * q4]);
                  v[4 * q4] = u[0];
                  v[4 * q4 + 1] = u[1];
                  v[4 * q4 + 2] = u[2];
                  v[4 * q4 + 3] = u[3];
                }
              } else {
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                  float b[4], t[4];
                  T.at4(kFxC * j + 16 * h + 4 * q4, b, t);
#pragma unroll
                  for (int q = 0; q < 4; ++q) v[4 * q4 + q] = fabsf(t[q]);
                }
              }
#pragma unroll
              for (int q = 0; q < 16; ++q) s = s + v[q];
            }
          }
          s = rdl(s, 0);
          state_of(s, &E, &k);
          normalise(&E, &k);
          ++j;
          if (a.stamps) cy_fb += __builtin_amdgcn_s_memtime() - c1;
        }
      }
      const float r = value_of(E, k);
      res = neg ? (r == 0.0f ? 0.0f : -r) : r;
      if (a.stamps && lane == 0 && !RUN) {  // the clocks of the steps and the fallbacks
        a.stamps[8 * (long long)blockIdx.x + 5] = cy_step;
        a.stamps[8 * (long long)blockIdx.x + 6] = cy_fb;
      }
      if (a.stamps && lane == 0)  // diagnostics: walk steps, fallback chunks, stash misses, predicted
        a.stamps[8 * (long long)blockIdx.x + 7] =
            (unsigned long long)min(n_it, 1023u) | ((unsigned long long)min(n_fb, 1023u) << 10) |
            ((unsigned long long)min(n_miss, 1023u) << 20) |
            ((unsigned long long)min(S.nst, 1023) << 30);
    }
    if (lane == 0) S.res = res;
  }
  __syncthreads();
  fx_stamp(a, 4);
}

// One chain per workgroup: out[id * ldo + i].
template <int SRC, int K>
__global__ __launch_bounds__(kFxThreads) void k_fx_chain(FxArgs a) {
  constexpr int KC = K > 0 ? K : 1;
  __shared__ FxShared S;
  const int g = blockIdx.x / KC, i = blockIdx.x % KC;
  int id;
  if (!fx_group(a, g, &id)) return;  // (workgroup-uniform)
  FxTerms<SRC, K> T;
  T.init(a, id, i);
  uint32_t f;
  fx_walk<SRC, K, false>(a, T, S, &f, id, i);
  if (threadIdx.x == 0) a.out[(long long)id * a.ldo + i] = S.res;
}

// The expanded belief's cdf (std::partial_sum, search_tree_cuda.cu:176-183)
// and forwardSampling's 9 x N draws from it (:311-366), as k_fc_* + k_fc_cdf +
// k_tree_sample do in four launches: out[0] = the row's sum, cdf[x] every
// running sum, then counts[a * 16 + z] and the kept children z * 9 + a in
// std::set order (klist, *kcount).  The running sums: each wave takes its
// chunks 16 at a time through a wave-private LDS tile (coalesced loads in,
// lane c < 16 runs chunk c's 64 adds from its exact start value, coalesced
// stores out).  The state of a draw is the first x with cdf[x] >= r: on a
// non-decreasing cdf (no negative or non-finite cell) the first 16 cells
// whose last running sum reaches r (a search in LDS), then the first such
// cell among them; else the plain binary search.
constexpr int kFxTileLd = kFxC + 4;  // (a padded tile row: lanes 0..15 on distinct banks)
__global__ __launch_bounds__(kFxThreads) void k_fx_cdf_sample(FxArgs a, SampleArgs s) {
  __shared__ FxShared S;
  __shared__ int cnt[144];
  __shared__ float sub[kFxThreads * kFxC / 16];  // the last running sum of every 16 cells
  __shared__ __attribute__((aligned(16))) float tile[16][16 * kFxTileLd];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int q = tid; q < 144; q += kFxThreads) cnt[q] = 0;
  FxTerms<FX_ROW, 0> T;
  T.init(a, a.g0, 0);
  uint32_t f;
  fx_walk<FX_ROW, 0, true>(a, T, S, &f, a.g0, 0);
  const int n = a.n, nch = (n + kFxC - 1) / kFxC;
  const bool seq_all = (f & kBad) || ((f & kPos) && (f & kNeg));
  const bool neg = (f & kNeg) && !(f & kPos);
  float* tl = tile[w];
  for (int r16 = 0; r16 < 4; ++r16) {
    const int j0 = 64 * w + 16 * r16;  // this round's 16 chunks = 1024 cells from x0
    if (j0 >= nch) break;  // (wave-uniform)
    const int x0 = kFxC * j0;
    // in: 4 KB of terms, coalesced (signed after a mixed chain, else |terms|)
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int xl = 256 * q4 + 4 * lane;  // cell within the round
      float b[4] = {0.0f, 0.0f, 0.0f, 0.0f}, t[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (x0 + xl < n) T.at4(x0 + xl, b, t);
      const int c = xl / kFxC, o = xl % kFxC;
      *reinterpret_cast<f4a*>(&tl[c * kFxTileLd + o]) =
          seq_all ? f4a{t[0], t[1], t[2], t[3]}
                  : f4a{fabsf(t[0]), fabsf(t[1]), fabsf(t[2]), fabsf(t[3])};
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // chunk j0 + lane: its 64 running sums in place, from the exact start value
    if (lane < 16 && j0 + lane < nch) {
      float v = S.start[j0 + lane];
      float* row = &tl[lane * kFxTileLd];
#pragma unroll 8
      for (int q = 0; q < kFxC; ++q) {
        v = v + row[q];
        row[q] = seq_all || !neg ? v : (v == 0.0f ? 0.0f : -v);
        if (q % 16 == 15) sub[(x0 + lane * kFxC + q) / 16] = v;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // out: coalesced 16-B stores (cells in [n, ld) get running sums inside the
    // row's zero tail; none past the row stride)
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int xl = 256 * q4 + 4 * lane;
      const int c = xl / kFxC, o = xl % kFxC;
      if (x0 + xl < a.ld)
        *reinterpret_cast<f4a*>(a.cdf + x0 + xl) =
            *reinterpret_cast<const f4a*>(&tl[c * kFxTileLd + o]);
    }
    __builtin_amdgcn_wave_barrier();  // (the tile's next round)
  }
  fx_stamp(a, 5);
  if (tid == 0) a.out[0] = S.res;
  const int N = s.N, W = s.g.width;
  if (N <= 0) return;  // (the running sums only)
  __syncthreads();  // (the cdf: stores of this workgroup, visible to it after the barrier)
  const bool mono = !(f & kNeg) && !(f & kBad);
  const float* __restrict__ cdf = a.cdf;
  for (int jt = tid; jt < 9 * N; jt += kFxThreads) {
    const int act = jt / N, j = jt - act * N;
    const float r = s.r[jt];
    int s1 = n;  // the first x with cdf[x] >= r (n: none)
    if (mono) {
      // the first 16 cells whose last running sum reaches r (LDS), then the
      // first such cell among them
      const int nsub = (n + 15) / 16;
      int lo = 0, hi = nsub;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sub[mid] < r) lo = mid + 1;
        else hi = mid;
      }
      if (lo < nsub) {
        float cv[16];
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const f4a v = *reinterpret_cast<const f4a*>(cdf + 16 * lo + 4 * q4);
#pragma unroll
          for (int q = 0; q < 4; ++q) cv[4 * q4 + q] = v[q];
        }
#pragma unroll
        for (int q = 15; q >= 0; --q)
          if (16 * lo + q < n && cv[q] >= r) s1 = 16 * lo + q;
      }
    } else {
      int lo = 0, hi = n;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] < r) lo = mid + 1;
        else hi = mid;
      }
      s1 = lo;
    }
    if (s1 >= n) {  // the reference runs off its arrays: the last cell with mass
      s1 = n - 1;
      while (s1 > 0 && cdf[s1] == cdf[s1 - 1]) --s1;
    }
    const int y1 = s1 / W, x1 = s1 - y1 * W;
    float td = 0.0f;
    uint32_t s2i = 0;
    bool found = false;
    for (int q = 0; q < 9; ++q) {
      const float tv = s.T.p[(long long)y1 * s.T.rs + (long long)(9 * act + q) * s.T.ps + x1];
      td = q == 0 ? tv : td + tv;
      if (!found && s.u1[j] <= td) {
        s2i = (uint32_t)q;
        found = true;
      }
    }
    uint32_t s2 = (uint32_t)s1 + (s2i / 3 - 1) * (uint32_t)W + (s2i % 3 - 1);
    if (s2 >= (uint32_t)n) s2 = (uint32_t)s1;  // (never with a row-stochastic T)
    const int y2 = (int)(s2 / (uint32_t)W), x2 = (int)(s2 - (uint32_t)y2 * (uint32_t)W);
    float ld = 0.0f;
    int o = 0;
    found = false;
    for (int q = 0; q < 16; ++q) {
      const float lv = s.L.p[(long long)y2 * s.L.rs + (long long)q * s.L.ps + x2];
      ld = q == 0 ? lv : ld + lv;
      if (!found && s.u2[j] <= ld) {
        o = q;
        found = true;
      }
    }
    atomicAdd(&cnt[act * 16 + o], 1);
  }
  __syncthreads();
  fx_stamp(a, 6);
  if (tid == 0) {
    int m = 0;
    for (int act = 0; act < 9; ++act)
      for (int z = 0; z < 16; ++z)
        if (cnt[act * 16 + z]) s.klist[m++] = z * 9 + act;
    *s.kcount = m;
  }
  for (int q = tid; q < 144; q += kFxThreads) s.counts[q] = cnt[q];
}

// ---------------------------------------------------------------- PBVI candidates
// evaluatePbviCpu (point_based_value_iteration_cuda.cu:678-699) wants the
// first maximum over S x-ordered fp32 chains per row.  Most alphas cannot be
// it: with D_i an approximate dot (the split-x f32 MFMA GEMM: fmaf chains of
// kchunk terms, then the split partials in order) and E_i the reference's
// chain, |E_i - D_i| <= c * P_i + n * 2^-148, c = (n + kchunk + splits + 8) u
// (u = 2^-24, recursive-summation bounds of both sums in any order, plus the
// products' rounding), P_i = sum_x |b_x alpha_i[x]| -- |D_i| (1 + 2c) when
// every term has one sign (b >= 0, alpha_i single-signed), else
// ||b||_1 max_x |alpha_i[x]|.  Alpha i is a candidate when its upper bound
// D_i + d_i reaches the largest lower bound max_j (D_j - d_j): every other
// alpha's chain lies strictly below the maximum's, so it can be neither the
// maximum nor tie it.  The candidates' chains run exactly (FC_LIST); the
// others' entries are -inf.  A row with a non-finite entry or dot takes
// every alpha as a candidate.

// per alpha i < S: max_x |alpha_i[x]| (x < n) and its sign / finiteness flags
__global__ __launch_bounds__(256) void k_alpha_stats(const float* __restrict__ al, int S, int n,
                                                     int ld, float* __restrict__ amax,
                                                     uint32_t* __restrict__ aflag) {
  __shared__ float sM[4];
  __shared__ uint32_t sF[4];
  const int i = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float* __restrict__ p = al + (long long)i * ld;
  float m = 0.0f;
  uint32_t f = 0u;
  for (int x = threadIdx.x; x < n; x += 256) {
    const float v = p[x];
    f |= !isfinite(v) ? kBad : v > 0.0f ? kPos : v < 0.0f ? kNeg : 0u;
    m = fmaxf(m, fabsf(v));
  }
  for (int o = 32; o > 0; o >>= 1) {
    m = fmaxf(m, __shfl_xor(m, o));
    f |= (uint32_t)__shfl_xor((int)f, o);
  }
  if (lane == 0) {
    sM[w] = m;
    sF[w] = f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    amax[i] = fmaxf(fmaxf(sM[0], sM[1]), fmaxf(sM[2], sM[3]));
    aflag[i] = sF[0] | sF[1] | sF[2] | sF[3];
  }
}

__device__ __forceinline__ double block_max_d(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ double block_sum_d(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

// one block per row q < *kcount (klist[q], or q): candidates of the row
__global__ __launch_bounds__(256) void k_pbvi_cands(PbviCandArgs c) {
  __shared__ double red[4];
  const int q = blockIdx.x;
  if (c.kcount ? q >= *c.kcount : q >= c.nrows) return;
  const int r = c.klist ? c.klist[q] : q;
  const float* __restrict__ b = c.rows + (long long)r * c.row_stride;
  double l1 = 0.0;
  int neg = 0, bad = 0;
  for (int x = threadIdx.x; x < c.n; x += 256) {
    const float v = b[x];
    bad |= !isfinite(v);
    neg |= v < 0.0f;
    l1 += fabs((double)v);
  }
  l1 = block_sum_d(l1, red);
  const int rneg = __syncthreads_or(neg), rbad = __syncthreads_or(bad);
  const double cr = (double)c.c_rel, tiny = (double)c.n * 0x1p-148;
  const float* __restrict__ D = c.approx + (long long)r * c.lda;
  double lo = -INFINITY;
  int dbad = 0;
  for (int i = threadIdx.x; i < c.S; i += 256) {
    const double d = (double)D[i];
    if (!isfinite(d)) {
      dbad = 1;
      continue;
    }
    const uint32_t f = c.aflag[i];
    const bool single = !rneg && !(f & kBad) && !((f & kPos) && (f & kNeg));
    const double P = single ? fabs(d) * (1.0 + 2.0 * cr) : l1 * (double)c.amax[i] * (1.0 + 1e-6);
    lo = fmax(lo, d - (cr * P + tiny));
  }
  lo = block_max_d(lo, red);
  const bool all = rbad || __syncthreads_or(dbad);
  for (int i = threadIdx.x; i < c.S; i += 256) {
    bool cand = all;
    if (!cand) {
      const double d = (double)D[i];
      const uint32_t f = c.aflag[i];
      const bool single = !rneg && !(f & kBad) && !((f & kPos) && (f & kNeg));
      const double P = single ? fabs(d) * (1.0 + 2.0 * cr) : l1 * (double)c.amax[i] * (1.0 + 1e-6);
      cand = d + (cr * P + tiny) >= lo;
    }
    if (cand) {
      const int k = atomicAdd(c.pcount, 1);
      c.plist[k] = make_int2(r, i);
    } else {
      c.exact[(long long)r * c.lde + i] = -INFINITY;
    }
  }
}

// The kernels walk their groups (drive: chains) in grid strides: the grids
// are capped, so that a large device-counted set (FC_LIST: up to 144 x S
// chains, most of them beyond the count) neither overflows a grid dimension
// nor dispatches a workgroup per inactive group.
constexpr int kFcGroupBlocks = 16384;  // sums / tables: segments x groups per launch
constexpr int kFcDriveBlocks = 8192;   // drive: one wave per chain
constexpr int kFcDevGroups = 64;       // groups dispatched for a device group count (gcount)

// k_fc_walk for chains of at most kWkEntries chunks (PP2_FC_WALK=0, or
// pp2_debug_fc_walk(0): k_fc_drive everywhere)
int g_fc_walk = -1;
// k_fc_sumtab for sums + tables (opt-in, PP2_FC_SUMTAB=1: on the 256^2
// plan step the children's set took 41 us in it against 11 + 19 in the two
// launches -- workgroups spinning on their predecessors' totals hold slots
// the later segments' need); its launch tags, unique over the process
// (stale totals never match)
int g_fc_sumtab = -1;
bool fc_sumtab_enabled() {
  if (g_fc_sumtab < 0)
    g_fc_sumtab = getenv("PP2_FC_SUMTAB") && getenv("PP2_FC_SUMTAB")[0] == '1';
  return g_fc_sumtab != 0;
}
int g_fc_k9wave = -1;  // (PP2_FC_K9WAVE=1: every K = 9 set a wave per chain)
bool fc_k9wave_enabled() {
  if (g_fc_k9wave < 0) g_fc_k9wave = getenv("PP2_FC_K9WAVE") && getenv("PP2_FC_K9WAVE")[0] == '1';
  return g_fc_k9wave != 0;
}
int g_fc_kept_gy = -2;
int fc_kept_gy() {
  if (g_fc_kept_gy == -2) {
    const char* e = getenv("PP2_FC_KEPT_GY");
    g_fc_kept_gy = e ? atoi(e) : 0;
  }
  return g_fc_kept_gy;
}
int g_fc_plan9 = -1;
bool fc_plan9_enabled() {
  if (g_fc_plan9 < 0) g_fc_plan9 = getenv("PP2_FC_PLAN9") && getenv("PP2_FC_PLAN9")[0] == '1';
  return g_fc_plan9 != 0;
}
std::atomic<unsigned> g_epoch{0};
unsigned next_epoch() { return ++g_epoch; }
// pp2_debug_fc_stats: driver counters per set kind (8 ints each, summed over
// launches; nullptr: off)
int* g_fc_stats = nullptr;
bool fc_walk_enabled() {
  if (g_fc_walk < 0) g_fc_walk = !(getenv("PP2_FC_WALK") && getenv("PP2_FC_WALK")[0] == '0');
  return g_fc_walk != 0;
}

template <int BASE, int K>
hipError_t launch_set(hipStream_t st, int groups, const FcArgs& a0, int phases) {
  constexpr int KC = K > 0 ? K : 1;
  FcArgs a = a0;
  a.ngroups = groups;
  // (K = 9 crossing plans: PP2_FC_PLAN9=1 -- tabled by k_fc_tables9, a wave
  // per chain)
  if (K > 0 && !fc_plan9_enabled()) a.plan = nullptr;
  const int nseg = fc_segments(a.n);
  if (g_fc_stats && !a.stats) a.stats = g_fc_stats + 32 * (2 * BASE + (K > 0));
  if (BASE == FC_KEPT) a.by_id = 1;
  // a device group list (the kept children: ~40 of 144 on the 256^2 plan
  // step) -- workgroups for 64 groups, looping over more: dispatching the
  // 144-group grid's idle workgroups costs the dispatcher several us
  const int gdisp = a.glist && a.gcount ? std::min(groups, kFcDevGroups) : groups;
  int gy = std::min(gdisp, std::max(1, kFcGroupBlocks / nseg));
  const bool sums = phases & (FC_TABLES | FC_SUMS), tabs = phases & (FC_TABLES | FC_TAB);
  // (PP2_FC_KEPT_GY: the kept children's tables over fewer workgroup rows,
  // each looping over several children with its partner quads loaded once)
  if (BASE == FC_KEPT && tabs && !sums && fc_kept_gy() > 0) gy = std::min(gy, fc_kept_gy());
  if (sums && tabs && a.agg && fc_sumtab_enabled()) {
    a.epoch = next_epoch();
    hipLaunchKernelGGL((k_fc_sumtab<BASE, K>), dim3(nseg, gy), dim3(256), 0, st, a);
  } else {
    // (a wave per chain for one-group K = 9 sets, whose tables are latency:
    // the 9 rewards' 12 -> 8 us; with many groups the 9 waves' repeated base
    // values cost more -- the kept children's FIB sets: 31 -> 47 us)
    // (kept_unit sums: k_fc_sums, whose flags come from the cells' and
    // partners' signs)
    if (K == 9 && ((groups == 1 && !a.gcount) || fc_k9wave_enabled()) &&
        !(BASE == FC_KEPT && a.kept_unit && sums)) {
      if (sums) hipLaunchKernelGGL((k_fc_sums9<BASE>), dim3(nseg, gy), dim3(576), 0, st, a);
      if (tabs) hipLaunchKernelGGL((k_fc_tables9<BASE>), dim3(nseg, gy), dim3(576), 0, st, a);
    } else {
      if (sums) hipLaunchKernelGGL((k_fc_sums<BASE, K>), dim3(nseg, gy), dim3(256), 0, st, a);
      if (tabs) hipLaunchKernelGGL((k_fc_tables<BASE, K>), dim3(nseg, gy), dim3(256), 0, st, a);
    }
  }
  if (phases & FC_DRIVE) {
    if constexpr (BASE == FC_KEPT) {
      // the dots of the normalised rows the tables stored: FC_ROW chains
      FcArgs w = a;
      w.row = a.kept_rows;
      w.row_stride = a.ld;
      return launch_set<FC_ROW, K>(st, groups, w, FC_DRIVE);
    } else {
      if (fc_walk_enabled() && fc_chunks(a.n) <= kWkEntries)
        hipLaunchKernelGGL((k_fc_walk<BASE, K>), dim3(std::min(gdisp * KC, kFcDriveBlocks)),
                           dim3(64), 0, st, a);
      else
        hipLaunchKernelGGL((k_fc_drive<BASE, K>), dim3(std::min(gdisp * KC, kFcDriveBlocks)),
                           dim3(64), 0, st, a);
      if (BASE == FC_ROW && K == 0 && a.cdf)
        hipLaunchKernelGGL(k_fc_cdf, dim3((fc_chunks(a.n) + 3) / 4), dim3(256), 0, st, a);
    }
  }
  return hipGetLastError();
}

}  // namespace

bool fc_sumtab_active() { return fc_sumtab_enabled(); }

hipError_t launch_fchain(hipStream_t st, int base, int K, int groups, const FcArgs& a,
                         int phases) {
  if (groups <= 0) return hipSuccess;
  const int kc = K > 0 ? K : 1;
  if (a.n <= 0 || a.n > kFcMaxCells || (K != 0 && K != 9) || !a.out || !a.csum || !a.cflag ||
      !a.tab || (base == FC_KEPT || a.by_id ? 144 : groups) * kc > a.max_chains ||
      fc_chunks(a.n) > a.max_chunks)
    return hipErrorInvalidValue;
  if (base == FC_KEPT) {
    if (K != 9 || !a.pred || !a.lrows || a.row || a.cdf || groups > 144 ||
        (!a.glist && a.g0 + groups > 144))
      return hipErrorInvalidValue;
    if ((phases & (FC_TABLES | FC_SUMS)) && !a.mass && !a.msum && !a.kept_unit)
      return hipErrorInvalidValue;
    // (kept_unit: the sums pass alone -- a fused sums + tables launch would
    // table the unnormalised cells)
    if (a.kept_unit && (phases & FC_TABLES)) return hipErrorInvalidValue;
    if ((phases & (FC_TABLES | FC_TAB | FC_DRIVE)) && (!a.mass || !a.kept_rows))
      return hipErrorInvalidValue;
  }
  if (a.ld < a.n || a.ld % 4 != 0) return hipErrorInvalidValue;
  if (base == FC_CHILD && (!a.pred || !a.lrows || K != 0)) return hipErrorInvalidValue;
  if (base == FC_ROW && !a.row) return hipErrorInvalidValue;
  if (base == FC_LIST && (K != 0 || !a.row || !a.partners || !a.plist || !a.gcount || a.glist ||
                          a.cdf))
    return hipErrorInvalidValue;
  if (base != FC_LIST && a.plist) return hipErrorInvalidValue;
  if (K != 0 && !a.partners) return hipErrorInvalidValue;
  if (a.cdf && (base != FC_ROW || K != 0 || groups != 1 || !a.cst)) return hipErrorInvalidValue;
  if (base == FC_ROW && K == 0) return launch_set<FC_ROW, 0>(st, groups, a, phases);
  if (base == FC_ROW && K == 9) return launch_set<FC_ROW, 9>(st, groups, a, phases);
  if (base == FC_ROW) return hipErrorInvalidValue;
  if (base == FC_CHILD) return launch_set<FC_CHILD, 0>(st, groups, a, phases);
  if (base == FC_LIST) return launch_set<FC_LIST, 0>(st, groups, a, phases);
  if (base == FC_KEPT) return launch_set<FC_KEPT, 9>(st, groups, a, phases);
  return hipErrorInvalidValue;
}

namespace {
template <int SRC, int K>
hipError_t launch_fx_set(hipStream_t st, int groups, const FxArgs& a0) {
  constexpr int KC = K > 0 ? K : 1;
  FxArgs a = a0;
  a.ngroups = groups;
  hipLaunchKernelGGL((k_fx_chain<SRC, K>), dim3((unsigned)(groups * KC)), dim3(kFxThreads), 0, st,
                     a);
  return hipGetLastError();
}
}  // namespace

bool fx_fits(int n, int ld) { return n > 0 && n <= kFxC * kFxThreads && ld >= n && ld % 64 == 0; }

hipError_t launch_fx(hipStream_t st, int base, int K, int groups, const FxArgs& a) {
  if (groups <= 0) return hipSuccess;
  if (!fx_fits(a.n, a.ld) || (K != 0 && K != 9) || !a.out || groups * (K > 0 ? K : 1) > 65535)
    return hipErrorInvalidValue;
  if (K != 0 && !a.partners) return hipErrorInvalidValue;
  if (base == FX_ROW && !a.row) return hipErrorInvalidValue;
  if (base != FX_ROW && (!a.pred || !a.lrows)) return hipErrorInvalidValue;
  if (base == FX_KEPT && (!a.sums || K != 9)) return hipErrorInvalidValue;
  if (base == FX_CHILD && K != 0) return hipErrorInvalidValue;
  if ((base == FX_CHILD || base == FX_KEPT) && !a.glist && a.g0 + groups > 144)
    return hipErrorInvalidValue;
  if (base == FX_ROW && K == 0) return launch_fx_set<FX_ROW, 0>(st, groups, a);
  if (base == FX_ROW && K == 9) return launch_fx_set<FX_ROW, 9>(st, groups, a);
  if (base == FX_CHILD) return launch_fx_set<FX_CHILD, 0>(st, groups, a);
  if (base == FX_KEPT) return launch_fx_set<FX_KEPT, 9>(st, groups, a);
  return hipErrorInvalidValue;
}

hipError_t launch_fx_cdf_sample(hipStream_t st, const FxArgs& a0, const SampleArgs& s) {
  if (!fx_fits(a0.n, a0.ld) || !a0.row || !a0.cdf || !a0.out || s.N < 0 || 9 * s.N > (1 << 20))
    return hipErrorInvalidValue;
  if (s.N > 0 && (s.n != a0.n || !s.r || !s.u1 || !s.u2 || !s.counts || !s.klist || !s.kcount ||
                  !s.T.p || !s.L.p || (long long)s.g.rows * s.g.width != a0.n))
    return hipErrorInvalidValue;
  FxArgs a = a0;
  a.ngroups = 1;
  a.glist = nullptr;
  a.gcount = nullptr;
  hipLaunchKernelGGL(k_fx_cdf_sample, dim3(1), dim3(kFxThreads), 0, st, a, s);
  return hipGetLastError();
}

hipError_t launch_alpha_stats(hipStream_t st, const float* al, int S, int n, int ld, float* amax,
                              uint32_t* aflag) {
  if (S <= 0 || n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_alpha_stats, dim3(S), dim3(256), 0, st, al, S, n, ld, amax, aflag);
  return hipGetLastError();
}

hipError_t launch_pbvi_cands(hipStream_t st, const PbviCandArgs& c) {
  if (c.nrows <= 0) return hipSuccess;
  if (!c.rows || !c.approx || !c.amax || !c.aflag || !c.exact || !c.plist || !c.pcount ||
      c.S <= 0 || c.n <= 0 || (c.klist == nullptr) != (c.kcount == nullptr))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_pbvi_cands, dim3(c.nrows), dim3(256), 0, st, c);
  return hipGetLastError();
}

hipError_t launch_tree_sample(hipStream_t st, const SampleArgs& s) {
  if (s.N <= 0 || s.n <= 0 || !s.cdf || !s.r || !s.u1 || !s.u2 || !s.counts || !s.klist ||
      !s.kcount)
    return hipErrorInvalidValue;
  if (!s.rows != !s.rows_out) return hipErrorInvalidValue;
  FcRowTable t;
  if (s.rows) t = *s.rows;
  hipLaunchKernelGGL(k_tree_sample, dim3(1), dim3(1024), 0, st, s, t);
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

hipError_t launch_store_kept(hipStream_t st, const int* klist, const int* kcount,
                             const float* pred, const float* lrows, const float* sums, float* dst,
                             int n, int ld, const FcRowTable* rows) {
  if (n <= 0) return hipSuccess;
  FcRowTable t;
  if (rows) t = *rows;
  hipLaunchKernelGGL(k_store_kept, dim3((n + 255) / 256, 144), dim3(256), 0, st, klist, kcount,
                     pred, lrows, sums, dst, n, ld, t);
  return hipGetLastError();
}

hipError_t launch_fib_cands(hipStream_t st, const FcArgs& a, uint16_t* cmask) {
  if (!cmask || !a.glist || !a.gcount || !a.csum || !a.cflag || !a.out || !a.mass ||
      (!a.msum && !a.kept_unit) || a.n <= 0)
    return hipErrorInvalidValue;
  FcArgs b = a;
  b.ngroups = 144;  // (the kept children: at most 144, gcount of them)
  hipLaunchKernelGGL(k_fib_cands, dim3(kFcDevGroups), dim3(64), 0, st, b, cmask);
  return hipGetLastError();
}

hipError_t launch_copy_kept(hipStream_t st, const int* klist, const int* kcount, const float* src,
                            int n, int ld, const FcRowTable* rows) {
  if (n <= 0) return hipSuccess;
  if (!rows || ld % 4 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_copy_kept, dim3((n + 1023) / 1024, 144), dim3(256), 0, st, klist, kcount,
                     src, n, ld, *rows);
  return hipGetLastError();
}

void FcScratch::release() {
  for (void* p : {(void*)csum, (void*)cflag, (void*)tab, (void*)cst, (void*)plan, (void*)agg})
    if (p) (void)hipFree(p);
  agg = nullptr;
  csum = nullptr;
  cflag = nullptr;
  tab = nullptr;
  cst = nullptr;
  plan = nullptr;
  chains = 0;
  chunks = 0;
}

bool FcScratch::reserve(int n, int max_chains) {
  release();
  const size_t nch = (size_t)fc_chunks(n), nseg = (size_t)fc_segments(n);
  const size_t mc = (size_t)(max_chains > 0 ? max_chains : 1);
  if (hipMalloc(&csum, mc * nch * sizeof(float)) != hipSuccess ||
      hipMalloc(&cflag, mc * nseg * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc(&tab, mc * nch * sizeof(uint2)) != hipSuccess ||
      hipMalloc(&cst, (nch + 1) * sizeof(int2)) != hipSuccess ||
      hipMalloc(&plan, mc * nch * 2 * sizeof(uint4)) != hipSuccess ||
      hipMalloc(&agg, mc * nseg * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(agg, 0, mc * nseg * sizeof(unsigned long long)) != hipSuccess) {
    release();
    return false;
  }
  chains = max_chains;
  chunks = (int)nch;
  return true;
}

void FcScratch::attach(FcArgs* a) const {
  static const bool plans = !(getenv("PP2_FC_PLAN") && getenv("PP2_FC_PLAN")[0] == '0');
  a->csum = csum;
  a->cflag = cflag;
  a->tab = tab;
  a->cst = cst;
  a->plan = plans ? plan : nullptr;  // (PP2_FC_PLAN=0: no crossing plans, for A/B runs)
  a->agg = agg;
  a->max_chains = chains;
  a->max_chunks = chunks;
}

}  // namespace pp2

// Diagnostic entry point for tests/test_gpu_fchain.py (not part of pp2.h):
// the FC_ROW chains of one host row x[n] on device 0 -- K = 0: out[0] =
// accumulate(x) and, with cdf, every running sum; K = 9: out[i] =
// inner_product(x, partners[i]) (partners: 9 rows of n).  Synchronous.
extern "C" int pp2_debug_fchain_row2(int n, const float* x, const float* partners, int K,
                                     float* out, float* cdf, int* stats, float* ms);
extern "C" int pp2_debug_fchain_row(int n, const float* x, const float* partners, int K,
                                    float* out, float* cdf) {
  return pp2_debug_fchain_row2(n, x, partners, K, out, cdf, nullptr, nullptr);
}
// (stats[8]: the driver's {iterations, fallback chunks, exact rounds, stash
// hits}, summed over its chains, then 100 MHz ticks summed over the chains
// in {flags, first window + stash, the walk} and the chains; ms: the chain
// set's event time, median of 5 runs after a warm-up)
extern "C" int pp2_debug_fchain_row2(int n, const float* x, const float* partners, int K,
                                     float* out, float* cdf, int* stats, float* ms) {
  if (n < 0 || !x || !out || (K != 0 && K != 9) || (K == 9 && !partners) || (cdf && K != 0))
    return 1;
  if (n == 0) {
    for (int i = 0; i < (K ? 9 : 1); ++i) out[i] = 0.0f;
    return 0;
  }
  const size_t ld = ((size_t)n + 63) / 64 * 64;
  float *dx = nullptr, *dp = nullptr, *dout = nullptr, *dcdf = nullptr;
  pp2::FcScratch scr;
  int st = 0;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && st == 0) st = 2;
    return st == 0;
  };
  if (!scr.reserve(n, 9)) return 3;
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
    scr.attach(&a);
    int* dstats = nullptr;
    if (stats && ok(hipMalloc(&dstats, 16 * sizeof(int))) &&
        ok(hipMemset(dstats, 0, 16 * sizeof(int))))
      a.stats = dstats;
    if (ms && st == 0) {
      hipEvent_t e0, e1;
      float t[5];
      if (ok(hipEventCreate(&e0)) && ok(hipEventCreate(&e1))) {
        pp2::FcArgs w = a;
        w.stats = nullptr;
        ok(pp2::launch_fchain(nullptr, pp2::FC_ROW, K, 1, w));
        for (int r = 0; r < 5 && st == 0; ++r) {
          ok(hipEventRecord(e0, nullptr));
          ok(pp2::launch_fchain(nullptr, pp2::FC_ROW, K, 1, w));
          ok(hipEventRecord(e1, nullptr));
          ok(hipEventSynchronize(e1));
          ok(hipEventElapsedTime(&t[r], e0, e1));
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        for (int i = 1; i < 5; ++i)
          for (int j = i; j > 0 && t[j] < t[j - 1]; --j) std::swap(t[j], t[j - 1]);
        *ms = t[2];
      }
    }
    if (ok(pp2::launch_fchain(nullptr, pp2::FC_ROW, K, 1, a)) && ok(hipDeviceSynchronize()) &&
        ok(hipMemcpy(out, dout, (K == 9 ? 9 : 1) * sizeof(float), hipMemcpyDeviceToHost)) && cdf)
      ok(hipMemcpy(cdf, dcdf, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
    if (dstats) {
      if (st == 0) ok(hipMemcpy(stats, dstats, 8 * sizeof(int), hipMemcpyDeviceToHost));
      (void)hipFree(dstats);
    }
  }
  for (float* p : {dx, dp, dout, dcdf})
    if (p) (void)hipFree(p);
  return st;
}

// Diagnostic (tests/tools only): one FC_ROW K = 0 chain set on a host row,
// and its scratch: csum[nch] (k_fc_sums), tab[2 nch] (k_fc_tables: entry,
// flags), cst[2 (nch + 1)] (k_fc_drive's chunk start states).
extern "C" int pp2_debug_fchain_tables(int n, const float* x, float* csum, uint32_t* tab,
                                       int* cst) {
  if (n <= 0 || !x) return 1;
  const size_t ld = ((size_t)n + 63) / 64 * 64, nch = (size_t)pp2::fc_chunks(n);
  float *dx = nullptr, *dout = nullptr, *dcdf = nullptr;
  pp2::FcScratch scr;
  int st = 0;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && st == 0) st = 2;
    return st == 0;
  };
  if (!scr.reserve(n, 1)) return 3;
  if (ok(hipMalloc(&dx, ld * sizeof(float))) && ok(hipMalloc(&dout, 16 * sizeof(float))) &&
      ok(hipMalloc(&dcdf, ld * sizeof(float))) && ok(hipMemset(dx, 0, ld * sizeof(float))) &&
      ok(hipMemcpy(dx, x, (size_t)n * sizeof(float), hipMemcpyHostToDevice))) {
    pp2::FcArgs a;
    a.n = n;
    a.ld = (int)ld;
    a.row = dx;
    a.out = dout;
    a.cdf = dcdf;
    scr.attach(&a);
    if (ok(pp2::launch_fchain(nullptr, pp2::FC_ROW, 0, 1, a)) && ok(hipDeviceSynchronize())) {
      if (csum) ok(hipMemcpy(csum, scr.csum, nch * sizeof(float), hipMemcpyDeviceToHost));
      if (tab) ok(hipMemcpy(tab, scr.tab, nch * sizeof(uint2), hipMemcpyDeviceToHost));
      if (cst) ok(hipMemcpy(cst, scr.cst, (nch + 1) * sizeof(int2), hipMemcpyDeviceToHost));
    }
  }
  for (float* p : {dx, dout, dcdf})
    if (p) (void)hipFree(p);
  return st;
}

// Diagnostic (tests/test_gpu_fchain.py): the FC_LIST chain set of the
// (row, alpha) pairs on device 0 -- out[r * S + i] = inner_product(x[r],
// alphas[i]) for every listed pair (r, i) (other entries of out untouched).
// x: R rows of n, alphas: S rows of n.  Synchronous.
extern "C" int pp2_debug_fchain_pairs(int n, int R, const float* x, int S, const float* alphas,
                                      const int* pairs, int npairs, float* out) {
  if (n <= 0 || R <= 0 || S <= 0 || npairs < 0 || !x || !alphas || !out || (npairs > 0 && !pairs))
    return 1;
  for (int k = 0; k < npairs; ++k)
    if (pairs[2 * k] < 0 || pairs[2 * k] >= R || pairs[2 * k + 1] < 0 || pairs[2 * k + 1] >= S)
      return 1;
  const size_t ld = ((size_t)n + 63) / 64 * 64;
  const int cap = std::max(1, npairs);
  float *dx = nullptr, *da = nullptr, *dout = nullptr;
  int2* dlist = nullptr;
  int* dcnt = nullptr;
  pp2::FcScratch scr;
  int st = 0;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && st == 0) st = 2;
    return st == 0;
  };
  if (!scr.reserve(n, cap)) return 3;
  if (ok(hipMalloc(&dx, (size_t)R * ld * sizeof(float))) &&
      ok(hipMalloc(&da, (size_t)S * ld * sizeof(float))) &&
      ok(hipMalloc(&dout, (size_t)R * S * sizeof(float))) &&
      ok(hipMalloc(&dlist, (size_t)cap * sizeof(int2))) && ok(hipMalloc(&dcnt, sizeof(int))) &&
      ok(hipMemset(dx, 0, (size_t)R * ld * sizeof(float))) &&
      ok(hipMemset(da, 0, (size_t)S * ld * sizeof(float))) &&
      ok(hipMemcpy(dout, out, (size_t)R * S * sizeof(float), hipMemcpyHostToDevice)) &&
      ok(hipMemcpy2D(dx, ld * sizeof(float), x, (size_t)n * sizeof(float), (size_t)n * sizeof(float),
                     R, hipMemcpyHostToDevice)) &&
      ok(hipMemcpy2D(da, ld * sizeof(float), alphas, (size_t)n * sizeof(float),
                     (size_t)n * sizeof(float), S, hipMemcpyHostToDevice)) &&
      (npairs == 0 || ok(hipMemcpy(dlist, pairs, (size_t)npairs * sizeof(int2), hipMemcpyHostToDevice))) &&
      ok(hipMemcpy(dcnt, &npairs, sizeof(int), hipMemcpyHostToDevice))) {
    pp2::FcArgs a;
    a.n = n;
    a.ld = (int)ld;
    a.row = dx;
    a.row_stride = (long long)ld;
    a.partners = da;
    a.plist = dlist;
    a.gcount = dcnt;
    a.out = dout;
    a.ldo = S;
    scr.attach(&a);
    if (ok(pp2::launch_fchain(nullptr, pp2::FC_LIST, 0, cap, a)) && ok(hipDeviceSynchronize()))
      ok(hipMemcpy(out, dout, (size_t)R * S * sizeof(float), hipMemcpyDeviceToHost));
  }
  for (void* p : {(void*)dx, (void*)da, (void*)dout, (void*)dlist, (void*)dcnt})
    if (p) (void)hipFree(p);
  return st;
}

// Diagnostic (tests/test_gpu_fchain.py): the fused chain sets on device 0.
// mode 0: FX_ROW chains of one host row x[n] (K = 0: out[0] and, with cdf,
//   every running sum through k_fx_cdf_sample without draws; K = 9: out[i] =
//   inner_product(x, partners[i])).
// mode 1: the children of 9 prediction rows pred[9][n] and 16 likelihood rows
//   L[16][n]: out[c] = accumulate of child c = z * 9 + a (FX_CHILD, all 144),
//   then for the kcount children klist[] the normalised rows (rows[c][n]) and
//   their 9 dots with partners (out[144 + 9 c + i], FX_KEPT).
// mode 2: as mode 1 through the planner's chain sets instead (pp2_tree.cpp):
//   FC_CHILD tables + drive, then the kept children's FC_KEPT sums, tables,
//   drive; K's bit 0 = kept_unit (the sums over the unnormalised cells), bit
//   1 = the FIB candidate masks (launch_fib_cands: pruned dots are -inf).
// ms (if set): the set's event time, median of 5 runs after a warm-up.  Synchronous.
extern "C" int pp2_debug_fx(int mode, int n, const float* x, const float* partners, int K,
                            const float* pred, const float* lrows, const int* klist, int kcount,
                            float* out, float* cdf, float* rows, float* ms) {
  if (n <= 0 || n > 65536 || (mode != 2 && K != 0 && K != 9) || (mode == 2 && (K < 0 || K > 3)) ||
      !out || (mode == 0 && !x) ||
      (mode >= 1 && (!pred || !lrows || !partners || kcount < 0 || kcount > 144 ||
                     (kcount > 0 && !klist))) ||
      (mode != 0 && mode != 1 && mode != 2) || (K == 9 && !partners && mode == 0))
    return 1;
  pp2::FcScratch sc_child, sc_kept;
  uint16_t* dcm = nullptr;
  if (mode == 2 && (!sc_child.reserve(n, 144) || !sc_kept.reserve(n, 144 * 9) ||
                    hipMalloc(&dcm, 144 * sizeof(uint16_t)) != hipSuccess))
    return 2;
  const size_t ld = ((size_t)n + 63) / 64 * 64;
  float *dx = nullptr, *dp = nullptr, *dout = nullptr, *dcdf = nullptr, *dpred = nullptr,
        *dl = nullptr, *drows = nullptr;
  int* dk = nullptr;
  int st = 0;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && st == 0) st = 2;
    return st == 0;
  };
  auto up = [&](float** d, const float* h, int nrow) {
    return ok(hipMalloc(d, (size_t)nrow * ld * sizeof(float))) &&
           ok(hipMemset(*d, 0, (size_t)nrow * ld * sizeof(float))) &&
           (!h || ok(hipMemcpy2D(*d, ld * sizeof(float), h, (size_t)n * sizeof(float),
                                 (size_t)n * sizeof(float), nrow, hipMemcpyHostToDevice)));
  };
  const int nout = mode == 0 ? 16 : 144 + 144 * 9;
  if (ok(hipMalloc(&dout, nout * sizeof(float))) && ok(hipMemset(dout, 0, nout * sizeof(float))) &&
      (mode != 0 || up(&dx, x, 1)) && (!partners || up(&dp, partners, 9)) &&
      (mode != 0 || !cdf || up(&dcdf, nullptr, 1)) &&
      (mode == 0 || (up(&dpred, pred, 9) && up(&dl, lrows, 16) && up(&drows, nullptr, 144) &&
                     ok(hipMalloc(&dk, 145 * sizeof(int))) &&
                     (kcount == 0 || ok(hipMemcpy(dk, klist, kcount * sizeof(int),
                                                  hipMemcpyHostToDevice))) &&
                     ok(hipMemcpy(dk + 144, &kcount, sizeof(int), hipMemcpyHostToDevice))))) {
    auto run = [&]() -> hipError_t {
      if (mode == 2) {
        pp2::FcArgs ch;
        ch.n = n;
        ch.ld = (int)ld;
        ch.pred = dpred;
        ch.lrows = dl;
        ch.out = dout;
        ch.ldo = 1;
        sc_child.attach(&ch);
        hipError_t e = pp2::launch_fchain(nullptr, pp2::FC_CHILD, 0, 144, ch, pp2::FC_TABLES);
        if (e == hipSuccess) e = pp2::launch_fchain(nullptr, pp2::FC_CHILD, 0, 144, ch, pp2::FC_DRIVE);
        pp2::FcArgs kd;
        kd.n = n;
        kd.ld = (int)ld;
        kd.pred = dpred;
        kd.lrows = dl;
        kd.partners = dp;
        kd.msum = ch.csum;
        kd.out = dout + 144;
        kd.ldo = 9;
        kd.glist = dk;
        kd.gcount = dk + 144;
        kd.kept_unit = K & 1;
        sc_kept.attach(&kd);
        if (e == hipSuccess) e = pp2::launch_fchain(nullptr, pp2::FC_KEPT, 9, 144, kd, pp2::FC_SUMS);
        kd.mass = dout;
        kd.kept_rows = drows;
        if (e == hipSuccess && (K & 2)) {
          e = pp2::launch_fib_cands(nullptr, kd, dcm);
          kd.cmask = dcm;
        }
        if (e == hipSuccess) e = pp2::launch_fchain(nullptr, pp2::FC_KEPT, 9, 144, kd, pp2::FC_TAB);
        if (e == hipSuccess) e = pp2::launch_fchain(nullptr, pp2::FC_KEPT, 9, 144, kd, pp2::FC_DRIVE);
        return e;
      }
      pp2::FxArgs a;
      a.n = n;
      a.ld = (int)ld;
      a.partners = dp;
      a.out = dout;
      if (mode == 0) {
        a.row = dx;
        a.ldo = K == 9 ? 9 : 1;
        if (K == 0 && cdf) {
          a.cdf = dcdf;
          pp2::SampleArgs sa{};
          sa.N = 0;
          return pp2::launch_fx_cdf_sample(nullptr, a, sa);
        }
        return pp2::launch_fx(nullptr, pp2::FX_ROW, K, 1, a);
      }
      a.pred = dpred;
      a.lrows = dl;
      a.ldo = 1;
      hipError_t e = pp2::launch_fx(nullptr, pp2::FX_CHILD, 0, 144, a);
      if (e != hipSuccess) return e;
      pp2::FxArgs b = a;
      b.sums = dout;
      b.out = dout + 144;
      b.ldo = 9;
      b.glist = dk;
      b.gcount = dk + 144;
      b.rows_out = drows;
      return pp2::launch_fx(nullptr, pp2::FX_KEPT, 9, 144, b);
    };
    if (ms && st == 0) {
      hipEvent_t e0, e1;
      float t[5];
      if (ok(hipEventCreate(&e0)) && ok(hipEventCreate(&e1))) {
        ok(run());
        for (int r = 0; r < 5 && st == 0; ++r) {
          ok(hipEventRecord(e0, nullptr));
          ok(run());
          ok(hipEventRecord(e1, nullptr));
          ok(hipEventSynchronize(e1));
          ok(hipEventElapsedTime(&t[r], e0, e1));
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        for (int i = 1; i < 5; ++i)
          for (int j = i; j > 0 && t[j] < t[j - 1]; --j) std::swap(t[j], t[j - 1]);
        *ms = t[2];
      }
    }
    if (st == 0) ok(hipMemset(dout, 0, nout * sizeof(float)));
    if (ok(run()) && ok(hipDeviceSynchronize()) &&
        ok(hipMemcpy(out, dout, nout * sizeof(float), hipMemcpyDeviceToHost))) {
      if (cdf && dcdf) ok(hipMemcpy(cdf, dcdf, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
      if (rows && drows)
        ok(hipMemcpy2D(rows, (size_t)n * sizeof(float), drows, ld * sizeof(float),
                       (size_t)n * sizeof(float), 144, hipMemcpyDeviceToHost));
    }
  }
  for (void* p : {(void*)dx, (void*)dp, (void*)dout, (void*)dcdf, (void*)dpred, (void*)dl,
                  (void*)drows, (void*)dk, (void*)dcm})
    if (p) (void)hipFree(p);
  return st;
}

// Diagnostic (tests/test_gpu_fchain.py, round-5 ADVICE): the planner's PBVI
// candidate filter as ref_pbvi_bounds runs it (pp2_tree.cpp, PP2_PBVI_FCHAIN=1)
// on host rows x[R][n] and alphas[S][n]: the split-x MFMA GEMM's approximate
// dots, k_pbvi_cands with the bound priced from gemm_kchunk, the candidates'
// exact chains (FC_LIST), the first argmax per row -> idx[r], val[r];
// *ncand = the candidates kept.  Synchronous, device 0.
extern "C" int pp2_debug_pbvi_cands(int n, int R, const float* x, int S, const float* alphas,
                                    int ksplit, int* idx, float* val, int* ncand) {
  if (n <= 0 || R <= 0 || R > 256 || S <= 0 || !x || !alphas || !idx || !val || ksplit < 1)
    return 1;
  const int ld = (n + pp2::kPbviChunk - 1) / pp2::kPbviChunk * pp2::kPbviChunk;
  const int Mp = (R + pp2::kGemmTile - 1) / pp2::kGemmTile * pp2::kGemmTile;
  const int Sp = (S + pp2::kGemmTile - 1) / pp2::kGemmTile * pp2::kGemmTile;
  const long long sstride = (long long)Mp * Sp;
  float *dx = nullptr, *da = nullptr, *dpart = nullptr, *dapprox = nullptr, *damax = nullptr,
        *dexact = nullptr, *dv = nullptr;
  uint32_t* dflag = nullptr;
  int2* dlist = nullptr;
  int *dcnt = nullptr, *didx = nullptr;
  pp2::FcScratch scr;
  int st = 0;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && st == 0) st = 2;
    return st == 0;
  };
  if (!scr.reserve(n, R * S)) return 3;
  if (ok(hipMalloc(&dx, (size_t)Mp * ld * sizeof(float))) &&
      ok(hipMalloc(&da, (size_t)Sp * ld * sizeof(float))) &&
      ok(hipMalloc(&dpart, (size_t)ksplit * sstride * sizeof(float))) &&
      ok(hipMalloc(&dapprox, (size_t)sstride * sizeof(float))) &&
      ok(hipMalloc(&damax, (size_t)Sp * sizeof(float))) &&
      ok(hipMalloc(&dflag, (size_t)Sp * sizeof(uint32_t))) &&
      ok(hipMalloc(&dexact, (size_t)R * S * sizeof(float))) &&
      ok(hipMalloc(&dv, (size_t)R * sizeof(float))) &&
      ok(hipMalloc(&didx, (size_t)R * sizeof(int))) &&
      ok(hipMalloc(&dlist, (size_t)R * S * sizeof(int2))) && ok(hipMalloc(&dcnt, sizeof(int))) &&
      ok(hipMemset(dx, 0, (size_t)Mp * ld * sizeof(float))) &&
      ok(hipMemset(da, 0, (size_t)Sp * ld * sizeof(float))) &&
      ok(hipMemset(dcnt, 0, sizeof(int))) &&
      ok(hipMemcpy2D(dx, ld * sizeof(float), x, (size_t)n * sizeof(float), (size_t)n * sizeof(float),
                     R, hipMemcpyHostToDevice)) &&
      ok(hipMemcpy2D(da, ld * sizeof(float), alphas, (size_t)n * sizeof(float),
                     (size_t)n * sizeof(float), S, hipMemcpyHostToDevice)) &&
      ok(pp2::launch_alpha_stats(nullptr, da, S, n, ld, damax, dflag)) &&
      ok(pp2::launch_gemm_nt(nullptr, dx, da, dpart, Mp, Sp, ld, 1, 0, 0, ksplit, sstride)) &&
      ok(pp2::launch_sum_splits(nullptr, dpart, ksplit, sstride, (int)sstride, dapprox))) {
    pp2::PbviCandArgs ca;
    ca.rows = dx;
    ca.row_stride = ld;
    ca.n = n;
    ca.nrows = R;
    ca.approx = dapprox;
    ca.lda = Sp;
    ca.amax = damax;
    ca.aflag = dflag;
    ca.S = S;
    const long long kchunk = pp2::gemm_kchunk(ld, ksplit);
    ca.c_rel = (float)((double)((long long)n + kchunk + ksplit + 8) * 0x1p-24 * 1.01);
    ca.exact = dexact;
    ca.lde = S;
    ca.plist = dlist;
    ca.pcount = dcnt;
    pp2::FcArgs a;
    a.n = n;
    a.ld = ld;
    a.row = dx;
    a.row_stride = ld;
    a.partners = da;
    a.plist = dlist;
    a.gcount = dcnt;
    a.out = dexact;
    a.ldo = S;
    scr.attach(&a);
    if (ok(pp2::launch_pbvi_cands(nullptr, ca)) &&
        ok(pp2::launch_fchain(nullptr, pp2::FC_LIST, 0, R * S, a)) &&
        ok(pp2::launch_argmax_rows(nullptr, dexact, R, S, S, didx, dv)) &&
        ok(hipDeviceSynchronize()) &&
        ok(hipMemcpy(idx, didx, (size_t)R * sizeof(int), hipMemcpyDeviceToHost)) &&
        ok(hipMemcpy(val, dv, (size_t)R * sizeof(float), hipMemcpyDeviceToHost)) && ncand)
      ok(hipMemcpy(ncand, dcnt, sizeof(int), hipMemcpyDeviceToHost));
  }
  for (void* p : {(void*)dx, (void*)da, (void*)dpart, (void*)dapprox, (void*)damax, (void*)dflag,
                  (void*)dexact, (void*)dv, (void*)didx, (void*)dlist, (void*)dcnt})
    if (p) (void)hipFree(p);
  return st;
}

// Diagnostic (tests): choose the chain-set driver -- 1: k_fc_walk where it
// fits (the default), 0: k_fc_drive everywhere.  Returns the previous choice.
extern "C" int pp2_debug_fc_walk(int on) {
  const int prev = pp2::fc_walk_enabled() ? 1 : 0;
  pp2::g_fc_walk = on ? 1 : 0;
  return prev;
}

// Diagnostic (tools/prof_planner.py, PP2_FC_STATS=1): the drivers' counters
// summed per set kind over every launch -- out[16 * (2 * base + (K > 0)) + c],
// c as pp2_debug_fchain_row2's stats; k_fc_walk's fallback chunks by cause in
// k_fc_walk's c = 8 (breaks), 9 (mispredicted segments), 10 (breaks walked
// by their crossing plans), 11 .. 14 (s_memtime cycles in segments, fetches of exact chunks,
// exact rounds, chunk 0), 15 .. 21 (the longest chain and its counts), 22 / 23
// (the tables' crossing plans and their s_memtime cycles).
// (256 ints)  enable=1 allocates (before the sets to
// count are launched), out != nullptr copies the 64 counters out and clears them.
extern "C" int pp2_debug_fc_stats(int* out, int enable) {
  if (enable && !pp2::g_fc_stats) {
    if (hipMalloc(&pp2::g_fc_stats, 256 * sizeof(int)) != hipSuccess) return 1;
    if (hipMemset(pp2::g_fc_stats, 0, 256 * sizeof(int)) != hipSuccess) return 1;
  }
  if (out && pp2::g_fc_stats) {
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpy(out, pp2::g_fc_stats, 256 * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
      return 1;
    if (hipMemset(pp2::g_fc_stats, 0, 256 * sizeof(int)) != hipSuccess) return 1;
  }
  return 0;
}

// Diagnostic (tests): sums + tables as one launch (1) or two (0, the default).
// Returns the previous choice.
extern "C" int pp2_debug_fc_sumtab(int on) {
  const int prev = pp2::fc_sumtab_enabled() ? 1 : 0;
  pp2::g_fc_sumtab = on ? 1 : 0;
  return prev;
}
