// pp2_coded_dev.h -- device helpers of the dictionary-coded kernels
// (pp2_coded.hip: one step / step pairs; pp2_resident.hip: the tile-resident
// loop): LDS staging, stencil windows of beliefs / values / codes, the coded
// belief gather and the factored Bellman backup.  Per cell the arithmetic is
// the dense kernels' (same operands, same fmaf order).
#pragma once
#include "pp2_device.h"

namespace pp2 {
namespace {

// ---------------------------------------------------------------- kernels
// Two LDS layouts of the sweep rows:
//  * full     (kDictTC = 90 floats per entry): [a][gT_a0..gT_a8, C_a];
//  * factored (sparse; pp2_internal.h): per-action tables of the distinct
//    (gT support quad, C_a) pairs and one 16-B record of byte offsets per
//    entry -- only the base-kernel support of each action (at most 4 cells;
//    the host checks every other T entry of every row is +0.0).
// gT = fl(gamma * T), rounded once on the host exactly as the dense sweep
// rounds gamma * T per cell (one fp32 multiply, round to nearest).  The belief
// gather reads raw T from a per-action table (tu: E x 5 sparse / E x 9 full).
// Sparse backups skip the T == 0 terms: fmaf(gamma*0, J, cost) == cost for
// the finite, non-negative J and cost of the MDP (J starts at 0, C >= +0,
// checked on the host), so values and actions stay bit-identical to the
// dense kernel.
template <bool SPARSE>
struct Layout {
  static constexpr int tu = tu_width(SPARSE);  // raw T_u floats per entry (belief gather)
};

// Global -> LDS copy of n floats with LDS-DMA (global_load_lds_dwordx4: no
// VGPR round trip, so the registers of an already-issued tile load stay
// free).  One wave-instruction writes 1 KiB contiguously at a wave-uniform
// base; the last one's tail lanes re-read the final 16 B of src and land in
// the slack up to lds_span(n) floats.  The __syncthreads() that follows
// waits for the DMA (vmcnt(0)).
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

__host__ __device__ constexpr int lds_span(int n) { return (n + 255) & ~255; }

__device__ __forceinline__ void stage_rows(const float* __restrict__ src, int n, float* dst) {
  const int n4 = (n + 3) >> 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int c = wave; c * 64 < n4; c += nw) {
    int i = c * 64 + lane;
    if (i >= n4) i = n4 - 1;
    __builtin_amdgcn_global_load_lds((glb_void*)(src + 4 * i), (lds_void*)(dst + c * 256), 16, 0,
                                     0);
  }
}

// Factored-row Bellman backup of cell k of N (k_mdp_sweep's arithmetic) from
// its IW record {w0, w1, w2}: per action a quad from QT (a float for the
// one-cell stay support) and the cost from CT at the same byte offset; the
// support positions index jn at compile time.  Actions are compared in
// ascending order, so best/arg are the dense kernel's.  ARG = false: values
// only, best = minnum over the actions (see coded_sweep4).
template <int N, bool ARG>
__device__ __forceinline__ void sweep_cell_fact(const float* sTC, uint32_t w0, uint32_t w1,
                                                uint32_t w2, const float (&jn)[9][N], int k,
                                                float& best, uint32_t& arg) {
  const char* qt = reinterpret_cast<const char*>(sTC + kFactQT);
  const char* ct = reinterpret_cast<const char*>(sTC + kFactCT);
#pragma unroll
  for (int a = 0; a < 9; ++a) {
    const uint32_t w = a < 4 ? w0 : a < 8 ? w1 : w2;
    const uint32_t off = __builtin_amdgcn_ubfe(w, 8 * (a % 4), 8);
    const int tab = a * kFactK * 16;  // byte offset of action a's table
    float tv[4];
    if (kSupN[a] == 1) {
      tv[0] = *reinterpret_cast<const float*>(qt + tab + off);
    } else {
      const f4a t = *reinterpret_cast<const f4a*>(qt + tab + off);
      tv[0] = t[0]; tv[1] = t[1]; tv[2] = t[2]; tv[3] = t[3];
    }
    float cost = *reinterpret_cast<const float*>(ct + tab + off);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < kSupN[a]) cost = __builtin_fmaf(tv[j], jn[kSup[a][j]][k], cost);
    if constexpr (ARG) {
      if (cost < best) { best = cost; arg = (uint32_t)a; }
    } else {
      best = __builtin_fminf(best, cost);
    }
  }
}

// The backup of N cells from their codes: cell-outer, one IW record per cell,
// the scheduling barrier keeps one cell's loads live at a time.
template <int N, bool ARG>
__device__ __forceinline__ void coded_sweep_sparse(const float* sTC, const uint32_t (&cc)[N],
                                                   const float (&jn)[9][N], float (&best)[N],
                                                   uint32_t (&arg)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) { best[k] = FLT_MAX; arg[k] = 0; }
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint4 iw = *reinterpret_cast<const uint4*>(sTC + kFactIW + 4 * cc[k]);
    sweep_cell_fact<N, ARG>(sTC, iw.x, iw.y, iw.z, jn, k, best[k], arg[k]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// The same with the cells' IW records held in registers (the resident loop).
// G > 0: action-outer -- the table reads of one action for a group of G cells
// are in flight together (one LDS round trip per action and group instead of
// one per cell and action); per cell the same fmaf chain and ascending action
// order, so the results are the cell-outer ones bit for bit.  It pays where a
// SIMD holds few waves to hide the round trips (3-row tiles: 4.72 -> 4.46 us
// per step) and costs 2-4 % at 4 waves per SIMD (profiles/r04/ab_sweep_ao.txt).
template <int N, bool ARG, int G = 0>
__device__ __forceinline__ void coded_sweep_iw(const float* sTC, const uint32_t (&iw)[N][3],
                                               const float (&jn)[9][N], float (&best)[N],
                                               uint32_t (&arg)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) { best[k] = FLT_MAX; arg[k] = 0; }
  if constexpr (G > 0) {
    static_assert(N % G == 0, "cell groups");
    const char* qt = reinterpret_cast<const char*>(sTC + kFactQT);
    const char* ct = reinterpret_cast<const char*>(sTC + kFactCT);
#pragma unroll
    for (int a = 0; a < 9; ++a) {
      const int tab = a * kFactK * 16;
#pragma unroll
      for (int k0 = 0; k0 < N; k0 += G) {
        float tv[G][4], cost[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int k = k0 + g;
          const uint32_t w = a < 4 ? iw[k][0] : a < 8 ? iw[k][1] : iw[k][2];
          const uint32_t off = __builtin_amdgcn_ubfe(w, 8 * (a % 4), 8);
          if (kSupN[a] == 1) {
            tv[g][0] = *reinterpret_cast<const float*>(qt + tab + off);
          } else {
            const f4a t = *reinterpret_cast<const f4a*>(qt + tab + off);
            tv[g][0] = t[0]; tv[g][1] = t[1]; tv[g][2] = t[2]; tv[g][3] = t[3];
          }
          cost[g] = *reinterpret_cast<const float*>(ct + tab + off);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int k = k0 + g;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < kSupN[a]) cost[g] = __builtin_fmaf(tv[g][j], jn[kSup[a][j]][k], cost[g]);
          if constexpr (ARG) {
            if (cost[g] < best[k]) { best[k] = cost[g]; arg[k] = (uint32_t)a; }
          } else {
            best[k] = __builtin_fminf(best[k], cost[g]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // one group's reads live at a time
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      sweep_cell_fact<N, ARG>(sTC, iw[k][0], iw[k][1], iw[k][2], jn, k, best[k], arg[k]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Bellman backup of 4 cells from their codes (k_mdp_sweep's arithmetic).
// ARG = false: values only (the resident loop's intermediate steps store no
// actions), best = minnum over the actions -- the same value as the strict-<
// scan, since every cost is an fmaf result (canonical, flushed, never -0 or
// NaN under the sparse rows' preconditions); one v_min per action instead of
// a compare and two selects.
template <bool SPARSE, bool ARG = true>
__device__ __forceinline__ void coded_sweep4(const float* sTC, const uint32_t (&cc)[4],
                                             const float (&jn)[9][4], float gamma,
                                             float (&best)[4], uint32_t (&arg)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) { best[k] = FLT_MAX; arg[k] = 0; }
  if constexpr (SPARSE) {
    coded_sweep_sparse<4, ARG>(sTC, cc, jn, best, arg);
  } else {
    // one action at a time: 4 cells x 10 dictionary floats live (a fully
    // unrolled action loop hoists all 360 LDS reads and spills)
#pragma unroll 1
    for (int a = 0; a < 9; ++a) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f2a* row = reinterpret_cast<const f2a*>(sTC + cc[k] * kDictTC + a * 10);
        const f2a t01 = row[0], t23 = row[1], t45 = row[2], t67 = row[3], t8c = row[4];
        const float tv[9] = {t01[0], t01[1], t23[0], t23[1], t45[0], t45[1], t67[0], t67[1], t8c[0]};
        float cost = t8c[1];
#pragma unroll
        for (int i = 0; i < 9; ++i) cost = __builtin_fmaf(tv[i], jn[i][k], cost);
        if (cost < best[k]) { best[k] = cost; arg[k] = (uint32_t)a; }
      }
    }
  }
}

__device__ __forceinline__ void load_jn(const float* __restrict__ J_in, int wp, int y, int x0,
                                        bool le, bool re, float (&jn)[9][4]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int oy = i / 3 - 1, ox = i % 3 - 1;
    const float* jp = J_in + (long long)(y + oy) * wp + x0 + ox;
    if (ox == 0) ldv<4, true>(jp, jn[i]);
    else ldv<4, false>(jp, jn[i]);
    if (ox < 0 && le) jn[i][0] = 0.0f;
    if (ox > 0 && re) jn[i][3] = 0.0f;
  }
}

// A lane's 3-row stencil window over its 4 cells: x0-1 .. x0+4 of rows
// y-1, y, y+1 (one aligned 16-B load and two dword loads per row).  Values
// outside the grid's x range are 0.
struct Win6 {
  float v[3][6];
};

__device__ __forceinline__ void load_win6(const float* __restrict__ base, int wp, int y, int x0,
                                          bool le, bool re, Win6& w) {

#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float* p = base + (long long)(y + r - 1) * wp + x0;
    const f4a m = *reinterpret_cast<const f4a*>(p);
    const float l = p[-1], rt = p[4];
    w.v[r][0] = le ? 0.0f : l;
    w.v[r][1] = m[0];
    w.v[r][2] = m[1];
    w.v[r][3] = m[2];
    w.v[r][4] = m[3];
    w.v[r][5] = re ? 0.0f : rt;
  }
}

// Packed codes of the same window: per row the dword at x0-2 (x0-1 in its
// high half), the 4 codes at x0..x0+3, the dword at x0+4 (x0+4 in its low half).
struct CodeWin6 {
  uint32_t lw[3], m0[3], m1[3], rw[3];
  __device__ __forceinline__ uint32_t at(int r, int c) const {
    switch (c) {
      case 0: return lw[r] >> 16;
      case 1: return m0[r] & 0xffffu;
      case 2: return m0[r] >> 16;
      case 3: return m1[r] & 0xffffu;
      case 4: return m1[r] >> 16;
      default: return rw[r] & 0xffffu;
    }
  }
};

__device__ __forceinline__ void load_codes6(const uint16_t* __restrict__ code, int wp, int y,
                                            int x0, CodeWin6& w) {
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const uint16_t* cp = code + (long long)(y + r - 1) * wp + x0;
    const uint2 m = *reinterpret_cast<const uint2*>(cp);
    w.m0[r] = m.x;
    w.m1[r] = m.y;
    w.lw[r] = *reinterpret_cast<const uint32_t*>(cp - 2);
    w.rw[r] = *reinterpret_cast<const uint32_t*>(cp + 4);
  }
}

template <bool NT>
__device__ __forceinline__ void store4(float* __restrict__ p, const float (&v)[4]) {
  const f4a t = {v[0], v[1], v[2], v[3]};
  if constexpr (NT) __builtin_nontemporal_store(t, reinterpret_cast<f4a*>(p));
  else *reinterpret_cast<f4a*>(p) = t;
}

template <bool NT>
__device__ __forceinline__ void store_ja(float* __restrict__ J_out, uint8_t* __restrict__ A,
                                         long long off, const float (&best)[4],
                                         const uint32_t (&arg)[4]) {
  store4<NT>(J_out + off, best);
  const uint32_t a4 = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  if constexpr (NT) __builtin_nontemporal_store(a4, reinterpret_cast<uint32_t*>(A + off));
  else *reinterpret_cast<uint32_t*>(A + off) = a4;
}

// Support slot of T[.][u][i] in the sparse layout, or -1 (T == 0 there).
__host__ __device__ constexpr int sup_slot(int u, int i) {
  for (int j = 0; j < kSupN[u]; ++j)
    if (kSup[u][j] == i) return j;
  return -1;
}

// The two halves of a coded fused step for one lane's 4 cells.  U >= 0: the
// action is known at compile time (sparse layout), so only its <= 4 support
// terms are gathered -- the others are fmaf(+0, b, p) == p (b >= 0, p never
// -0) -- in the same ascending-s order.
template <bool SPARSE, int U = -1>
__device__ __forceinline__ void belief_vals(const Geom& g, const float* sTu, const float* sL,
                                            const int (&slot)[9], float inv,
                                            const CodeWin6& cw, const Win6& win, int x0,
                                            float (&p)[4], float& local) {
  using LY = Layout<SPARSE>;
  const bool lx = x0 == 0, rx = x0 + 4 == g.wp;
  // p = L_z * sum_s T[x+off_s][u][8-s] b(x+off_s), in s order
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = 0.0f;
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const int oy = s / 3, ox = s % 3 - 1;
    const int sl = U >= 0 ? sup_slot(U, 8 - s) : slot[8 - s];
    if (U >= 0 && sl < 0) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float tv = sl >= 0 ? sTu[cw.at(oy, k + 1 + ox) * LY::tu + sl] : 0.0f;
      if (ox < 0 && k == 0 && lx) tv = 0.0f;
      if (ox > 0 && k == 3 && rx) tv = 0.0f;
      p[k] = __builtin_fmaf(tv, win.v[oy][k + 1 + ox], p[k]);
    }
    __builtin_amdgcn_sched_barrier(0);  // <= 4 gathers in flight (64-VGPR budget)
  }
  local = 0.0f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    p[k] = p[k] * sL[cw.at(1, k + 1)];
    p[k] = p[k] * inv;
    local += p[k];
  }
}

template <bool SPARSE, int U = -1, bool NT = false>
__device__ __forceinline__ void belief_cells(const Geom& g, const float* sTu, const float* sL,
                                             const int (&slot)[9], float inv,
                                             const CodeWin6& cw, const Win6& win, int y, int x0,
                                             float* __restrict__ b_out, float& local) {
  float p[4];
  belief_vals<SPARSE, U>(g, sTu, sL, slot, inv, cw, win, x0, p, local);
  store4<NT>(b_out + (long long)y * g.wp + x0, p);
}

template <bool SPARSE, bool NT = false>
__device__ __forceinline__ void sweep_cells(const Geom& g, const float* sTC, float gamma,
                                            uint32_t m0, uint32_t m1, const Win6& win, int y,
                                            int x0, bool own, float* __restrict__ J_out,
                                            uint8_t* __restrict__ A) {
  float jn[9][4];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) jn[i][k] = win.v[i / 3][k + i % 3];
  const uint32_t cc[4] = {m0 & 0xffffu, m0 >> 16, m1 & 0xffffu, m1 >> 16};
  float best[4];
  uint32_t arg[4];
  coded_sweep4<SPARSE>(sTC, cc, jn, gamma, best, arg);
  const long long off = (long long)y * g.wp + x0;
  if (own) {
    store_ja<NT>(J_out, A, off, best, arg);
  } else {
    store4<NT>(J_out + off, best);
  }
}

// J or b window of a lane from an LDS region holding the plane from flat cell
// r0 on.
__device__ __forceinline__ void region_win6(const float* sR, int wp, int y, int x0, long long r0,
                                            bool le, bool re, Win6& w) {
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const float* p = sR + ((long long)(y + r - 1) * wp + x0 - r0);
    const f4a m = *reinterpret_cast<const f4a*>(p);
    const float l = p[-1], rt = p[4];
    w.v[r][0] = le ? 0.0f : l;
    w.v[r][1] = m[0];
    w.v[r][2] = m[1];
    w.v[r][3] = m[2];
    w.v[r][4] = m[3];
    w.v[r][5] = re ? 0.0f : rt;
  }
}

__device__ __forceinline__ void belief_u(int u, const Geom& g, const float* sTu, const float* sL,
                                         float inv, const CodeWin6& cw, const Win6& w, int x0,
                                         float (&p)[4], float& local) {
  const int slot[9] = {-1, -1, -1, -1, -1, -1, -1, -1, -1};  // unused (U >= 0)
  switch (u) {
#define PP2_BV(UU) \
  case UU: belief_vals<true, UU>(g, sTu, sL, slot, inv, cw, w, x0, p, local); break;
    PP2_BV(0) PP2_BV(1) PP2_BV(2) PP2_BV(3) PP2_BV(4) PP2_BV(5) PP2_BV(6) PP2_BV(7)
    default: belief_vals<true, 8>(g, sTu, sL, slot, inv, cw, w, x0, p, local);
#undef PP2_BV
  }
}

template <bool ARG = true>
__device__ __forceinline__ void sweep_vals(const float* sTC, float gamma, const CodeWin6& cw,
                                           const Win6& w, float (&best)[4], uint32_t (&arg)[4]) {
  float jn[9][4];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) jn[i][k] = w.v[i / 3][k + i % 3];
  const uint32_t cc[4] = {cw.m0[1] & 0xffffu, cw.m0[1] >> 16, cw.m1[1] & 0xffffu, cw.m1[1] >> 16};
  coded_sweep4<true, ARG>(sTC, cc, jn, gamma, best, arg);
}

}  // namespace
}  // namespace pp2
