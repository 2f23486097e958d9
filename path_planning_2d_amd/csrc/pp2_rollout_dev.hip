// pp2_rollout_dev.hip -- the batched fp16 rollout step kernel (gfx950).
//
// BASELINE configs[4]: C copies of a belief, each advanced by the reference
// update (a2/a3: point_based_value_iteration_cuda.cu:88-133 with the
// renormalisation of search_tree_cuda.cu:225-229) under its own (u, z) per
// step, scoring its QNode reward <b, R[:,u]> (search_tree_cuda.cu:168-173).
// Beliefs are fp16 planes [copy][row -1 .. rows][wp], max-normalised per copy
// (the update of step k multiplies by 1 / max_k); the math is fp32.
//
// The step is HBM-bound on 2 B read + 2 B written per cell-copy (measured
// ceiling for this traffic on MI355X: a plain streaming copy runs 4.5-5.9
// TB/s read+write, tools/micro/copy_bw.hip).  The kernel moves each belief
// byte once:
//  * a wave walks DOWN a band of kBandRows rows of one 256-column segment
//    (64 lanes x 4 cells) and keeps each copy's rows y-1, y, y+1 in
//    registers; row y+1 comes from an LDS ring that LDS-DMA
//    (global_load_lds, no VGPRs) fills NS-1 rows ahead -- beliefs, codes,
//    R_u and the segment-edge dwords of every copy -- with explicit vmcnt
//    waits (the compiler's own would drain the ring at every LDS read);
//  * the x-1 / x+4 neighbours come from the adjacent lanes by DPP wave
//    shifts (v_mov_b32_dpp wave_shr:1 / wave_shl:1); lanes 0 and 63, which
//    have no neighbour lane, keep the DPP's `old` operand: the edge dword;
//  * the CH copies of a workgroup share the step's action, so the T_u
//    coefficients of a row (from the coded model's LDS table, by the codes
//    of the 3x3 neighbourhood, or from the dense T planes) are gathered once
//    for all of them; on a sparse model only the action's <= 4 support terms
//    are gathered (the others are fmaf(+0, b, p) == p exactly, b >= 0);
//  * the fp16 -> fp32 decode folds into v_fma_mix_f32, the stored-sum
//    statistic into v_dot2c_f32_f16, the output pack into v_cvt_pk_f16_f32;
//  * each copy's {stored sum, stored max, reward dot} stays in registers for
//    the band and is written as one partial per (copy, wave), reduced per
//    copy by k_rollout_reduce (pp2_kernels.hip) in a fixed order.
// Per cell the arithmetic is the dense update's: p = sum_s fmaf(T, b, p) in
// ascending stencil order s, then p * fl(L_z / max).  The coded and dense
// model sources give bit-identical beliefs and statistics.

#include <type_traits>

#include "pp2_device.h"

namespace pp2 {
namespace {

constexpr int kSegCells = 256;  // columns of one wave (64 lanes x 4 cells)
constexpr int kBandRows = 32;   // rows one wave walks
constexpr int kRollStats = 3;   // stored sum, stored max, reward dot

enum Src { kSparse = 0, kFull = 1, kDense = 2 };

// Number of stencil terms and the stencil index s of term t (ascending s).
// Sparse: the support of action U (kSup[U][.] ascending in i = 8 - s).
template <int SRC, int U>
__host__ __device__ constexpr int n_terms() { return SRC == kSparse ? kSupN[U] : 9; }
template <int SRC, int U>
__host__ __device__ constexpr int term_s(int t) {
  return SRC == kSparse ? 8 - kSup[U][kSupN[U] - 1 - t] : t;
}
// Column of term t in a tu table row (sparse: support slot; full: i = 8 - s).
template <int SRC, int U>
__host__ __device__ constexpr int term_col(int t) {
  return SRC == kSparse ? kSupN[U] - 1 - t : 8 - t;
}

// One row of a lane's window: cells x0..x0+3 as two fp16 (or uint16 code)
// pairs, and the two dwords the DPP wave shifts deliver: l (high half =
// cell x0-1) and r (low half = cell x0+4).  v_fma_mix_f32 reads either half
// of a dword directly, so no unpacking is done.
struct Row4 {
  uint32_t lo, hi, l, r;
};

__device__ __forceinline__ uint32_t at(const Row4& w, int c) {
  switch (c) {
    case 0: return w.l >> 16;
    case 1: return w.lo & 0xffffu;
    case 2: return w.lo >> 16;
    case 3: return w.hi & 0xffffu;
    case 4: return w.hi >> 16;
    default: return w.r & 0xffffu;
  }
}

__device__ __forceinline__ float hf(uint32_t h) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)h);
}

// A row as read from the ring: the lane's 4 cells (8 B), and the edge dword
// that lanes 0 / 63 use as the neighbour outside the segment (lane 0: the
// dword ending at x0-1, lane 63: the dword starting at x0+4; zeros outside
// the grid).
struct Raw {
  uint2 m;
  uint32_t e;
};

__device__ __forceinline__ const char* cptr(const void* base, uint32_t off) {
  return reinterpret_cast<const char*>(base) + off;
}

// Window row from a raw load: lane i gets lane i-1's high dword and lane
// i+1's low dword by DPP wave shifts; a lane without a source lane (0 for
// wave_shr, 63 for wave_shl) keeps the `old` operand, its loaded edge dword.
__device__ __forceinline__ Row4 make_row(const Raw& q) {
  Row4 w;
  w.lo = q.m.x;
  w.hi = q.m.y;
  w.l = (uint32_t)__builtin_amdgcn_update_dpp((int)q.e, (int)q.m.y, 0x138, 0xf, 0xf, false);
  w.r = (uint32_t)__builtin_amdgcn_update_dpp((int)q.e, (int)q.m.x, 0x130, 0xf, 0xf, false);
  return w;
}

struct BandArgs {
  Geom g;
  PlaneSet T, L, R;
  const uint16_t* code;  // code plane at row -1
  const _Float16* bin;   // copy 0's plane at row -1
  _Float16* bout;
  long long cstride;  // halfs per copy plane (outputs)
  long long istride;  // between the copies' input planes (0: one shared image)
  float* partials;
  int nwaves;
};

typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// LDS-DMA (global_load_lds): global -> LDS without VGPRs, so a wave keeps
// NS-1 rows of loads in flight at no register cost.  The compiler does not
// track these copies: band() waits for them with an explicit s_waitcnt.
__device__ __forceinline__ void dma4(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((glb_void*)g, (lds_void*)l, 4, 0, 0);
}
__device__ __forceinline__ void dma16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((glb_void*)g, (lds_void*)l, 16, 0, 0);
}

// Ring slot of one row (bytes): CH belief rows of the segment (512 B each),
// the code row (512), the R_u row (1 KB) and 64 edge dwords (lane l of the
// edge copy writes dword l: 2j / 2j+1 = copy j's x-1 / x+256 dwords, 2CH /
// 2CH+1 the code row's).
// W16 (row stride wp % 8 == 0, and 16-B aligned copy planes): the belief
// rows by 16-B LDS-DMA, two copies' rows per instruction (lanes 0-31 /
// 32-63), the code row by half a wave -- 5 DMA instructions per row instead
// of 12 (512^2 x 4096 x 5: 5.34 vs 5.46-5.69 ms, profiles/r05/ab_rollout_dma16.txt).
template <int CH, bool W16>
struct Slot {
  // (W16 stages two copies' rows per 16-B instruction: an odd CH would leave
  // the last copy's rows unstaged)
  static_assert(!W16 || CH % 2 == 0, "16-B belief staging needs an even copy count");
  static constexpr int code = CH * 512, r = code + 512, edge = r + 1024, bytes = edge + 256;
  static constexpr int groups = W16 ? CH / 2 + 3 : 2 * CH + 4;  // DMA instructions per row
};

// Ring budget of a band build (kBandSlots = NS): every row of a wave's ring
// travels as one DMA group of G instructions into its own slot, and band()
// waits on hand-counted vmcnt values of up to (NS - 2) (G + CH) (the younger
// groups plus the stores of the phases between), which must fit the 6-bit
// counter; the 4 waves' rings of WPS workgroups must fit one CU's 160 KB of
// LDS beside the dictionary tables (the launch checks the dynamic part).
template <int CH, int NS, int WPS, bool W16>
struct RingBudget {
  static_assert(NS >= 3, "the window needs rows y-1, y, y+1 resident plus one in flight");
  static_assert((NS - 2) * (Slot<CH, W16>::groups + CH) < 64, "vmcnt wait exceeds 6 bits");
  static constexpr int ring_bytes = 4 * NS * Slot<CH, W16>::bytes;
  static_assert(WPS * ring_bytes <= 160 * 1024, "rings of WPS workgroups exceed the CU's LDS");
};

// One wave's band: rows [ya, yb) of the segment starting at xs.
// sTu: [E][TW] T_u table (coded); sLz: [CH][E] L_z * (1 / max) of each copy;
// ring: this wave's NS slots.  Row r of a copy / code plane is at byte
// offset 2 (r + 1) wp (row -1 = 0, the zero halo row that cells outside the
// grid and lanes past the row end read instead).  Those lanes' outputs are
// exactly 0 (zero beliefs; codes of the all-zero halo tuple, L = 0); they
// store them into row -1 and add 0 to every statistic, so no lane is masked
// (the dense source zeroes their L_z explicitly: its L plane is read at the
// clamped cell).
template <int CH, int NS, int SRC, int U, bool W16>
__device__ __forceinline__ void band(const BandArgs& a, const float* sTu, const float* sLz,
                                     char* ring, int E, int ecid, const int (&cid)[CH],
                                     const int (&zc)[CH], const float (&inv)[CH], int u, int ya,
                                     int yb, int xs, int lane, float (&acc)[CH][kRollStats]) {
  using SL_ = Slot<CH, W16>;
  static_assert(sizeof(RingBudget<CH, NS, 1, W16>) > 0, "");
  constexpr int NT = n_terms<SRC, U>();
  constexpr int TW = tu_width(SRC == kSparse);
  constexpr int G = SL_::groups;
  const Geom& g = a.g;
  const int x0 = xs + 4 * lane;  // this lane's first cell (compute)
  const bool xok = x0 < g.wp;
  const int xc = xok ? x0 : g.wp - 4;
  const uint32_t rowb = 2u * (uint32_t)g.wp;  // bytes per plane row
  // DMA lanes: 2 cells per lane and copy instruction (h = 0, 1 halves)
  const int dx0 = xs + 2 * lane, dx1 = dx0 + 128;
  const bool d0ok = dx0 < g.wp, d1ok = dx1 < g.wp;
  const uint32_t db0 = 2u * (uint32_t)dx0, db1 = 2u * (uint32_t)dx1;
  // edge lanes: 2j / 2j+1 -> copy j's dword at xs-2 / xs+256, 2CH / 2CH+1 the
  // code row's; outside the grid -> row -1 (zeros)
  const int ej = lane >> 1, es_ = lane & 1;
  const bool eside_ok = es_ == 0 ? xs > 0 : xs + 256 < g.wp;
  const uint32_t ebyte = 2u * (uint32_t)(es_ == 0 ? xs - 2 : xs + 256);
  const void* ebase = ej < CH ? (const void*)(a.bin + (long long)ecid * a.istride)
                              : (const void*)a.code;
  const bool eok = eside_ok && ej <= CH;
  const _Float16* bb[CH];
  _Float16* ob[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    bb[j] = a.bin + (long long)cid[j] * a.istride;
    ob[j] = a.bout + (long long)cid[j] * a.cstride;
  }
  const float* rbase = a.R.p + (long long)u * a.R.ps + xs;
  const bool rok = xs + 4 * lane < g.wp;  // R lane (4 floats)
  // issue the DMA group of row r (beliefs, codes, edges, R_u) into a slot
  // 16-B DMA lanes: 8 cells of copy 2k + (lane >> 5) per instruction k
  const int qx = xs + 8 * (lane & 31);
  const bool qok = qx < g.wp;
  const uint32_t qb = 2u * (uint32_t)qx;
  auto issue = [&](int r, char* slot) {
    const uint32_t ro = (uint32_t)(r + 1) * rowb;
    if constexpr (W16) {
#pragma unroll
      for (int k = 0; k < CH / 2; ++k) {
        const _Float16* src = lane < 32 ? bb[2 * k] : bb[2 * k + 1];
        dma16(cptr(src, qok ? ro + qb : 0u), slot + 2 * k * 512);
      }
      if (lane < 32) dma16(cptr(SRC != kDense ? (const void*)a.code : (const void*)bb[0],
                                SRC != kDense && qok ? ro + qb : 0u),
                           slot + SL_::code);
    } else {
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        dma4(cptr(bb[j], d0ok ? ro + db0 : 0u), slot + j * 512);
        dma4(cptr(bb[j], d1ok ? ro + db1 : 0u), slot + j * 512 + 256);
      }
      if constexpr (SRC != kDense) {
        dma4(cptr(a.code, d0ok ? ro + db0 : 0u), slot + SL_::code);
        dma4(cptr(a.code, d1ok ? ro + db1 : 0u), slot + SL_::code + 256);
      } else {
        dma4(cptr(bb[0], 0u), slot + SL_::code);  // keep G fixed (zeros)
        dma4(cptr(bb[0], 0u), slot + SL_::code + 256);
      }
    }
    const int rr = r < yb ? (r >= 0 ? r : 0) : yb - 1;  // R rows stay inside the grid
    dma16(rbase + (rok ? (long long)rr * a.R.rs + 4 * lane : 0), slot + SL_::r);
    dma4(cptr(ebase, eok ? ro + ebyte : 0u), slot + SL_::edge);
  };
  // wait until at most n VMEM ops are outstanding.  vmcnt counts loads,
  // LDS-DMA copies and stores in issue order (gfx9 has no separate store
  // counter), and every phase issues its DMA group, then its CH stores, in
  // a fixed order (compiler barriers at the phase boundaries), so "row y+1
  // has landed" is vmcnt <= (the ops issued after its group).
  auto wait_n = [&](auto n) {
    constexpr int N = decltype(n)::value;
    static_assert(N < 64, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  };
  auto slot_of = [&](int r) { return ring + ((r - ya + 1) % NS) * SL_::bytes; };
  const int e_own = lane == 0 ? 0 : 1;  // lane 0 -> the x-1 dword, lane 63 -> x+256
  // Ring reads are inline asm: the compiler tracks LDS-DMA writes only
  // coarsely and would put a vmcnt(0) -- a drain of every row in flight --
  // before any LDS read it sees.  read_rows() issues a slot's reads, waits
  // for them (lgkmcnt), and pins the results below that wait.
  auto read_rows = [&](const char* slot, Raw (&q)[CH + 1]) {
    const uint32_t rb = (uint32_t)(uintptr_t)(slot) + 8u * (uint32_t)lane;
    const uint32_t eb2 = (uint32_t)(uintptr_t)(slot) + SL_::edge + 4u * (uint32_t)e_own;
#pragma unroll
    for (int j = 0; j <= CH; ++j) {
      if (SRC == kDense && j == CH) break;
      asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(q[j].m) : "v"(rb), "i"(j * 512));
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(q[j].e) : "v"(eb2), "i"(8 * j));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j <= CH; ++j) {
      if (SRC == kDense && j == CH) break;
      asm volatile("" : "+v"(q[j].m), "+v"(q[j].e));
    }
  };
  auto read_r = [&](const char* slot, float (&r4)[4]) {
    const uint32_t ab = (uint32_t)(uintptr_t)(slot) + SL_::r + 16u * (uint32_t)lane;
    f4a t;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(ab) : "memory");
    r4[0] = t[0]; r4[1] = t[1]; r4[2] = t[2]; r4[3] = t[3];
  };
  Row4 W[CH][3], CW[3];
  // prologue: rows ya-1 .. ya+NS-2 in flight; rows ya-1, ya into window slots
  // 0, 1 once their groups have landed
#pragma unroll
  for (int r = 0; r < NS; ++r) issue(ya - 1 + r <= yb ? ya - 1 + r : yb, ring + r * SL_::bytes);
  wait_n(std::integral_constant<int, (NS - 2) * G>{});
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    Raw q[CH + 1];
    read_rows(ring + r * SL_::bytes, q);
#pragma unroll
    for (int j = 0; j < CH; ++j) W[j][r] = make_row(q[j]);
    if constexpr (SRC != kDense) CW[r] = make_row(q[CH]);
  }

  auto step = [&](auto phase, int y) {
    constexpr int P = decltype(phase)::value;
    constexpr int S0 = P % 3, S1 = (P + 1) % 3, S2 = (P + 2) % 3;  // rows y-1, y, y+1
    // refill the slot of row y-1 (fully consumed) with row y+NS-1, then
    // wait for row y+1's group (NS-2 younger groups may stay in flight)
    {
      asm volatile("" ::: "memory");  // the slot's last reads stay above its refill
      const int rn = y + NS - 1 <= yb ? y + NS - 1 : yb;
      issue(rn, slot_of(y - 1));
    }
    // ops issued after row y+1's group: the NS-2 younger groups, plus the
    // stores of the phases between (none yet in the band's first phase;
    // one phase's in the second; NS-2 phases' from then on)
    if (y >= ya + NS - 2) wait_n(std::integral_constant<int, (NS - 2) * (G + CH)>{});
    else if (y == ya) wait_n(std::integral_constant<int, (NS - 2) * G>{});
    else wait_n(std::integral_constant<int, (NS - 2) * G + CH>{});
    const char* sn = slot_of(y + 1);
    const char* sc = slot_of(y);
    {
      Raw q[CH + 1];
      read_rows(sn, q);
#pragma unroll
      for (int j = 0; j < CH; ++j) W[j][S2] = make_row(q[j]);
      if constexpr (SRC != kDense) CW[S2] = make_row(q[CH]);
    }
    float rcur[4];
    read_r(sc, rcur);
    constexpr int SL[3] = {S0, S1, S2};
    // T_u coefficients of the row's NT stencil terms (shared by the copies)
    float tv[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int s = term_s<SRC, U>(t);
      const int oy = s / 3, ox = s % 3 - 1;
      if constexpr (SRC == kDense) {
        const float* tp = a.T.p + (long long)(y - 1 + oy) * a.T.rs +
                          (long long)(9 * u + 8 - s) * a.T.ps + xc + ox;
        if (ox == 0) ldv<4, true>(tp, tv[t]);
        else ldv<4, false>(tp, tv[t]);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          tv[t][k] = sTu[at(CW[SL[oy]], k + 1 + ox) * TW + term_col<SRC, U>(t)];
      }
    }
    uint32_t lzo[4] = {0, 0, 0, 0};  // coded: the cells' own codes (L_z rows)
    if constexpr (SRC != kDense) {
#pragma unroll
      for (int k = 0; k < 4; ++k) lzo[k] = at(CW[S1], k + 1);
    }
    const uint32_t so = xok ? (uint32_t)(y + 1) * rowb + 2u * (uint32_t)x0 : 0u;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      float li[4];  // L_z * (1 / max) of the 4 cells
      if constexpr (SRC == kDense) {
        float lz[4];
        ldv<4, true>(a.L.p + (long long)y * a.L.rs + (long long)zc[j] * a.L.ps + xc, lz);
#pragma unroll
        for (int k = 0; k < 4; ++k) li[k] = xok ? lz[k] * inv[j] : 0.0f;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) li[k] = sLz[j * E + lzo[k]];
      }
      float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int s = term_s<SRC, U>(t);
        const int oy = s / 3, ox = s % 3 - 1;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          p[k] = __builtin_fmaf(tv[t][k], hf(at(W[j][SL[oy]], k + 1 + ox)), p[k]);
      }
      float v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = p[k] * li[k];
      // stored values; max(fp16(v)) == fp16(max(v)) (rounding is monotone),
      // so the max is taken on v and rounded once per wave
      const h2v h01 = {(_Float16)v[0], (_Float16)v[1]};
      const h2v h23 = {(_Float16)v[2], (_Float16)v[3]};
      const h2v one = {(_Float16)1.0f, (_Float16)1.0f};
      acc[j][0] = __builtin_amdgcn_fdot2(h01, one, acc[j][0], false);
      acc[j][0] = __builtin_amdgcn_fdot2(h23, one, acc[j][0], false);
      acc[j][1] = fmaxf(fmaxf(acc[j][1], v[0]), v[1]);
      acc[j][1] = fmaxf(fmaxf(acc[j][1], v[2]), v[3]);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc[j][2] = __builtin_fmaf(hf(at(W[j][S1], k + 1)), rcur[k], acc[j][2]);
      const u2v o = {__builtin_bit_cast(uint32_t, h01), __builtin_bit_cast(uint32_t, h23)};
      __builtin_nontemporal_store(o, reinterpret_cast<u2v*>(reinterpret_cast<char*>(ob[j]) + so));
    }
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  // whole 3-row groups (every window slot returns to its register), then
  // the tail
  int y = ya;
  for (; y + 3 <= yb; y += 3) {
    step(P0{}, y);
    step(P1{}, y + 1);
    step(P2{}, y + 2);
  }
  if (y < yb) step(P0{}, y);
  if (y + 1 < yb) step(P1{}, y + 1);
  // drain: no DMA may still target this wave's ring when the slot memory
  // is reused (by the next workgroup on the CU)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// grid: nchunks x gx workgroups of 4 waves (1-D, XCD-remapped so that the
// waves of one chunk run on one XCD and share its L2 for the band halos).
// Wave v of a chunk walks band v / nseg of segment v % nseg.
template <int CH, int NS, int WPS, int SRC, bool W16>
__global__ __launch_bounds__(kBlock, WPS) void k_rollout_band(
    BandArgs a, const float* __restrict__ tu_all, long long tstride,
    const float* __restrict__ dl, int es, int E, int gx, int nseg, int nband,
    const int* __restrict__ chunk_u, const int* __restrict__ chunk_first,
    const int* __restrict__ copies, const uint8_t* __restrict__ zs,
    const float* __restrict__ in_stats) {
  constexpr int TW = tu_width(SRC == kSparse);
  static_assert(sizeof(RingBudget<CH, NS, WPS, W16>) > 0, "");
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int ch = lin / gx, bx = lin % gx;
  const int u = chunk_u[ch], first = chunk_first[ch];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // the rings are their own LDS object, so the compiler's LDS-DMA tracking
  // can tell them from the dictionary tables (sTu [E][TW], sLz [CH][E])
  __shared__ __attribute__((aligned(16))) char rings[4 * NS * Slot<CH, W16>::bytes];
  extern __shared__ float rlds[];
  char* ring = rings + w * NS * Slot<CH, W16>::bytes;
  float* sTu = rlds;
  float* sLz = sTu + ((E * TW + 3) & ~3);
  int cid[CH], zc[CH];
  float inv[CH], acc[CH][kRollStats];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = copies[first + j];
    cid[j] = c;
    zc[j] = zs[c];
    inv[j] = 1.0f / in_stats[c * kRollStats + 1];  // 1 / stored max
    acc[j][0] = acc[j][1] = acc[j][2] = 0.0f;
  }
  if constexpr (SRC != kDense) {
    const float* tu = tu_all + (long long)u * tstride;
    for (int i = threadIdx.x; i < E * TW; i += kBlock) sTu[i] = tu[i];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const float* lz = dl + (long long)zc[j] * es;
      for (int e = threadIdx.x; e < E; e += kBlock) sLz[j * E + e] = lz[e] * inv[j];
    }
    __syncthreads();
  }
  // the copy whose edge dwords this lane fetches (lanes 2j, 2j+1 -> copy j)
  const int ecid = copies[first + ((lane >> 1) < CH ? (lane >> 1) : CH - 1)];
  const int v = bx * 4 + w;
  const int seg = v % nseg, bnd = v / nseg;
  if (bnd < nband) {
    const int ya = bnd * kBandRows;
    const int yb = ya + kBandRows < a.g.rows ? ya + kBandRows : a.g.rows;
    const int xs = seg * kSegCells;
    if constexpr (SRC == kSparse) {
      switch (u) {
#define PP2_BAND_U(UU)                                                                         \
  case UU:                                                                                     \
    band<CH, NS, kSparse, UU, W16>(a, sTu, sLz, ring, E, ecid, cid, zc, inv, u, ya, yb, xs, lane, acc); \
    break;
        PP2_BAND_U(0) PP2_BAND_U(1) PP2_BAND_U(2) PP2_BAND_U(3) PP2_BAND_U(4)
        PP2_BAND_U(5) PP2_BAND_U(6) PP2_BAND_U(7)
        default:
          band<CH, NS, kSparse, 8, W16>(a, sTu, sLz, ring, E, ecid, cid, zc, inv, u, ya, yb, xs, lane, acc);
#undef PP2_BAND_U
      }
    } else {
      band<CH, NS, SRC, 0, W16>(a, sTu, sLz, ring, E, ecid, cid, zc, inv, u, ya, yb, xs, lane, acc);
    }
  }
  // one partial per (copy, wave); repeated copies of a partial chunk write
  // identical values.  The max is of the unrounded values: round it here.
  const int gw = bx * 4 + w;
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const float sm = wave_sum(acc[j][0]);
    const float mx = (float)(_Float16)wave_max(acc[j][1]);
    const float rw = wave_sum(acc[j][2]);
    if (lane == 0) {
      float* pp = a.partials + ((long long)cid[j] * a.nwaves + gw) * kRollStats;
      pp[0] = sm;
      pp[1] = mx;
      pp[2] = rw;
    }
  }
}

int band_nseg(const Geom& g) { return (g.wp + kSegCells - 1) / kSegCells; }
int band_nband(const Geom& g) { return (g.rows + kBandRows - 1) / kBandRows; }
int band_gx(const Geom& g) { return (band_nseg(g) * band_nband(g) + 3) / 4; }

// Band shape: 4 copies per chunk, 4 LDS ring slots, 2 waves per SIMD.  The
// other shapes measured (MI355X, 512^2 x 4096 copies x 5 steps): (4,4,2) 6.01
// ms, (4,3,2) 6.21, (2,4,3) 6.25, (8,3,1) 6.36, (4,4,3) 6.20.
#ifndef PP2_BAND_SLOTS  // (A/B builds: EXTRA_FLAGS=-DPP2_BAND_SLOTS=n)
#define PP2_BAND_SLOTS 4
#endif
constexpr int kBandCopies = 4, kBandSlots = PP2_BAND_SLOTS, kBandWaves = 2;

}  // namespace

int rollout_chunk() { return kBandCopies; }
int rollout_min_chunk() { return 2; }
int rollout_step_waves(const Geom& g) { return band_gx(g) * 4; }

hipError_t launch_rollout_step(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet L,
                               PlaneSet R, const uint16_t* code, const float* tu_all,
                               long long tstride, int tw, const float* dl, int es, int E,
                               bool sparse, const void* bin, void* bout, long long cstride,
                               long long istride, int nchunks, const int* chunk_u, const int* chunk_first,
                               const int* copies, const uint8_t* zs, const float* in_stats,
                               float* partials, float* stats_out, int ncopies) {
  const int gx = band_gx(g), nseg = band_nseg(g), nband = band_nband(g);
  const int nw = gx * 4;
  BandArgs a;
  a.g = g;
  a.T = T;
  a.L = L;
  a.R = R;
  a.code = code ? code - g.wp : nullptr;  // row -1
  a.bin = (const _Float16*)bin;            // copy planes start at row -1
  a.bout = (_Float16*)bout;
  a.cstride = cstride;
  a.istride = istride;
  a.partials = partials;
  a.nwaves = nw;
  const long long nblocks = (long long)gx * nchunks;
  if (nblocks <= 0) return hipSuccess;
  const int CH = rollout_chunk();
  const size_t lds = E > 0 ? (size_t)(((E * tw + 3) & ~3) + CH * E) * sizeof(float) : 0;
  // the rings (static) and the tables (dynamic) of one workgroup must fit
  // the CU's LDS; the tables of kDictMax entries always do with 4 slots
  if (lds + (size_t)RingBudget<kBandCopies, kBandSlots, 1, true>::ring_bytes > 160 * 1024)
    return hipErrorInvalidValue;
#define PP2_BAND(CC, PP, WW, W16)                                                                 \
  do {                                                                                            \
    static unsigned long long attr[3] = {0, 0, 0};                                                \
    allow_lds(reinterpret_cast<const void*>(&k_rollout_band<CC, PP, WW, kSparse, W16>), attr[0]); \
    allow_lds(reinterpret_cast<const void*>(&k_rollout_band<CC, PP, WW, kFull, W16>), attr[1]);   \
    allow_lds(reinterpret_cast<const void*>(&k_rollout_band<CC, PP, WW, kDense, W16>), attr[2]);  \
    if (src == kSparse)                                                                           \
      hipLaunchKernelGGL((k_rollout_band<CC, PP, WW, kSparse, W16>), dim3((unsigned)nblocks),     \
                         dim3(kBlock), lds, st, a, tu_all, tstride, dl, es, E, gx, nseg,          \
                         nband, chunk_u, chunk_first, copies, zs, in_stats);                      \
    else if (src == kFull)                                                                        \
      hipLaunchKernelGGL((k_rollout_band<CC, PP, WW, kFull, W16>), dim3((unsigned)nblocks),       \
                         dim3(kBlock), lds, st, a, tu_all, tstride, dl, es, E, gx, nseg,          \
                         nband, chunk_u, chunk_first, copies, zs, in_stats);                      \
    else                                                                                          \
      hipLaunchKernelGGL((k_rollout_band<CC, PP, WW, kDense, W16>), dim3((unsigned)nblocks),      \
                         dim3(kBlock), lds, st, a, tu_all, tstride, dl, es, E, gx, nseg,          \
                         nband, chunk_u, chunk_first, copies, zs, in_stats);                      \
  } while (0)
  const int src = E <= 0 ? kDense : sparse ? kSparse : kFull;
  // 16-B DMA staging: 8-cell lanes must not straddle the row end, and the
  // copy planes must be 16-B aligned (PP2_BAND_DMA16=0 forces 4-B staging)
  const char* w16env = getenv("PP2_BAND_DMA16");
  const bool w16 = g.wp % 8 == 0 && istride % 8 == 0 && cstride % 8 == 0 &&
                   (reinterpret_cast<uintptr_t>(bin) & 15) == 0 && !(w16env && w16env[0] == '0');
  if (w16) PP2_BAND(kBandCopies, kBandSlots, kBandWaves, true);
  else PP2_BAND(kBandCopies, kBandSlots, kBandWaves, false);
#undef PP2_BAND
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_rollout_reduce(st, partials, nw, ncopies, stats_out);
}


// ---------------------------------------------------------------- leaf pass
// The leaf FIB dots of every copy (fast_informed_bound_cuda.cu:278-297's
// <b_D, alpha_i>, i < 9, and the copy's mass) as ONE GEMM on the matrix
// cores: D[copy][col] = sum over cells of b[copy][cell] * B[cell][col], with
// the copies' fp16 planes as A (exact: the stored beliefs ARE fp16) and B's
// columns {1, hi_0..hi_8, lo_0..lo_8}: alpha_i * 2^k_i = hi_i + lo_i in two
// fp16 halves (k_i a per-plane power of two bringing max |alpha_i| into
// [2^13, 2^14): hi + lo carries ~22 bits of it, the rest is below 2^-22 of
// the value or of the plane's max).  Every product is exact in fp32 and the
// MFMA sums in fp32, so the dots match the fp32 fmaf pass (k_rollout_leaf)
// to fp32 rounding -- the fp16 rollout's tolerance (rel 3e-3) is far above.
// Each wave takes 64 copies (two 32-row tiles sharing every B fragment) over
// a slab of kLeafSlab cells; A is streamed once (2 B per cell-copy), B is
// re-read per wave from L2.  The k index of a 32x32x16 step is a permutation
// of 16 consecutive cells: lane (r, h) loads cells 8h .. 8h+7 of its copy r
// (16 B) and of its column r of B, so A and B use the same cells.
namespace {

constexpr int kLeafCols = 19;      // 1 + 9 hi + 9 lo
constexpr int kLeafColsPad = 32;   // B's columns in memory (the MFMA's N; zero past kLeafCols)
#ifndef PP2_LEAF_SLAB
#define PP2_LEAF_SLAB 8192
#endif
#ifndef PP2_LEAF_NS
#define PP2_LEAF_NS 2
#endif
constexpr int kLeafNS = PP2_LEAF_NS;  // LDS ring stages per wave (8 KB each)
constexpr int kLeafSlab = PP2_LEAF_SLAB;  // cells per block (B is padded to a multiple; 64 x NS x n)
constexpr int kLeafParts = 32;     // |alpha| max partials per plane
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16acc __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void k_leaf_alpha_max(Geom g, PlaneSet F, float* __restrict__ part) {
  __shared__ float red[4];
  const int plane = blockIdx.y;
  const long long n = (long long)g.rows * g.wp;
  float m = 0.0f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += 256LL * gridDim.x) {
    const long long y = i / g.wp, x = i - y * g.wp;
    const float v = fabsf(F.p[y * F.rs + plane * F.ps + x]);
    m = v > m ? v : m;  // (a NaN is skipped; the dots carry it anyway)
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    part[plane * kLeafParts + blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// B as columns [kLeafColsPad][ldb] fp16 (ldb a multiple of kLeafSlab, zero
// past the grid's cells and in columns >= kLeafCols); kexp[i] = k_i.
__global__ __launch_bounds__(256) void k_leaf_alpha_pack(Geom g, PlaneSet F,
                                                         const float* __restrict__ part,
                                                         _Float16* __restrict__ B, long long ldb,
                                                         int* __restrict__ kexp) {
  __shared__ float sc[9];
  if (threadIdx.x < 9) {
    float m = 0.0f;
    for (int j = 0; j < kLeafParts; ++j) m = fmaxf(m, part[threadIdx.x * kLeafParts + j]);
    int k = 0;
    if (m > 0.0f && m <= FLT_MAX) {
      const int e = (int)((__float_as_uint(m) >> 23) & 0xffu) - 127;  // (FTZ: m is normal)
      k = 13 - e;
      k = k < -120 ? -120 : k > 120 ? 120 : k;
    }
    sc[threadIdx.x] = ldexpf(1.0f, k);
    if (blockIdx.x == 0) kexp[threadIdx.x] = k;
  }
  __syncthreads();
  const long long n = (long long)g.rows * g.wp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < ldb; i += 256LL * gridDim.x) {
    const bool in = i < n;
    const long long y = in ? i / g.wp : 0, x = in ? i - y * g.wp : 0;
    B[i] = (_Float16)(in ? 1.0f : 0.0f);
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const float v = in ? F.p[y * F.rs + q * F.ps + x] * sc[q] : 0.0f;  // (exact: a power of two)
      const _Float16 hi = (_Float16)v;
      B[(1 + q) * ldb + i] = hi;
      B[(10 + q) * ldb + i] = (_Float16)(v - (float)hi);
    }
#pragma unroll
    for (int q = kLeafCols; q < kLeafColsPad; ++q) B[q * ldb + i] = (_Float16)0.0f;
  }
}

// part[(copy * kLeafCols + col) * nslab + slab].  One wave per workgroup: 64
// copies (two 32-row tiles) over one slab.  A is staged through a per-wave
// LDS ring by LDS-DMA (no VGPRs): a stage is 64 cells of the 64 copies, one
// whole 128-B line per copy row, 8 lanes per line (coalesced; loading the
// MFMA fragments straight from HBM touches 32 lines per instruction for 32 B
// each and ran at 2.8 TB/s).  Lane l of DMA instruction i loads unit
// (l & 7) ^ (l >> 3) of copy 8i + (l >> 3) into ring unit l, so ring unit u
// of local copy c holds global unit u ^ (c & 7): the fragment reads (copy r,
// unit 2s + h) then spread over the banks.  The compiler does not track
// LDS-DMA: the ring is read by inline asm after an explicit vmcnt wait.
__global__ __launch_bounds__(64) void k_rollout_leaf_mfma(const _Float16* __restrict__ b,
                                                          const _Float16* __restrict__ zrow,
                                                          long long cstride, int copies,
                                                          long long ncells,
                                                          const _Float16* __restrict__ B,
                                                          long long ldb, float* __restrict__ part,
                                                          int nslab) {
  constexpr int kSlot = 64 * 128;  // bytes per stage: 64 copies x 64 cells
  __shared__ __attribute__((aligned(16))) char ring[kLeafNS * kSlot];
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int slab = blockIdx.x, c0 = blockIdx.y * 64;
  const long long cell0 = (long long)slab * kLeafSlab;
  // DMA roles: copy 8i + dc, 8-cell unit du of the stage
  const int dc = lane >> 3, du = (lane & 7) ^ dc;
  // B has kLeafColsPad columns (zero past kLeafCols): every lane loads, no branch
  const h8v* bp = reinterpret_cast<const h8v*>(B + (long long)r * ldb + cell0 + 8 * h);
  constexpr int nst = kLeafSlab / 64;
  static_assert(nst % kLeafNS == 0 && kLeafNS >= 2 && kLeafNS <= 3, "whole ring rounds");
  auto issue = [&](int k, char* slot) {
    const long long cell = cell0 + 64 * k + 8 * du;
    const bool ok = cell < ncells;  // (ncells is a multiple of 8)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const _Float16* g = b + (long long)min(c0 + 8 * i + dc, copies - 1) * cstride + cell;
      uintptr_t ga = (uintptr_t)(ok ? g : zrow);
      asm("" : "+v"(ga));  // one VGPR-addressed DMA per i (not one per side of the select)
      __builtin_amdgcn_global_load_lds((glb_void*)ga, (lds_void*)(slot + i * 1024), 16, 0, 0);
    }
  };
  // B's fragments by inline asm as well: the compiler's own wait for them
  // would be a vmcnt(0) (it does not follow the pipeline across the loop),
  // which also drains the next stage's DMA; stage() waits for them itself
  auto ldb4 = [&](int k, h8v (&y)[4]) {
    const h8v* q = bp + 8 * k;
#pragma unroll
    for (int st = 0; st < 4; ++st)
      asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(y[st]) : "v"(q), "i"(32 * st) : "memory");
  };
  // the fragment reads of a stage: tile t, step st -> copy 32t + r, unit 2st + h
  uint32_t roff[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int st = 0; st < 4; ++st)
      roff[t][st] = (uint32_t)(((32 * t + r) * 8 + ((2 * st + h) ^ (r & 7))) * 16);
  f16acc acc0 = {}, acc1 = {};
  h8v Bf[kLeafNS][4];
  // stage k from slot k % NS with B fragments Bf[k % NS]; stage k + NS - 1
  // (its slot, its fragments) issued first, so NS - 1 stages stay in flight
  // (MORE: stage k + NS - 1 exists -- a compile-time flag, so that the
  // issue and its wait stay one branch-free block: tools/asm_hazard_check.py
  // follows each wait to the loads it covers)
  auto stage = [&](int k, auto kk, auto more) {
    constexpr int q = decltype(kk)::value;  // k % NS
    constexpr int qn = (q + kLeafNS - 1) % kLeafNS;
    if constexpr (decltype(more)::value) {
      asm volatile("" ::: "memory");  // slot qn's reads (stage k-1) completed (lgkmcnt(0))
      issue(k + kLeafNS - 1, ring + qn * kSlot);
      ldb4(k + kLeafNS - 1, Bf[qn]);
      // stage k's DMA and B loads landed (the NS - 1 younger groups of 12 may not have)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(12 * (kLeafNS - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    h8v A[2][4];
    const uint32_t base = (uint32_t)(uintptr_t)(ring + q * kSlot);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int st = 0; st < 4; ++st)
        asm volatile("ds_read_b128 %0, %1" : "=v"(A[t][st]) : "v"(base + roff[t][st]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int st = 0; st < 4; ++st) asm volatile("" : "+v"(A[t][st]));
#pragma unroll
    for (int st = 0; st < 4; ++st) asm volatile("" : "+v"(Bf[q][st]));  // (landed: the vmcnt above)
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0][st], Bf[q][st], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[1][st], Bf[q][st], acc1, 0, 0, 0);
    }
  };
#pragma unroll
  for (int j = 0; j < kLeafNS - 1; ++j) {
    issue(j, ring + j * kSlot);
    ldb4(j, Bf[j]);
  }
  using Yes = std::true_type;
  using No = std::false_type;
  int k = 0;
  for (; k + kLeafNS < nst; k += kLeafNS) {
    stage(k, std::integral_constant<int, 0>{}, Yes{});
    stage(k + 1, std::integral_constant<int, 1>{}, Yes{});
    if constexpr (kLeafNS > 2) stage(k + 2, std::integral_constant<int, 2 % kLeafNS>{}, Yes{});
  }
  // the last round (k = nst - NS): only its first stage has a stage NS - 1 ahead
  stage(k, std::integral_constant<int, 0>{}, Yes{});
  stage(k + 1, std::integral_constant<int, 1>{}, No{});
  if constexpr (kLeafNS > 2) stage(k + 2, std::integral_constant<int, 2 % kLeafNS>{}, No{});
  // D: column r (= lane & 31), rows (v & 3) + 8 (v >> 2) + 4 h
  if (r < kLeafCols) {
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int row = (v & 3) + 8 * (v >> 2) + 4 * h;
      const int ca = c0 + row, cb = c0 + 32 + row;
      if (ca < copies) part[((long long)ca * kLeafCols + r) * nslab + slab] = acc0[v];
      if (cb < copies) part[((long long)cb * kLeafCols + r) * nslab + slab] = acc1[v];
    }
  }
}

// out[copy][10] = {sum, dot_0 .. dot_8}: per slab hi + lo, the slabs in a
// fixed order, times 2^-k_i.
__global__ __launch_bounds__(64) void k_rollout_leaf_mfma_reduce(const float* __restrict__ part, int nslab,
                                                                 int copies, const int* __restrict__ kexp,
                                                                 float* __restrict__ out) {
  const int c = blockIdx.x;
  if (c >= copies) return;
  const float* pc = part + (long long)c * kLeafCols * nslab;
  float s = 0.0f;
  for (int j = threadIdx.x; j < nslab; j += 64) s += pc[j];
  s = wave_sum(s);
  if (threadIdx.x == 0) out[c * 10] = s;
  for (int q = 0; q < 9; ++q) {
    float d = 0.0f;
    for (int j = threadIdx.x; j < nslab; j += 64) d += pc[(1 + q) * nslab + j] + pc[(10 + q) * nslab + j];
    d = wave_sum(d);
    if (threadIdx.x == 0) out[c * 10 + 1 + q] = ldexpf(d, -kexp[q]);
  }
}

}  // namespace

bool rollout_leaf_mfma_ok(const Geom& g, long long cstride) {
#ifdef PP2_LEAF_FMAF
  return false;  // diagnostic A/B builds only: the fmaf pass everywhere
#endif
  return g.wp % 8 == 0 && cstride % 8 == 0;
}
long long rollout_leaf_ldb(const Geom& g) {
  const long long n = (long long)g.rows * g.wp;
  return (n + kLeafSlab - 1) / kLeafSlab * kLeafSlab;
}
size_t rollout_leaf_scratch_bytes(const Geom& g, int ncopies) {
  const long long ldb = rollout_leaf_ldb(g), nslab = ldb / kLeafSlab;
  return (size_t)kLeafColsPad * ldb * sizeof(_Float16) + 9 * kLeafParts * sizeof(float) + 64 +
         (size_t)ncopies * kLeafCols * nslab * sizeof(float);
}

hipError_t launch_rollout_leaf_mfma(hipStream_t st, const Geom& g, PlaneSet F, const void* b,
                                    long long cstride, int ncopies, void* scratch, float* out,
                                    bool pack) {
  const long long ldb = rollout_leaf_ldb(g), nslab = ldb / kLeafSlab;
  _Float16* B = reinterpret_cast<_Float16*>(scratch);
  float* amax = reinterpret_cast<float*>(B + (size_t)kLeafColsPad * ldb);
  int* kexp = reinterpret_cast<int*>(amax + 9 * kLeafParts);
  float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(kexp) + 64);
  if (pack) {  // (B and the scales of the same alphas are still in the scratch otherwise)
    hipLaunchKernelGGL(k_leaf_alpha_max, dim3(kLeafParts, 9), dim3(256), 0, st, g, F, amax);
    const unsigned pb = (unsigned)std::min<long long>((ldb + 255) / 256, 1024);
    hipLaunchKernelGGL(k_leaf_alpha_pack, dim3(pb), dim3(256), 0, st, g, F, amax, B, ldb, kexp);
  }
  hipLaunchKernelGGL(k_rollout_leaf_mfma, dim3((unsigned)nslab, (unsigned)((ncopies + 63) / 64)),
                     dim3(64), 0, st, (const _Float16*)b + g.wp, (const _Float16*)b, cstride,
                     ncopies, (long long)g.rows * g.wp, B, ldb, part, (int)nslab);
  hipLaunchKernelGGL(k_rollout_leaf_mfma_reduce, dim3(ncopies), dim3(64), 0, st, part, (int)nslab,
                     ncopies, kexp, out);
  return hipGetLastError();
}

}  // namespace pp2
