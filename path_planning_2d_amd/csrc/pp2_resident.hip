// pp2_resident.hip -- the tile-resident loop (gfx950): a run of n north-star
// steps (belief update + MDP Bellman sweep, k_loop_step's semantics) in ONE
// launch, for the unsharded sparse-coded context.
//
// Per launch of the one-step / step-pair kernels the grid pays a dependent
// kernel boundary, a dictionary staging, an HBM round trip of b and J and a
// lock-stepped load -> gather -> backup -> store chain with nothing to overlap
// it (pairs also recompute a one-row halo: 1.5x step-1 work at 1024^2).  Here
// every CU keeps ONE tile of rt whole rows resident for the whole run:
//   * the tile's b and J live in LDS (ping-pong buffers with zero pads at
//     the x edges); the dictionary (factored sweep rows, T_u of all 9
//     actions, L_z of all 16 observations) is staged once per launch;
//   * a lane owns one quad of 4 cells and keeps its code window in registers;
//   * only the tile's first and last rows cross CUs.  Their waves take the
//     neighbours' rows of step t-1 first (poll the data-tagged granules of
//     the neighbour waves over their columns with sc1 loads until every tag
//     matches), compute with issue priority and store their own row as
//     granules (one sc1 store each) into an exchange slot (step & 1): the
//     data is the flag, so no drain and no separate flag (MI355X_MICROARCH.md
//     § visibility, handoff-1to1).  A producer rewrites a slot only after it
//     took the consumer's granules of the following step, i.e. after the
//     consumer's loads of it have returned.  Interior waves never touch
//     global memory;
//   * a normalisation block start needs the exact mass of the previous belief:
//     every tile adds to an arrival counter after its step's wave partials are
//     drained, and wave 0 of each tile reduces all partials (k_sum_finalize's
//     tree, sc1 loads) once the counter is full.  The partials of step t go to
//     ring slot t % kResidentRing (no tile runs more than one block ahead of
//     the slowest, so a slot is never rewritten while a block start reads it);
//   * the last step stores b, J and A for the whole grid (non-temporal) and its
//     partials to the context's pending buffer -- b and J into the OTHER
//     ping-pong buffers, so the run's inputs survive it.
// Per cell the arithmetic is k_loop_step_coded's (same operands, same fmaf
// order; off-grid neighbours are +0 from the pads, and fmaf(T, +0, p) == p
// for the finite T resident_plan's caller checks), the partials use the dense
// kernels' cell -> (block, wave) map, and normalisation follows
// blocked_loop_step exactly, so b, masses, J and A equal the
// one-launch-per-step path bit for bit.
//
// Row shards run the same kernel on a view: the owned rows
// plus e halo rows per side, refreshed e deep before the launch, for n <= e
// steps (the rows outside the view read as 0, so the view's outer rows go
// stale one row per step and never reach the owned ones).  Only owned rows
// store b', J', A and give the final mass partials.  Block starts inside the
// run scale the belief by a power of two chosen from the mass of the whole
// view (every cell is <= it, so no halo row can overflow), summed into
// *scale_out; the host rebases every shard to a common power of two at the
// next halo exchange (launch_shard_rebase), where the global mass is known.
//
// Hand-off safety (MI355X_MICROARCH.md § visibility): every granule is ONE
// 16-B sc1 store of four values, each 4-B word carrying the slot use's tag
// bit in its (otherwise zero) sign bit, so the check holds at single-copy
// atomic granularity whatever the store tears into; every granule is consumed
// by sc1 loads only; the mass partials go out as sc1 stores drained before
// one lane's counter add (the guide's table, row 1).  Slot uses and arrival
// counters continue over the context's launches (host-side counts), so no
// per-launch reset is needed.  Every wait is bounded: after kSpinTicks of the
// 100 MHz clock it raises the sticky error word (and the pinned host word)
// and returns, so a grid that is not fully resident ends with an error
// instead of hanging; the host then re-runs the launch from its intact inputs
// with the launch-per-step kernels (pp2_runtime.cpp resident_settle).  A
// launch queued behind an unverified one reads the error word first and
// exits before any global store if it is raised (the host re-runs it too).
#include <algorithm>
#include <cstring>

#include "pp2_coded_dev.h"

namespace pp2 {

#ifdef PP2_RES_TRACE
// Diagnostic build only (tools/micro/resident_trace.py): s_memrealtime
// (100 MHz) per step of tiles 0..15 for waves 0, 5, 9 and 12 (rows 0..3 at
// 1024^2): step top, window rows in hand, computed and published, after the
// step barrier.
__device__ unsigned long long g_rtrace[16][64][4][4];
#define PP2_RT(ph)                                                                    \
  if (tile < 16 && t < 64 && lane == 0 && (wave == 0 || wave == 5 || wave == 9 || wave == 12)) \
  g_rtrace[tile][t][wave == 0 ? 0 : wave == 5 ? 1 : wave == 9 ? 2 : 3][ph] =          \
      __builtin_amdgcn_s_memrealtime()
// prologue / epilogue of every tile (wave 0): entry, tables staged, loop top,
// outputs stored; class planes built, tile loaded + published, mass reduced
__device__ unsigned long long g_rtrace_pro[1024][8];
#define PP2_RP(ph) \
  if (tile < 1024 && threadIdx.x == 0) g_rtrace_pro[tile][ph] = __builtin_amdgcn_s_memrealtime()
#else
#define PP2_RT(ph) (void)0
#define PP2_RP(ph) (void)0
#endif

namespace {

typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
constexpr int kSc1 = 16;                              // buffer aux bit: sc1
constexpr unsigned long long kSpinTicks = 25000000ull;  // 0.25 s at 100 MHz
constexpr int kPrologueParts = 4096;  // pending partials reduced from registers

__device__ __forceinline__ Rsrc make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ f4a ld4_sc1(Rsrc r, int off) {
  return __builtin_bit_cast(f4a, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
}
__device__ __forceinline__ float ld1_sc1(Rsrc r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSc1));
}
__device__ __forceinline__ unsigned ld_flag(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool reached(unsigned v, unsigned target) {
  return (int)(v - target) >= 0;  // epoch arithmetic, wrap-safe
}
// Raise the sticky error word (polled by every wait) and the pinned host word
// the host reads after the launch (a vector store over the fabric).
__device__ __forceinline__ void raise_err(unsigned* err, unsigned* err_host) {
  st_flag(err, 1u);
  if (err_host) __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The calling wave waits until flag[idx(i)] has reached target for every lane
// i < nf (lane i polls one word; relaxed sc1 loads, s_sleep between polls).
// Bounded: gives up after kSpinTicks (or at once when the error word is
// already raised), raising it.  The wavefront acquire only keeps the compiler
// from moving the caller's later (sc1) loads above the poll.
__device__ __forceinline__ bool wave_wait(const unsigned* f0, int nf, unsigned target, unsigned* err,
                                          unsigned* err_host) {
  const int lane = threadIdx.x & 63;
  const unsigned long long t0 = wall_clock64();
  for (int spin = 0;; ++spin) {
    const unsigned v = lane < nf ? ld_flag(f0 + lane) : target;
    if (__all(reached(v, target))) break;
    if ((spin & 7) == 7) {
      if (ld_flag(err) != 0u || wall_clock64() - t0 > kSpinTicks) {
        if (lane == 0) raise_err(err, err_host);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return true;
}

// Shard block starts inside a run: the power-of-two shift that brings the
// shard's owned mass S into [2^96, 2^97) (0 for S == 0 or non-finite; at most
// 127, so 2^shift is a normal float and no value overflows: every cell is
// <= S).  Multiplying by 2^shift is exact, so shards that pick different
// shifts are rebased exactly later (launch_shard_rebase).
__device__ __forceinline__ int pow2_shift(float S) {
  if (!(S > 0.0f) || !(S < FLT_MAX)) return 0;
  const int e = (int)((__float_as_uint(S) >> 23) & 0xffu) - 127;  // ilogb (S is normal: FTZ)
  const int sh = 96 - e;
  return sh < 0 ? 0 : sh > 127 ? 127 : sh;
}
__device__ __forceinline__ float pow2f(int k) { return __uint_as_float((uint32_t)(127 + k) << 23); }
// Lagged shard block starts (shard mode 2): the shift at block start t is
// chosen from X = S * 2^prev, S the view's mass of step t-1-depth (before the
// previous block start's shift prev): the mass only decreases (T is
// column-stochastic over the view, L <= 1, rows outside the view read 0), so
// X bounds the mass of step t-1 and the scaled mass stays below 2^121 --
// it lands in [2^120 * (decay over depth steps), 2^121).  The target 2^120
// (not 2^96) keeps the headroom of the non-lagged scheme over the up to
// 2 x depth steps of decay between two such shifts.
__device__ __forceinline__ int pow2_shift_lagged(float S, int prev) {
  if (!(S > 0.0f) || !(S < FLT_MAX)) return 0;
  const int e = (int)((__float_as_uint(S) >> 23) & 0xffu) - 127;
  const int sh = 120 - e - prev;
  return sh < 0 ? 0 : sh > 127 ? 127 : sh;
}

// wave_reduce_partials (pp2_device.h) with sc1 loads: the partials were
// stored by other CUs inside this launch.  Same association, bit for bit.
// kRedQ quads per lane in flight per round trip.
#ifndef PP2_REDQ
#define PP2_REDQ 8
#endif
constexpr int kRedQ = PP2_REDQ;
__device__ __forceinline__ float wave_reduce_partials_sc1(const float* p, int n) {
  const Rsrc r = make_rsrc(p);
  const int lane = threadIdx.x & 63;
  const int nq = n >> 2;
  float s = 0.0f;
  for (int base = lane; base < nq; base += 64 * kRedQ) {
    f4a w[kRedQ];
#pragma unroll
    for (int j = 0; j < kRedQ; ++j) {
      const int i = base + 64 * j;
      w[j] = ld4_sc1(r, 16 * (i < nq ? i : base));
    }
#pragma unroll
    for (int j = 0; j < kRedQ; ++j)
      if (base + 64 * j < nq) s += ((w[j][0] + w[j][1]) + w[j][2]) + w[j][3];
  }
  return wave_sum(s);
}

// The coded belief gather of action U for a lane's quad (belief_vals'
// arithmetic, the same fmaf order) by classes: the raw T of a source cell x'
// for action U is QR[U][class of x' for U][slot], the class byte offset (16 *
// class) read from the tile's plane of action U (rows ty-1 .. ty+1 at plane
// rows ty .. ty+2; x0-1 / x0+4 from the neighbour lanes' dwords by DPP wave
// shifts, lanes 0 / 63 read those dwords themselves), and L_z of the cell is
// LT[z][L class] with the 4 * class bytes of the lane's cells in lx4.  Every
// table read hits a <= 16-entry table (no bank conflicts), where code-indexed
// reads of 274-entry tables collide.  The window's off-grid cells are 0: the
// LDS rows carry zero pads and off-grid plane bytes are class 0, whose
// (finite, the host checks) T multiplies b = +0, and fmaf(T, +0, p) == p for
// the non-negative partial sums.
// TR (transposed tiles): the kernel's rows are the grid's columns, so the
// source cell at grid offset (oy - 1, ox) sits in window row ox + 1, window
// column k + oy of the lane's quad cell k; the terms keep the grid's
// ascending-s order (the same fmaf chain).
template <bool TR>
constexpr bool belief_row_used(int U, int r) {
  for (int s = 0; s < 9; ++s)
    if ((TR ? s % 3 : s / 3) == r && sup_slot(U, 8 - s) >= 0) return true;
  return false;
}
template <int U, bool TR>
__device__ __forceinline__ void belief_fact(const uint8_t* prow, int ps, int x0, uint32_t lx4,
                                            int z, const Win6& win, float (&p)[4]) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const char* qr = reinterpret_cast<const char*>(lds + kResQR) + U * kFactK * 16;
  const char* lt = reinterpret_cast<const char*>(lds + kResLT) + z * (kResLK * 4);
  const int lane = threadIdx.x & 63;
  // per window row: the class bytes of x0-1 .. x0+4
  uint32_t cb[3][6];
#pragma unroll
  for (int oy = 0; oy < 3; ++oy) {
    if (!belief_row_used<TR>(U, oy)) continue;
    const uint8_t* r = prow + oy * ps + 4 + x0;
    const uint32_t m = *reinterpret_cast<const uint32_t*>(r);
    uint32_t e = 0u;
    if (lane == 0 || lane == 63) e = *reinterpret_cast<const uint32_t*>(r + (lane == 0 ? -4 : 4));
    const uint32_t l = (uint32_t)__builtin_amdgcn_update_dpp((int)e, (int)m, 0x138, 0xf, 0xf, false);
    const uint32_t h = (uint32_t)__builtin_amdgcn_update_dpp((int)e, (int)m, 0x130, 0xf, 0xf, false);
    cb[oy][0] = l >> 24;
    cb[oy][1] = m & 0xffu;
    cb[oy][2] = __builtin_amdgcn_ubfe(m, 8, 8);
    cb[oy][3] = __builtin_amdgcn_ubfe(m, 16, 8);
    cb[oy][4] = m >> 24;
    cb[oy][5] = h & 0xffu;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = 0.0f;
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    // window row and column offset of grid offset s
    const int wr = TR ? s % 3 : s / 3, wc = TR ? s / 3 - 1 : s % 3 - 1;
    const int sl = sup_slot(U, 8 - s);
    if (sl < 0) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      p[k] = __builtin_fmaf(*reinterpret_cast<const float*>(qr + 4 * sl + cb[wr][k + 1 + wc]),
                            win.v[wr][k + 1 + wc], p[k]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    p[k] = p[k] * *reinterpret_cast<const float*>(lt + __builtin_amdgcn_ubfe(lx4, 8 * k, 8));
}

// The register-rich 2-D instance (TC = 3) holds the lane's class bytes of
// every used window row of every action in registers for the whole run (the
// class planes are static): per (action, row) the lane's own dword m and
// the two neighbour bytes lh (x0 - 1 in bits 0-7, x0 + 4 in bits 8-15), so
// the gather's table reads issue at the step's top, without the class-byte
// LDS round trip before them.  Slots in (action, row) order.
#ifndef PP2_RES_HOIST
#define PP2_RES_HOIST 1  // (A/B builds: 0 keeps the LDS class reads in the TC = 3 instance)
#endif
struct ClsSlots {
  int s[9][3];
  int n;
  constexpr ClsSlots() : s{}, n(0) {
    for (int u = 0; u < 9; ++u)
      for (int r = 0; r < 3; ++r) s[u][r] = belief_row_used<false>(u, r) ? n++ : -1;
  }
};
constexpr ClsSlots kCls{};
constexpr int kClsSlots = kCls.n;
struct ClassRegs {
  uint32_t m[kClsSlots], lh[(kClsSlots + 1) / 2];  // lh: two slots per dword
};
template <int U>
__device__ __forceinline__ void belief_fact_regs(const ClassRegs& cr, uint32_t lx4, int z,
                                                 const Win6& win, float (&p)[4]) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const char* qr = reinterpret_cast<const char*>(lds + kResQR) + U * kFactK * 16;
  const char* lt = reinterpret_cast<const char*>(lds + kResLT) + z * (kResLK * 4);
  uint32_t cb[3][6];
#pragma unroll
  for (int oy = 0; oy < 3; ++oy) {
    const int sl = kCls.s[U][oy];
    if (sl < 0) continue;
    const uint32_t m = cr.m[sl], lh = cr.lh[sl / 2] >> (16 * (sl & 1));
    cb[oy][0] = lh & 0xffu;
    cb[oy][1] = m & 0xffu;
    cb[oy][2] = __builtin_amdgcn_ubfe(m, 8, 8);
    cb[oy][3] = __builtin_amdgcn_ubfe(m, 16, 8);
    cb[oy][4] = m >> 24;
    cb[oy][5] = __builtin_amdgcn_ubfe(lh, 8, 8);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = 0.0f;
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const int wr = s / 3, wc = s % 3 - 1;
    const int sl = sup_slot(U, 8 - s);
    if (sl < 0) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      p[k] = __builtin_fmaf(*reinterpret_cast<const float*>(qr + 4 * sl + cb[wr][k + 1 + wc]),
                            win.v[wr][k + 1 + wc], p[k]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    p[k] = p[k] * *reinterpret_cast<const float*>(lt + __builtin_amdgcn_ubfe(lx4, 8 * k, 8));
}
__device__ __forceinline__ void belief_any_regs(int u, const ClassRegs& cr, uint32_t lx4, int z,
                                                const Win6& w, float (&p)[4]) {
  switch (u) {
#define PP2_BQ(UU)                               \
  case UU:                                       \
    belief_fact_regs<UU>(cr, lx4, z, w, p);      \
    break;
    PP2_BQ(0) PP2_BQ(1) PP2_BQ(2) PP2_BQ(3) PP2_BQ(4) PP2_BQ(5) PP2_BQ(6) PP2_BQ(7)
    default: belief_fact_regs<8>(cr, lx4, z, w, p);
#undef PP2_BQ
  }
}
// the lane's class dwords of plane rows ty .. ty + 2 (window rows 0 .. 2)
// (an odd slot count leaves the last lh dword's high half 0)
__device__ __forceinline__ void load_class_regs(const uint8_t* sP, int prows, int ps, int ty,
                                                int x0, ClassRegs& cr) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int U = 0; U < 9; ++U)
#pragma unroll
    for (int oy = 0; oy < 3; ++oy) {
      const int sl = kCls.s[U][oy];
      if (sl < 0) continue;
      const uint8_t* r = sP + (U * prows + ty + oy) * ps + 4 + x0;
      const uint32_t m = *reinterpret_cast<const uint32_t*>(r);
      uint32_t e = 0u;
      if (lane == 0 || lane == 63) e = *reinterpret_cast<const uint32_t*>(r + (lane == 0 ? -4 : 4));
      const uint32_t l = (uint32_t)__builtin_amdgcn_update_dpp((int)e, (int)m, 0x138, 0xf, 0xf, false);
      const uint32_t h = (uint32_t)__builtin_amdgcn_update_dpp((int)e, (int)m, 0x130, 0xf, 0xf, false);
      cr.m[sl] = m;
      const uint32_t lh = (l >> 24) | ((h & 0xffu) << 8);
      cr.lh[sl / 2] = (sl & 1) ? cr.lh[sl / 2] | (lh << 16) : lh;
    }
}

// sP: the tile's class planes [9][rt + 2][ps] (ps = wp + 8 bytes: 4 pad
// bytes on each side); this lane's rows start at plane row ty.
// p = the gathered quad times L_z (the block-start scale and the mass
// partial are applied by the caller)
template <bool TR>
__device__ __forceinline__ void belief_any(int u, const uint8_t* sP, int prows, int ps, int ty,
                                           int x0, uint32_t lx4, int z, const Win6& w,
                                           float (&p)[4]) {
  // The plane rows of action u, from the step's u through an opaque (not
  // volatile) asm: otherwise the compiler specialises the address per case
  // and hoists the 9 actions x 3 rows of plane addresses out of the step loop
  // into 27 VGPRs (and spills).
  int off = (u * prows + ty) * ps;
  asm("" : "+v"(off));
  const uint8_t* pu = sP + off;
  switch (u) {
#define PP2_BQ(UU)                                                     \
  case UU:                                                             \
    belief_fact<UU, TR>(pu, ps, x0, lx4, z, w, p); \
    break;
    PP2_BQ(0) PP2_BQ(1) PP2_BQ(2) PP2_BQ(3) PP2_BQ(4) PP2_BQ(5) PP2_BQ(6) PP2_BQ(7)
    default: belief_fact<8, TR>(pu, ps, x0, lx4, z, w, p);
#undef PP2_BQ
  }
}

// One window row (x0 - 1 .. x0 + 4) from a zero-padded LDS row: the lane's
// aligned 16 B, and x0 - 1 / x0 + 4 from the neighbouring lanes' quads by DPP
// wave shifts (wave_shr:1 / wave_shl:1; a wave holds 64 consecutive quads of
// one row).  Lanes 0 and 63 have no source lane and keep the DPP's `old`
// operand, the edge dword they read themselves (one 2-lane ds_read_b32 --
// every lane reading its own edge dwords, at a 16-B lane stride, costs a
// 4-way bank conflict per read).
__device__ __forceinline__ void row_lds(const float* row, int x0, float (&v)[6]) {
  const float* p = row + x0;
  const f4a m = *reinterpret_cast<const f4a*>(p);
  const int lane = threadIdx.x & 63;
  float e = 0.0f;
  if (lane == 0 || lane == 63) e = p[lane == 0 ? -1 : 4];
  v[0] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(e), __float_as_int(m[3]),
                                                    0x138, 0xf, 0xf, false));
  v[1] = m[0]; v[2] = m[1]; v[3] = m[2]; v[4] = m[3];
  v[5] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(e), __float_as_int(m[0]),
                                                    0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ void row_zero(float (&v)[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) v[i] = 0.0f;
}

// Edge-row hand-off by self-tagged words (MI355X_MICROARCH.md § visibility,
// handoff-1to1: the data is the flag).  Every value handed over -- belief and
// J -- is finite and >= +0 (the coded path's preconditions, pp2_runtime.cpp
// build_model_dict / pp2_belief_set), so bit 31 of its word is free: it
// carries the TAG BIT of the slot use, and every 4-B word validates itself
// (a 4-B aligned access is single-copy atomic, so no tearing of a granule --
// the guide observes 16-B sc1 stores untorn only per 8-B half -- can pass the
// check).  A lane's b and J quads go out as two 16-B granules, {b0..b3} and
// {j0..j3}, each ONE sc1 (write-through) store; the consumer polls them with
// sc1 loads until every word carries the expected bit -- no drain, no flag,
// one fabric round trip per hand-off, half the words of a {value, tag}
// format.  One bit suffices: a slot holds either its previous use (already
// consumed) or the current one, never older -- a producer rewrites a slot
// only after it took the consumer's granules of the following step, i.e.
// after the consumer's loads of the earlier use returned -- and the host
// numbers the uses of each slot continuously over the context's launches
// (slot_use), so consecutive uses alternate the bit; a fresh buffer is zero,
// which no first use (bit 1) matches.  Layout: [slot][tile][top, bottom][wave
// of the row][granule k < 2][lane], so a wave's k-th store and load cover
// 1 KiB contiguously; the sweep kernel uses granule 0 alone.
__device__ __forceinline__ int xch_gran(int ntiles, int wpr, int slot, int tl, int side, int w,
                                        int k, int ln) {
  return (((((slot * ntiles + tl) * 2 + side) * wpr + w) * kResidentGranules + k) * 64 + ln) * 16;
}
// Same-XCD hand-offs (PP2_RES_XCD_PLAIN): a plain store keeps the line in
// the XCD's L2, so the neighbour's sc1 (L1-bypassing, L2-served) loads take
// it there, where an sc1 store drops it and the reader fetches it over the
// fabric (MI355X_MICROARCH.md, visibility table).  Only where every reader
// of the granule runs on the producer's XCD: the tile -> XCD map of
// xcd_remap (block b on XCD b % 8 owns a contiguous range of tiles).
#ifndef PP2_RES_XCD_PLAIN
#define PP2_RES_XCD_PLAIN 1
#endif
#ifndef PP2_RES_XCD_AUX
#define PP2_RES_XCD_AUX 0  // the same-XCD stores' cache policy (0 plain, 1 sc0, 2 nt)
#endif
__device__ __forceinline__ int tile_xcd(int t, int n) {
  const int q = n / 8, r = n % 8;
  return t < r * (q + 1) ? t / (q + 1) : r + (q > 0 ? (t - r * (q + 1)) / q : 0);
}
__device__ __forceinline__ void st_quad_x(Rsrc r, int off, const float (&v)[4], unsigned bit,
                                          bool plain) {
  const unsigned m = bit << 31;
  const u4v t = {__float_as_uint(v[0]) | m, __float_as_uint(v[1]) | m, __float_as_uint(v[2]) | m,
                 __float_as_uint(v[3]) | m};
  if (plain) __builtin_amdgcn_raw_buffer_store_b128(t, r, off, 0, PP2_RES_XCD_AUX);
  else __builtin_amdgcn_raw_buffer_store_b128(t, r, off, 0, kSc1);
}
__device__ __forceinline__ bool tagged(const u4v& g, unsigned m) {
  return (((g[0] ^ m) | (g[1] ^ m) | (g[2] ^ m) | (g[3] ^ m)) >> 31) == 0u;
}
__device__ __forceinline__ float untag(unsigned w) { return __uint_as_float(w & 0x7fffffffu); }
// The wave polls granules g[k] at o + 1 KiB * k and (edge lanes) the single
// words e[k] at eo + 1 KiB * k until every word carries tag bit `bit`.
// Bounded like wave_wait; the empty asm keeps the loads inside the loop.
template <int NG>
__device__ __forceinline__ void take_granules(Rsrc r, int o, bool edge, int eo, unsigned bit,
                                              u4v (&g)[NG], unsigned (&e)[NG], unsigned* err,
                                              unsigned* err_host) {
  const unsigned m = bit << 31;
  const unsigned long long t0 = wall_clock64();
#pragma unroll
  for (int k = 0; k < NG; ++k) e[k] = m;
  for (int spin = 0;; ++spin) {
#pragma unroll
    for (int k = 0; k < NG; ++k) g[k] = __builtin_amdgcn_raw_buffer_load_b128(r, o + 1024 * k, 0, kSc1);
    if (edge) {
#pragma unroll
      for (int k = 0; k < NG; ++k) e[k] = __builtin_amdgcn_raw_buffer_load_b32(r, eo + 1024 * k, 0, kSc1);
    }
    bool ok = true;
#pragma unroll
    for (int k = 0; k < NG; ++k) ok = ok && tagged(g[k], m) && ((e[k] ^ m) >> 31) == 0u;
    if (__all(ok)) break;
    if ((spin & 7) == 7) {
      if (ld_flag(err) != 0u || wall_clock64() - t0 > kSpinTicks) {
        if ((threadIdx.x & 63) == 0) raise_err(err, err_host);
        return;
      }
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
  }
}
// 2-D tiles (tc > 1): a tile's first and last columns cross CUs as well.  The
// lane holding the first (last) cell of a row publishes {b, j} of that cell as
// ONE 8-B sc1 store (both words tagged, like the granules) into side granule
// [slot][tile][0 (first column) / 1 (last)][row], after the top / bottom
// region; the side lane of the neighbour tile takes the cells of its rows
// ty-1 .. ty+1 from it (rows -1 / rt from the diagonal tiles' rows rt-1 / 0,
// so the corners need no granule of their own).  The slot discipline is the
// granules': a producer rewrites a side slot only after it took the consumer's
// side cells of the following step, which that consumer published after its
// loads of the slot returned (the same wave polls, computes and publishes).
typedef unsigned u2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int side_gran(int sbase, int ntiles, int slot, int tl, int side, int r) {
  return sbase + (((slot * ntiles + tl) * 2 + side) * kResidentMaxRt + r) * 8;
}
__device__ __forceinline__ void st_pair(Rsrc r, int off, float b, float j, unsigned bit) {
  const unsigned m = bit << 31;
  const u2v t = {__float_as_uint(b) | m, __float_as_uint(j) | m};
  __builtin_amdgcn_raw_buffer_store_b64(t, r, off, 0, kSc1);
}
// take_granules<2> (when rows) and, on the wave's side lane (sd), the side
// cells at so[k] (k: rows ty-1 .. ty+1; < 0: off the grid, read as 0) in the
// same polls, so the two hand-offs cost one round trip.
__device__ __forceinline__ void take_rows_sides(Rsrc r, bool rows, int o, bool edge, int eo,
                                                bool sd, const int (&so)[3], int soff, unsigned bit,
                                                u4v (&g)[2], unsigned (&e)[2], u2v (&s)[3],
                                                unsigned* err, unsigned* err_host) {
  const unsigned m = bit << 31;
  const unsigned long long t0 = wall_clock64();
  e[0] = e[1] = m;
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = u2v{m, m};
#ifdef PP2_RES_NOXCH
  // diagnostic build only (tools/micro/resident_nowait.sh): no hand-off
  // loads at all -- the neighbours' rows read as tagged zeros
  g[0] = g[1] = u4v{m, m, m, m};
  return;
#endif
  for (int spin = 0;; ++spin) {
    if (rows) {
      g[0] = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, kSc1);
      g[1] = __builtin_amdgcn_raw_buffer_load_b128(r, o + 1024, 0, kSc1);
      if (edge) {
        e[0] = __builtin_amdgcn_raw_buffer_load_b32(r, eo, 0, kSc1);
        e[1] = __builtin_amdgcn_raw_buffer_load_b32(r, eo + 1024, 0, kSc1);
      }
    }
    if (sd) {
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (so[k] >= 0) s[k] = __builtin_amdgcn_raw_buffer_load_b64(r, so[k], soff, kSc1);
    }
    bool ok = true;
    if (rows)
      ok = tagged(g[0], m) && tagged(g[1], m) && (((e[0] ^ m) | (e[1] ^ m)) >> 31) == 0u;
#pragma unroll
    for (int k = 0; k < 3; ++k) ok = ok && (((s[k][0] ^ m) | (s[k][1] ^ m)) >> 31) == 0u;
#ifdef PP2_RES_NOWAIT
    ok = true;  // diagnostic build only (tools/micro/resident_nowait.sh): no hand-off waits
#endif
    if (__all(ok)) break;
    if ((spin & 7) == 7) {
      if (ld_flag(err) != 0u || wall_clock64() - t0 > kSpinTicks) {
        if ((threadIdx.x & 63) == 0) raise_err(err, err_host);
        return;
      }
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
  }
}
// One window row from the lane's aligned quad m and the edge dword e of the
// lane's wave-edge neighbour (lanes 0 / 63), the others by DPP wave shifts.
__device__ __forceinline__ void row_quad(const float (&m)[4], float e, float (&v)[6]) {
  v[0] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(e), __float_as_int(m[3]),
                                                    0x138, 0xf, 0xf, false));
  v[1] = m[0]; v[2] = m[1]; v[3] = m[2]; v[4] = m[3];
  v[5] = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(e), __float_as_int(m[0]),
                                                    0x130, 0xf, 0xf, false));
}

template <int CAP>
struct Trajectory {
  uint8_t uz[CAP];  // u | z << 4 per step
};

// TC: tile columns (a compile-time constant, so the whole-row instance has no
// side-lane code at all); LAG: shard mode 2's lagged block starts (their own
// instances, so that the unsharded loop carries none of their state); TR:
// transposed tiles (shard views, TC = 1): the kernel's grid is the view
// transposed -- its rows are the grid's columns (a.g.rows = the grid's row
// stride), its columns the view's rows (a.g.wp = the view's row count) -- so
// a tile is a strip of rt grid columns spanning the whole view and only its
// first and last columns cross CUs; HBM stays in the grid's layout (row
// stride a.ows), read and written transposed once per launch.
// TC = 3: the 2-D tiling (2 tile columns) with at most 768 threads -- 3 waves
// per SIMD, so a 168-VGPR budget instead of 128: the sweep's table reads of
// all 4 cells of an action in flight together (coded_sweep_iw G = 4).
template <int CAP, int TC, bool LAG, bool TR>
__global__ __launch_bounds__(TC == 3 ? 768 : 1024, TC == 3 ? 3 : 4) void k_loop_resident(
    const ResidentHead a, const Trajectory<CAP> tr) {
  static_assert(!TR || TC == 1, "transposed tiles are whole kernel rows");
  constexpr int kSweepG = TC == 3 ? 4 : TC > 1 ? 2 : 0;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // a tile: rt rows x tw columns (tc tile columns per row of tiles)
  constexpr int tc = TC == 3 ? 2 : TC;
  const int wp = a.g.wp, rows = a.g.rows, tw = wp / tc;
  const int tpr = tw >> 2, wpr = tw >> 8;  // lanes, waves per tile row
  const int xs = tw + 4;                // padded LDS row stride
  const int bufn = 4 + a.rt * xs;       // one padded tile buffer
  // LDS: class tables (QR, LT: constant offsets), factored sweep rows (QT, CT:
  // constant offsets; IW), class planes, b buffers 0, 1, J buffers 0, 1
  const int prows = a.rt + 2, ps = tw + 8;
  float* sTC = lds + lds_span(kResTab);  // (stage_rows writes up to the span)
  uint8_t* sP = reinterpret_cast<uint8_t*>(sTC + lds_span(rows_floats(a.E, true)));
  float* sB0 = reinterpret_cast<float*>(sP) + lds_span(9 * prows * ps / 4);
  float* sS = sB0 + 4 * bufn;
  float* sRed = sS + 16;  // (red_lds) the lagged block start's partials

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  if (tile == a.stall_tile) return;  // diagnostic: a tile that never arrives
  const int trow = tile / tc, cx = tile - trow * tc, gx = cx * tw;  // tile row, column, x
  PP2_RP(0);
  // a chained launch after one that timed out does nothing: its inputs are
  // that launch's garbage outputs (resident_settle re-runs both)
  const unsigned prior_err = ld_flag(a.sync + kResidentSyncErr);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // wave-uniform: a row holds wpr whole waves (wp % 256 == 0)
  const int ty = __builtin_amdgcn_readfirstlane(threadIdx.x / tpr);
  // 2-D tiles: a row's column waves rotate with the row, so that the side
  // waves (which wait on a neighbour tile) of consecutive rows land on
  // different SIMDs (wave w runs on SIMD w % 4) instead of all on one
  const int wraw = __builtin_amdgcn_readfirstlane((threadIdx.x % tpr) >> 6);
  const int wj = tc > 1 ? __builtin_amdgcn_readfirstlane((wraw + ty) % wpr) : wraw;
  const int x0 = wj * 256 + lane * 4;  // (tile-relative)
  const int y = trow * a.rt + ty;
  const bool valid = y < rows;
  // (a shard's view: owned rows only -- TR: the quad's grid rows x0 .. x0+3,
  // own0 / own1 multiples of 4)
  const bool own = TR ? x0 >= a.own0 && x0 < a.own1 : y >= a.own0 && y < a.own1;
  // HBM offset of kernel cell (yy, xx) (view row 0 = kernel column 0)
  auto hoff = [&](int yy, int xx) -> long long {
    return TR ? (long long)xx * a.ows + yy : (long long)yy * wp + xx;
  };
  // the tile's first row reads the row above from tile - tc and publishes
  // itself for it; its last row likewise with tile + tc
  const bool nb_up = valid && ty == 0 && trow > 0;
  const bool nb_dn = valid && ty == a.rt - 1 && y + 1 < rows;
  // 2-D tiles: the first wave of a row takes / publishes the left neighbour's
  // side cells on lane 0, the last wave the right one's on lane 63 (wpr >= 2:
  // never both in one wave)
  const bool sd_l = valid && wj == 0 && cx > 0;
  const bool sd_r = valid && wj == wpr - 1 && cx + 1 < tc;
  const bool sd_lane = (sd_l && lane == 0) || (sd_r && lane == 63);
  const int sbase = 2 * a.ntiles * 2 * (wp >> 8) * kResidentGranules * 64 * 16;  // side region
  unsigned* const err = a.sync + kResidentSyncErr;
  const Rsrc rx = make_rsrc(a.xch);
  auto sbuf = [&](int k, int slot) { return sB0 + (2 * k + slot) * bufn + 4; };
  // the boundary waves' hand-off: b and J of the lane's quad as two
  // self-tagged granules {b0..b3}, {j0..j3} in exchange slot `slot`
  // (whether the row granules' reader, tile -+ tc, shares this tile's XCD)
  const int myx = tile_xcd(tile, (int)gridDim.x);
  const bool plain_up = PP2_RES_XCD_PLAIN && nb_up && tile_xcd(tile - tc, (int)gridDim.x) == myx;
  const bool plain_dn = PP2_RES_XCD_PLAIN && nb_dn && tile_xcd(tile + tc, (int)gridDim.x) == myx;
  auto publish = [&](int slot, const float (&b)[4], const float (&j)[4], unsigned bit) {
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      if (side == 0 ? !nb_up : !nb_dn) continue;
      const int o = xch_gran(a.ntiles, wpr, slot, tile, side, wj, 0, lane);
      const bool plain = side == 0 ? plain_up : plain_dn;
      st_quad_x(rx, o, b, bit, plain);
      st_quad_x(rx, o + 1024, j, bit, plain);
    }
    if (sd_lane) {
      const int o = side_gran(sbase, a.ntiles, slot, tile, sd_l ? 0 : 1, ty);
      if (sd_l) st_pair(rx, o, b[0], j[0], bit);
      else st_pair(rx, o, b[3], j[3], bit);
    }
  };
  // ... and the neighbour's row (tile tl, side) of the slot use with tag bit
  // `bit`: poll its granules over this wave's columns (lanes 0 / 63 also the
  // neighbour waves' edge cells) until every word carries the bit
  // The side lane's granules of rows ty-1 .. ty+1 in slot 0 (rows -1 / rt from
  // the diagonal tiles; < 0 off the grid): fixed for the run, the slot's
  // offset goes in the loads' scalar offset.
  int so[3] = {-1, -1, -1};
  if (tc > 1 && sd_lane) {
    const int dir = sd_l ? -1 : 1, nside = sd_l ? 1 : 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int rr = ty + k - 1, yy = y + k - 1;
      if (yy < 0 || yy >= rows) continue;
      const int tl2 = rr < 0 ? tile - tc + dir : rr >= a.rt ? tile + tc + dir : tile + dir;
      so[k] = side_gran(sbase, a.ntiles, 0, tl2, nside, rr < 0 ? a.rt - 1 : rr >= a.rt ? 0 : rr);
    }
  }
  const int sslot = a.ntiles * 2 * kResidentMaxRt * 8;  // bytes per side slot
  // (rows: tile tl's row `side`; sides: this wave's side cells of rows ty-1 ..
  // ty+1 into sb / sj when sd -- one poll for both)
  auto take = [&](int slot, bool rows_in, int tl, int side, bool sd, unsigned bit, float (&vb)[6],
                  float (&vj)[6], float (&sb)[3], float (&sj)[3]) {
    const bool el = lane == 0 && wj > 0, er = lane == 63 && wj + 1 < wpr;
    const int o = xch_gran(a.ntiles, wpr, slot, tl, side, wj, 0, lane);
    // lane 0: b3 / j3 of wave wj-1's lane 63 (word 3 of its granules 0, 1);
    // lane 63: b0 / j0 of wave wj+1's lane 0 (word 0); 0 off the grid
    const int eo = el ? xch_gran(a.ntiles, wpr, slot, tl, side, wj - 1, 0, 63) + 12
                      : xch_gran(a.ntiles, wpr, slot, tl, side, wj + 1, 0, 0);
    u4v g[2];
    unsigned e[2];
    u2v s[3];
    take_rows_sides(rx, rows_in, o, el || er, eo, sd && sd_lane, so, slot * sslot, bit, g, e, s,
                    err, a.err_host);
    if (rows_in) {
      const float mb[4] = {untag(g[0][0]), untag(g[0][1]), untag(g[0][2]), untag(g[0][3])};
      const float mj[4] = {untag(g[1][0]), untag(g[1][1]), untag(g[1][2]), untag(g[1][3])};
      row_quad(mb, (el || er) ? untag(e[0]) : 0.0f, vb);
      row_quad(mj, (el || er) ? untag(e[1]) : 0.0f, vj);
    }
    if (sd) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        sb[k] = untag(s[k][0]);
        sj[k] = untag(s[k][1]);
      }
    }
  };

  // ---- prologue: dictionary, zero pads, codes, the tile's b / J into LDS
  // buffer 0, boundary rows into exchange slot 1 (as if step -1's output),
  // then the neighbours' rows for step 0.
  // Step 0's input mass, when a block starts with the previous launch's
  // partials pending: wave 0 issues all its loads of them first (<= 16 quads
  // per lane at <= 4096 partials, the resident grids' most), so that they
  // land while the tables stage; reduced below in wave_reduce_partials' order
  const bool start0 = a.kstep0 % a.depth == 0;
  const bool red0 = start0 && a.in_partials && wave == 0;
  const bool red0_regs = red0 && a.in_n <= kPrologueParts;
  f4a pq[kPrologueParts / 256];
  if (red0_regs) {
    const f4a* q = reinterpret_cast<const f4a*>(a.in_partials);
    const int nq = a.in_n >> 2;
#pragma unroll
    for (int j = 0; j < kPrologueParts / 256; ++j) {
      const int i = lane + 64 * j;
      pq[j] = q[i < nq ? i : 0];
    }
  }
  // the tile's b and J: loads issued first, so that their HBM latency
  // overlaps the table staging and the class planes (consumed below)
  f4a b_t = {0.0f, 0.0f, 0.0f, 0.0f}, j_t = {0.0f, 0.0f, 0.0f, 0.0f};
  if (valid) {
    if (TR) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        b_t[k] = a.b_in[hoff(y, x0 + k)];
        j_t[k] = a.j_in[hoff(y, x0 + k)];
      }
    } else {
      const long long off = (long long)y * wp + gx + x0;
      b_t = *reinterpret_cast<const f4a*>(a.b_in + off);
      j_t = *reinterpret_cast<const f4a*>(a.j_in + off);
    }
  }
  stage_rows(a.rfact, kResTab, lds);
  stage_rows(a.rows, rows_floats(a.E, true), sTC);
  for (int i = threadIdx.x; i < 4 * (a.rt + 1); i += blockDim.x) {
    const int buf = i / (a.rt + 1), r = i % (a.rt + 1);
    *reinterpret_cast<f4a*>(sB0 + buf * bufn + r * xs) = f4a{0.0f, 0.0f, 0.0f, 0.0f};
  }
  // the lane's cells: codes, their IW records (registers for the whole run)
  // and L class bytes
  uint32_t cc[4] = {0u, 0u, 0u, 0u}, iwr[4][3], lx4 = 0u;
  if (valid) {
    if (TR) {
#pragma unroll
      for (int k = 0; k < 4; ++k) cc[k] = a.code[hoff(y, x0 + k)];
    } else {
      const uint2 m = *reinterpret_cast<const uint2*>(a.code + (long long)y * wp + gx + x0);
      cc[0] = m.x & 0xffffu; cc[1] = m.x >> 16; cc[2] = m.y & 0xffffu; cc[3] = m.y >> 16;
    }
    const uint8_t* lx = reinterpret_cast<const uint8_t*>(a.rfact + kResLX);
#pragma unroll
    for (int k = 0; k < 4; ++k) lx4 |= (uint32_t)lx[cc[k]] << (8 * k);
  }
  __syncthreads();  // the staged tables
  PP2_RP(1);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint4 w = *reinterpret_cast<const uint4*>(sTC + kFactIW + 4 * cc[k]);
    iwr[k][0] = w.x; iwr[k][1] = w.y; iwr[k][2] = w.z;
  }
  // class planes of rows trow*rt-1 .. trow*rt+rt: byte x+4 of plane a, row r
  // = 16 * class of cell (y, gx + x) for action a (0 off the grid; the pads
  // hold the side neighbours' cells x = -1 / tw, 0 at the grid's x edges)
  for (int i = threadIdx.x; i < prows * tpr; i += blockDim.x) {
    const int r = i / tpr, xq = (i % tpr) * 4, yy = trow * a.rt + r - 1;
    uint32_t pl[9] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    if (yy >= 0 && yy < rows) {
      uint32_t c4[4];
      if (TR) {
#pragma unroll
        for (int k = 0; k < 4; ++k) c4[k] = a.code[hoff(yy, xq + k)];
      } else {
        const uint2 m = *reinterpret_cast<const uint2*>(a.code + (long long)yy * wp + gx + xq);
        c4[0] = m.x & 0xffffu; c4[1] = m.x >> 16; c4[2] = m.y & 0xffffu; c4[3] = m.y >> 16;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4 w = *reinterpret_cast<const uint4*>(sTC + kFactIW + 4 * c4[k]);
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          const uint32_t wq = q < 4 ? w.x : q < 8 ? w.y : w.z;
          pl[q] |= __builtin_amdgcn_ubfe(wq, 8 * (q % 4), 8) << (8 * k);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 9; ++q)
      *reinterpret_cast<uint32_t*>(sP + (q * prows + r) * ps + 4 + xq) = pl[q];
  }
  for (int i = threadIdx.x; i < 9 * prows; i += blockDim.x) {
    const int q = i / prows, yy = trow * a.rt + i % prows - 1;
    uint32_t lp = 0u, rp = 0u;
    if (yy >= 0 && yy < rows) {
      auto cls = [&](int x) {
        const uint4 w = *reinterpret_cast<const uint4*>(
            sTC + kFactIW + 4 * a.code[hoff(yy, x)]);
        return __builtin_amdgcn_ubfe(q < 4 ? w.x : q < 8 ? w.y : w.z, 8 * (q % 4), 8);
      };
      if (gx > 0) lp = cls(gx - 1) << 24;  // byte 3: x = -1
      if (gx + tw < wp) rp = cls(gx + tw);  // byte 0: x = tw
    }
    *reinterpret_cast<uint32_t*>(sP + i * ps) = lp;
    *reinterpret_cast<uint32_t*>(sP + i * ps + 4 + tw) = rp;
  }
  PP2_RP(4);
  ClassRegs creg;
  if constexpr (TC == 3 && PP2_RES_HOIST) {
    __syncthreads();  // the class planes
    if (valid) load_class_regs(sP, prows, ps, ty, x0, creg);
  }
  if (prior_err != 0u) return;  // (uniform: before any global store)
  const bool bnd = nb_up || nb_dn || sd_l || sd_r;  // waves that cross CUs
  if (valid) {
    const f4a b = b_t, j = j_t;
    *reinterpret_cast<f4a*>(sbuf(0, 0) + ty * xs + x0) = b;
    *reinterpret_cast<f4a*>(sbuf(1, 0) + ty * xs + x0) = j;
    if (bnd) {
      const float bv[4] = {b[0], b[1], b[2], b[3]}, jv[4] = {j[0], j[1], j[2], j[3]};
      publish(1, bv, jv, (a.slot_use[1] + 1u) & 1u);
    }
  }
  // uses of exchange slots 0 / 1 so far (every tile counts every use, whether
  // or not its rows cross a tile edge)
  unsigned use[2] = {a.slot_use[0], a.slot_use[1] + 1u};
  PP2_RP(5);
  // step 0's input mass (k_sum_finalize's tree: lane-strided quads in
  // ascending order, then the butterfly)
  if (red0) {
    float S;
    if (red0_regs) {
      const int nq = a.in_n >> 2;
      float sl = 0.0f;
#pragma unroll
      for (int j = 0; j < kPrologueParts / 256; ++j)
        if (lane + 64 * j < nq) sl += ((pq[j][0] + pq[j][1]) + pq[j][2]) + pq[j][3];
      S = wave_sum(sl);
    } else {
      S = wave_reduce_partials(a.in_partials, a.in_n);
    }
    if (threadIdx.x == 0) {
      sS[0] = S;
      if (tile == 0 && a.in_sum_out) *a.in_sum_out = S;
    }
  }
  __syncthreads();
  float inv = 1.0f;
  if (start0)
    inv = (1.0f / (a.in_partials ? sS[0] : a.in_sum ? *a.in_sum : 1.0f)) * a.bscale;

  // the dense kernels' partial of this wave's 256 cells (row y, x gx + 256 wj)
  const int pi = y * (wp >> 8) + cx * wpr + wj;
  // the wave that takes a block start's arrivals and reduces the partials: an
  // interior one (row 1, not a side wave; SIMD 1) when the tile has interior
  // rows, so that the reduction overlaps the edge waves' hand-off and compute
  // instead of following them on wave 0 (an edge wave)
  const int redw = a.rt >= 3 && wpr >= 4 ? wpr + 1 : 0;
  unsigned arrivals = a.arrive_base;
  int shift = 0;  // shard runs: the power-of-two shifts of the block starts so far
  // Lagged shard block starts (shard mode 2; shards run kstep0 = 0, so block
  // starts fall on multiples of depth).  The shift of the block start at T
  // comes from step tl = T-1-depth's view mass, whose arrivals were due a
  // block earlier: the reduction wave polls the arrival counter for it at
  // the top of step T-2, pulls step tl's partials into sRed by LDS-DMA (sc1,
  // no VGPRs) at the top of step T-1 -- the wave has no global loads of its
  // own in flight, and step T-1's drain (T is an arrival step's successor)
  // completes the copy -- and sums them at the end of step T-1 into sS[0];
  // every wave takes the shift at the top of step T, before its gather.  No
  // barrier and no grid-wide wait of its own.  A tile whose poll came back
  // short (or without red_lds) waits and reduces at the end of step T-1
  // instead, in the same association: every tile gets the same bits.
  constexpr bool lag = LAG;
  int sh_prev = 0;  // the previous lagged block start's shift
  unsigned arr_v = 0u;
  bool red_ok = false;
  auto lag_start = [&](int T) {  // a lagged block start with a reduction
    return lag && T > 0 && T < a.n && T % a.depth == 0 && T - 1 - a.depth >= 0;
  };
  auto lag_target = [&](int T) { return a.arrive_base + (unsigned)(T / a.depth - 1) * a.ntiles; };
  float p[4] = {0.0f, 0.0f, 0.0f, 0.0f}, best[4] = {0.0f, 0.0f, 0.0f, 0.0f}, local = 0.0f;
  uint32_t arg[4] = {0u, 0u, 0u, 0u};
  PP2_RP(2);

  for (int t = 0; t < a.n; ++t) {
    const int u = tr.uz[t] & 15, z = tr.uz[t] >> 4;
    const int ci = t & 1, co = ci ^ 1;
    const bool last = t == a.n - 1;
    // ---- a block start inside the run needs the exact mass of step t-1's
    // belief (a shard: the mass of its whole view -- every cell is <= it, so
    // the power-of-two scale cannot overflow a halo row that holds more mass
    // than the owned ones).  The step's gather and backup go first: the mass
    // only scales the gathered quad, so the grid-wide arrival wait overlaps
    // this tile's compute instead of preceding it.
    const bool bs = t > 0 && (a.kstep0 + t) % a.depth == 0;
    if (t > 0 && !bs) inv = 1.0f;
    if (lag) {
      if (wave == redw) {
        if (lag_start(t + 1)) {  // step t+1-1-depth's partials into sRed
          red_ok = a.red_lds && reached(arr_v, lag_target(t + 1));
          if (red_ok) {
            const float* src = a.ring + (size_t)((t - a.depth) % kResidentRing) * a.nparts;
            const int nq = a.nparts >> 2;
            for (int c = 0; c * 64 < nq; ++c) {
              const int i = c * 64 + lane < nq ? c * 64 + lane : nq - 1;
              __builtin_amdgcn_global_load_lds((glb_void*)(src + 4 * i), (lds_void*)(sRed + c * 256), 16,
                                               0, kSc1);
            }
          }
        }
        if (lag_start(t + 2)) arr_v = ld_flag(a.sync + kResidentSyncArrive);
      }
      if (bs) {  // the shift from sS[0] (the end of step t-1), before the gather
        const int sh = t - 1 - a.depth >= 0 ? pow2_shift_lagged(sS[0], sh_prev) : 0;
        sh_prev = sh;
        shift += sh;
        inv = pow2f(sh);
      }
    }
    PP2_RT(0);
    local = 0.0f;
    // one quad of step t: window rows from LDS (step t-1), the neighbour rows
    // of step t-1, or 0 off the grid; b' before the scale in p
    auto step_quad = [&]() {
      Win6 wb, wj;
      float sb[3] = {0.0f, 0.0f, 0.0f}, sj[3] = {0.0f, 0.0f, 0.0f};
      const bool sd = sd_l || sd_r;
      const unsigned bit = use[co] & 1u;
      if (ty > 0) {
        row_lds(sbuf(0, ci) + (ty - 1) * xs, x0, wb.v[0]);
        row_lds(sbuf(1, ci) + (ty - 1) * xs, x0, wj.v[0]);
      } else if (nb_up) {  // the tile above's last row (and the side cells)
        take(co, true, tile - tc, 1, sd, bit, wb.v[0], wj.v[0], sb, sj);
      } else {
        row_zero(wb.v[0]);
        row_zero(wj.v[0]);
      }
      row_lds(sbuf(0, ci) + ty * xs, x0, wb.v[1]);
      row_lds(sbuf(1, ci) + ty * xs, x0, wj.v[1]);
      if (ty + 1 < a.rt && y + 1 < rows) {
        row_lds(sbuf(0, ci) + (ty + 1) * xs, x0, wb.v[2]);
        row_lds(sbuf(1, ci) + (ty + 1) * xs, x0, wj.v[2]);
      } else if (nb_dn) {  // the tile below's first row (and the side cells)
        take(co, true, tile + tc, 0, sd && !nb_up, bit, wb.v[2], wj.v[2], sb, sj);
      } else {
        row_zero(wb.v[2]);
        row_zero(wj.v[2]);
      }
      if (sd && !nb_up && !nb_dn) take(co, false, tile, 0, true, bit, wb.v[1], wj.v[1], sb, sj);
      if (sd_lane) {  // the side neighbour's cells x = -1 (lane 0) / tw (lane 63)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (sd_l) {
            wb.v[k][0] = sb[k];
            wj.v[k][0] = sj[k];
          } else {
            wb.v[k][5] = sb[k];
            wj.v[k][5] = sj[k];
          }
        }
      }
      PP2_RT(1);
      if constexpr (TC == 3 && PP2_RES_HOIST) {
        // opaque per step (empty asm): otherwise the compiler hoists the 9
        // actions' table addresses, loop-invariant now, out of the step loop
#pragma unroll
        for (int i = 0; i < kClsSlots; ++i) asm volatile("" : "+v"(creg.m[i]));
#pragma unroll
        for (int i = 0; i < (kClsSlots + 1) / 2; ++i) asm volatile("" : "+v"(creg.lh[i]));
        belief_any_regs(u, creg, lx4, z, wb, p);
      }
      else belief_any<TR>(u, sP, prows, ps, ty, x0, lx4, z, wb, p);
      float jn[9][4];  // grid stencil offset i = 3 (dy + 1) + dx + 1
#pragma unroll
      for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) jn[i][k] = TR ? wj.v[i % 3][k + i / 3] : wj.v[i / 3][k + i % 3];
      // (2-D tiles: the cells' table reads in pairs, coded_sweep_iw)
      if (last) coded_sweep_iw<4, true, kSweepG>(sTC, iwr, jn, best, arg);  // actions: last step only
      else coded_sweep_iw<4, false, kSweepG>(sTC, iwr, jn, best, arg);
      *reinterpret_cast<f4a*>(sbuf(1, co) + ty * xs + x0) = f4a{best[0], best[1], best[2], best[3]};
    };
    // the scale, the mass partial, b' into LDS and the boundary rows out --
    // the neighbours' next inputs
    auto finish_quad = [&]() {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        p[k] = p[k] * inv;
        local += p[k];
      }
      *reinterpret_cast<f4a*>(sbuf(0, co) + ty * xs + x0) = f4a{p[0], p[1], p[2], p[3]};
      if (bnd) {
        if (!last) publish(ci, p, best, (use[ci] + 1u) & 1u);
        __builtin_amdgcn_s_setprio(0);
      }
    };
    if (valid) {
      // the boundary waves take the neighbours' step t-1 rows (published at
      // the end of their step t-1) and compute with issue priority
      if (bnd) __builtin_amdgcn_s_setprio(2);  // 6.0 vs 7.4 us/step at 1024^2 without
      step_quad();
      if (!bs || lag) finish_quad();
    }
    if (bs && !lag) {
      if (wave == redw) {
        arrivals += a.ntiles;
        wave_wait(a.sync + kResidentSyncArrive, 1, arrivals, err, a.err_host);
        const float S = wave_reduce_partials_sc1(
            a.ring + (size_t)((t - 1) % kResidentRing) * a.nparts, a.nparts);
        if (lane == 0) sS[0] = S;
      }
      __syncthreads();
      if (a.shard) {
        const int sh = pow2_shift(sS[0]);
        shift += sh;
        inv = pow2f(sh);
      } else {
        inv = (1.0f / sS[0]) * a.bscale;
      }
      if (valid) finish_quad();
    }
    PP2_RT(2);
    if (last) break;  // the last step's outputs are stored after the loop
    ++use[ci];
    // ---- mass partials of step t (dense map), sc1 into the ring
    {
      const float v = wave_sum(local);
      if (lane == 0 && pi < a.nparts)
        st_flag(reinterpret_cast<unsigned*>(a.ring + (size_t)(t % kResidentRing) * a.nparts + pi),
                __float_as_uint(v));
    }
    // ---- arrive for the next step's block start (every wave drained first)
    const bool arrive = (a.kstep0 + t + 1) % a.depth == 0;
    if (arrive) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wave == redw && lag_start(t + 1)) {  // the lagged mass for the next step's block start
      float S;
      if (red_ok) {  // (the drain above completed the copy)
        const int nq = a.nparts >> 2;
        float sl = 0.0f;
        for (int i = lane; i < nq; i += 64) {
          const f4a w = *reinterpret_cast<const f4a*>(sRed + 4 * i);
          sl += ((w[0] + w[1]) + w[2]) + w[3];
        }
        S = wave_sum(sl);
      } else {
        wave_wait(a.sync + kResidentSyncArrive, 1, lag_target(t + 1), err, a.err_host);
        S = wave_reduce_partials_sc1(a.ring + (size_t)((t - a.depth) % kResidentRing) * a.nparts,
                                     a.nparts);
      }
      if (lane == 0) sS[0] = S;
    }
#ifndef PP2_RES_NOBAR
    __syncthreads();  // also: this step's LDS writes before the next step's reads
#endif
    if (arrive && threadIdx.x == 0)
      __hip_atomic_fetch_add(a.sync + kResidentSyncArrive, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    PP2_RT(3);
  }

  // ---- the last step: b, J, A of the (owned) rows and the owned mass
  // partials (a shard's halo rows are its neighbours' rows)
  if (own && TR) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long off = hoff(y, x0 + k);
      __builtin_nontemporal_store(p[k], a.b_out + off);
      __builtin_nontemporal_store(best[k], a.j_out + off);
      a.A[off] = (uint8_t)arg[k];
    }
  } else if (own) {
    const long long off = (long long)y * wp + gx + x0;
    store4<true>(a.b_out + off, p);
    store_ja<true>(a.j_out, a.A, off, best, arg);
  }
  const float v = wave_sum(own ? local : 0.0f);
  if (lane == 0 && pi < a.nparts) a.out_partials[pi] = v;
  if (a.scale_out && tile == 0 && threadIdx.x == 0) *a.scale_out = shift;
  PP2_RP(3);
}

// ---------------------------------------------------------------- MDP solve
// pp2_mdp_solve's value iteration (valueIteration, src/mdp/path_planning_2d.cu:
// 207-269) as resident sweeps: the tiles of k_loop_resident carry J only (two
// LDS buffers and the convergence snapshot), the edge rows of J cross CUs by
// the same granules (J alone: granules 0, 1), and after every block of 100 sweeps
// each tile publishes max |J - snapshot| over its cells; once the arrival
// counter is full every tile reads all of them (the max is exact in any
// order) and takes the same decision: stop when the norm is <= thresh or the
// block cap is reached, else go on.  Actions are computed (and stored) on
// each block's last sweep only; the last block's J, A and snapshot are
// stored, and tile 0 writes {sweeps, norm bits} to res.  nsweeps > 0 runs
// exactly that many sweeps instead, with no checks (pp2_mdp_sweep).
__global__ __launch_bounds__(1024, 4) void k_sweep_resident(const SweepRun a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wp = a.g.wp, rows = a.g.rows, tpr = wp >> 2, wpr = wp >> 8;
  const int xs = wp + 4;
  const int bufn = 4 + a.rt * xs;
  float* sTC = lds;
  float* sJ0 = sTC + lds_span(rows_floats(a.E, true));  // J buffers 0, 1, snapshot
  float* sM = sJ0 + 3 * bufn;                              // per-wave maxima, decision

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  if (tile == a.stall_tile) return;  // diagnostic: a tile that never arrives
  // a chained launch after one that timed out does nothing (resident_settle)
  const unsigned prior_err = ld_flag(a.sync + kResidentSyncErr);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ty = __builtin_amdgcn_readfirstlane(threadIdx.x / tpr);
  const int wj = __builtin_amdgcn_readfirstlane((threadIdx.x % tpr) >> 6);
  const int x0 = (threadIdx.x % tpr) * 4;
  const int y = tile * a.rt + ty;
  const bool valid = y < rows;
  const bool nb_up = valid && ty == 0 && tile > 0;
  const bool nb_dn = valid && ty == a.rt - 1 && y + 1 < rows;
  unsigned* const err = a.sync + kResidentSyncErr;
  const Rsrc rx = make_rsrc(a.xch);
  auto sbuf = [&](int i) { return sJ0 + i * bufn + 4; };
  // k_loop_resident's hand-off with J alone: granule 0, {j0..j3}
  const int myx = tile_xcd(tile, (int)gridDim.x);
  const bool plain_up = PP2_RES_XCD_PLAIN && nb_up && tile_xcd(tile - 1, (int)gridDim.x) == myx;
  const bool plain_dn = PP2_RES_XCD_PLAIN && nb_dn && tile_xcd(tile + 1, (int)gridDim.x) == myx;
  auto publish = [&](int slot, const float (&j)[4], unsigned bit) {
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      if (side == 0 ? !nb_up : !nb_dn) continue;
      st_quad_x(rx, xch_gran(a.ntiles, wpr, slot, tile, side, wj, 0, lane), j, bit,
                side == 0 ? plain_up : plain_dn);
    }
  };
  auto take = [&](int slot, int tl, int side, unsigned bit, float (&v)[6]) {
    const bool el = lane == 0 && wj > 0, er = lane == 63 && wj + 1 < wpr;
    const int o = xch_gran(a.ntiles, wpr, slot, tl, side, wj, 0, lane);
    // lane 0: j3 of wave wj-1's lane 63 (word 3); lane 63: j0 of wave wj+1's
    // lane 0 (word 0)
    const int eo = el ? xch_gran(a.ntiles, wpr, slot, tl, side, wj - 1, 0, 63) + 12
                      : xch_gran(a.ntiles, wpr, slot, tl, side, wj + 1, 0, 0);
    u4v g[1];
    unsigned e[1];
    take_granules(rx, o, el || er, eo, bit, g, e, err, a.err_host);
    const float m[4] = {untag(g[0][0]), untag(g[0][1]), untag(g[0][2]), untag(g[0][3])};
    row_quad(m, (el || er) ? untag(e[0]) : 0.0f, v);
  };

  stage_rows(a.rows, rows_floats(a.E, true), sTC);
  for (int i = threadIdx.x; i < 3 * (a.rt + 1); i += blockDim.x) {
    const int buf = i / (a.rt + 1), r = i % (a.rt + 1);
    *reinterpret_cast<f4a*>(sJ0 + buf * bufn + r * xs) = f4a{0.0f, 0.0f, 0.0f, 0.0f};
  }
  uint32_t c0 = 0, c1 = 0;  // the quad's codes
  const long long goff = (long long)y * wp + x0;
  if (prior_err != 0u) return;  // (uniform: before any global store)
  if (valid) {
    const uint2 m = *reinterpret_cast<const uint2*>(a.code + goff);
    c0 = m.x;
    c1 = m.y;
    const f4a j = *reinterpret_cast<const f4a*>(a.j_in + goff);
    *reinterpret_cast<f4a*>(sbuf(0) + ty * xs + x0) = j;
    *reinterpret_cast<f4a*>(sbuf(2) + ty * xs + x0) = *reinterpret_cast<const f4a*>(a.snap + goff);
    if (nb_up || nb_dn) {
      const float jv[4] = {j[0], j[1], j[2], j[3]};
      publish(1, jv, (a.slot_use[1] + 1u) & 1u);
    }
  }
  unsigned use[2] = {a.slot_use[0], a.slot_use[1] + 1u};  // slot uses so far
  __syncthreads();
  // the quad's IW records in registers for the whole run (k_loop_resident)
  uint32_t iwr[4][3];
  {
    const uint32_t cc[4] = {c0 & 0xffffu, c0 >> 16, c1 & 0xffffu, c1 >> 16};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 w = *reinterpret_cast<const uint4*>(sTC + kFactIW + 4 * cc[k]);
      iwr[k][0] = w.x; iwr[k][1] = w.y; iwr[k][2] = w.z;
    }
  }

  unsigned arrivals = a.arrive_base;
  float best[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t arg[4] = {0u, 0u, 0u, 0u};
  int s = 0, blk = 0;
  float norm = 0.0f;
  for (;; ++s) {
    const int ci = s & 1, co = ci ^ 1;
    // a block's last sweep (convergence check), or the last of a fixed count
    const bool fin = a.nsweeps > 0 && s == a.nsweeps - 1;
    const bool check = a.nsweeps == 0 && s % kSolveBlock == kSolveBlock - 1;
    if (valid) {
      if (nb_up || nb_dn) __builtin_amdgcn_s_setprio(2);
      Win6 w;
      if (ty > 0) row_lds(sbuf(ci) + (ty - 1) * xs, x0, w.v[0]);
      else if (nb_up) take(co, tile - 1, 1, use[co] & 1u, w.v[0]);
      else row_zero(w.v[0]);
      row_lds(sbuf(ci) + ty * xs, x0, w.v[1]);
      if (ty + 1 < a.rt && y + 1 < rows) row_lds(sbuf(ci) + (ty + 1) * xs, x0, w.v[2]);
      else if (nb_dn) take(co, tile + 1, 0, use[co] & 1u, w.v[2]);
      else row_zero(w.v[2]);
      float jn[9][4];
#pragma unroll
      for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) jn[i][k] = w.v[i / 3][k + i % 3];
      if (check || fin) coded_sweep_iw<4, true>(sTC, iwr, jn, best, arg);
      else coded_sweep_iw<4, false>(sTC, iwr, jn, best, arg);
      *reinterpret_cast<f4a*>(sbuf(co) + ty * xs + x0) = f4a{best[0], best[1], best[2], best[3]};
      if (nb_up || nb_dn) {
        publish(ci, best, (use[ci] + 1u) & 1u);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    ++use[ci];
    if (fin) break;
    if (!check) {
      __syncthreads();
      continue;
    }
    // ---- end of a block: max |J - snapshot| over the tile, snapshot := J
    float m = 0.0f;
    if (valid) {
      float* sn = sbuf(2) + ty * xs + x0;
      const f4a old = *reinterpret_cast<const f4a*>(sn);
#pragma unroll
      for (int k = 0; k < 4; ++k) m = fmaxf(m, fabsf(old[k] - best[k]));
      *reinterpret_cast<f4a*>(sn) = f4a{best[0], best[1], best[2], best[3]};
    }
    m = wave_max(m);
    if (lane == 0) sM[wave] = m;
    __syncthreads();
    if (wave == 0) {
      float tm = lane < (int)(blockDim.x >> 6) ? sM[lane] : 0.0f;
      tm = wave_max(tm);
      if (lane == 0)
        st_flag(reinterpret_cast<unsigned*>(a.tile_max + (blk & 1) * a.ntiles + tile),
                __float_as_uint(tm));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        __hip_atomic_fetch_add(a.sync + kResidentSyncArrive, 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      arrivals += a.ntiles;
      wave_wait(a.sync + kResidentSyncArrive, 1, arrivals, err, a.err_host);
      const Rsrc rm = make_rsrc(a.tile_max + (blk & 1) * a.ntiles);
      float g = 0.0f;
      for (int i = lane; i < a.ntiles; i += 64) g = fmaxf(g, ld1_sc1(rm, 4 * i));
      g = wave_max(g);
      if (lane == 0) sM[16] = g;
    }
    __syncthreads();
    norm = sM[16];
    ++blk;
    if (!((double)norm > a.thresh) || (a.cap_blocks > 0 && blk >= a.cap_blocks) ||
        blk >= a.max_blocks)
      break;
  }
  // ---- J (into j_out: the input survives the run), A and the snapshot of
  // the last block; the result
  const int done = s + 1;
  if (valid) {
    store4<false>(a.j_out + goff, best);
    const uint32_t a4 = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    *reinterpret_cast<uint32_t*>(a.A + goff) = a4;
    if (a.nsweeps == 0)  // the solve's snapshot (pp2_mdp_sweep leaves it alone)
      *reinterpret_cast<f4a*>(a.snap + goff) = f4a{best[0], best[1], best[2], best[3]};
  }
  if (tile == 0 && threadIdx.x == 0) {
    a.res[0] = done;
    a.res[1] = (int)__float_as_uint(norm);
  }
}

}  // namespace

size_t resident_lds_bytes(const Geom& g, int E, int rt, int tc) {
  const int tw = g.wp / tc;
  return ((size_t)lds_span(kResTab) + lds_span(rows_floats(E, true)) +
          lds_span(9 * (rt + 2) * (tw + 8) / 4) + 4 * (4 + (size_t)rt * (tw + 4)) + 16) *
         sizeof(float);
}

// The plan with tc tile columns: rt rows per tile so that the tiles fit the
// CUs, or false.
// The kernel instance of a tiling: 2-D tiles of <= 768 threads run the
// register-rich TC = 3 instance (PP2_RES_RICH=0 at build time: never).
static int resident_tc(int tc, int threads) {
#ifndef PP2_RES_RICH
#define PP2_RES_RICH 1
#endif
  return tc == 2 && threads <= 768 && PP2_RES_RICH ? 3 : tc;
}

static bool resident_plan_tc(const Geom& g, int E, int ncus, int tc, ResidentPlan* p,
                             bool trn = false) {
  if (tc < 1 || tc > 2 || g.wp % (256 * tc) != 0 || (tc > 1 && g.wp / tc < 512) || ncus < tc) return false;
  const int rt = (g.rows + ncus / tc - 1) / (ncus / tc);
  const long long threads = (long long)rt * (g.wp / tc / 4);
  if (threads > 1024 || rt > kResidentMaxRt) return false;
  const size_t lds = resident_lds_bytes(g, E, rt, tc);
  if (lds > kDictLdsMaxBytes) return false;
  if (trn && tc != 1) return false;
  static unsigned long long attr[16] = {};
  // the instance: TC = 3 for 2-D tiles of <= 768 threads (resident_tc)
  const int ktc = resident_tc(tc, (int)threads);
#define PP2_K(CAPV, TCV, LAGV, TRV) reinterpret_cast<const void*>(&k_loop_resident<CAPV, TCV, LAGV, TRV>)
#define PP2_KT(CAPV, LAGV)                                                                    \
  (trn ? PP2_K(CAPV, 1, LAGV, true)                                                           \
       : ktc == 1 ? PP2_K(CAPV, 1, LAGV, false)                                               \
                  : ktc == 2 ? PP2_K(CAPV, 2, LAGV, false) : PP2_K(CAPV, 3, LAGV, false))
  const void* ks[4] = {PP2_KT(kResidentShortSteps, false), PP2_KT(kResidentMaxSteps, false),
                       PP2_KT(kResidentShortSteps, true), PP2_KT(kResidentMaxSteps, true)};
#undef PP2_KT
#undef PP2_K
  const int ai = trn ? 8 : 4 * (ktc - 1) + (ktc == 3 ? 4 : 0);
  int nb = 1 << 30;
  for (int k = 0; k < 4; ++k) {
    allow_lds(ks[k], attr[ai + k]);
    int n1 = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n1, ks[k], (int)threads, lds) != hipSuccess ||
        n1 < 1) {
      (void)hipGetLastError();
      return false;
    }
    nb = std::min(nb, n1);
  }
  p->rt = rt;
  p->tc = tc;
  p->tr = trn;
  p->ntiles = (g.rows + rt - 1) / rt * tc;
  p->threads = (int)threads;
  p->lds = lds;
  // co-residency, checked before any launch: every tile must hold a CU slot
  // at once (the waits assume it).  1024-lane workgroups at these LDS sizes
  // get one slot per CU, so this is ntiles <= ncus; the guide's SGPR caveat
  // (one block fewer than the API answer) applies to 256-lane blocks at
  // several per CU, not here.
  return (long long)nb * ncus >= p->ntiles;
}

// Whole-row tiles, or two tile columns when whole rows would give tiles of
// fewer than 4 rows -- every row an edge row, so every wave of the CU waits
// on a neighbour -- and 2-D tiles hold 3 or more (tc_pref 0), or whenever they
// fit (tc_pref 2).  A 256-row share of the 2048^2 grid (its 512-row view)
// then runs 4 x 1024 tiles instead of 2 x 2048: 4.89 vs 5.03 us per step
// (tools/ab_tile_cols.py); its 384-row view (e = 64) 3 x 1024
// instead of 2 x 2048: 4.46 vs 4.88 (profiles/r04/ab_sweep_ao.txt).
bool resident_plan(const Geom& g, int E, int ncus, ResidentPlan* p, int tc_pref, bool allow_tr) {
  ResidentPlan p1, p2, pt;
  if (tc_pref == 3 && allow_tr && g.rows % 256 == 0 &&
      resident_plan_tc(transposed_geom(g), E, ncus, 1, &pt, true)) {
    *p = pt;
    return true;
  }
  const bool ok1 = resident_plan_tc(g, E, ncus, 1, &p1);
  const bool ok2 = tc_pref != 1 && resident_plan_tc(g, E, ncus, 2, &p2);
  // (automatic only with 1024-column tiles or wider: the measured shape, whose
  // rows keep interior waves beside the side waves)
  if (ok2 && ok1 && (tc_pref == 2 || (p1.rt < 4 && p2.rt >= 3 && g.wp / 2 >= 1024))) {
    *p = p2;
    return true;
  }
  if (ok1) *p = p1;
  return ok1;
}

hipError_t launch_loop_resident(hipStream_t st, const ResidentPlan& p, const ResidentRun& a) {
  if (a.n < 1 || a.n > kResidentMaxSteps || a.ntiles != p.ntiles || a.rt != p.rt || a.tc != p.tc ||
      a.depth < 1 || a.depth > kResidentRing - 2 || a.own0 < 0 || a.own1 > (p.tr ? a.g.wp : a.g.rows) ||
      a.own0 >= a.own1 || a.b_out == a.b_in || a.j_out == a.j_in ||
      (a.in_partials && a.in_partials == a.out_partials))
    return hipErrorInvalidValue;
  const ResidentHead& h = a;
  const size_t lds = p.lds + (a.red_lds ? (size_t)kResRedFloats * sizeof(float) : 0);
  if (a.red_lds && (a.shard != 2 || a.kstep0 != 0 || a.nparts > kResRedFloats || lds > kDictLdsMaxBytes))
    return hipErrorInvalidValue;
  const bool lag = a.shard == 2;
  // lagged block starts read ring slot t - depth while the fastest tiles can
  // be 2 depth + 1 steps ahead: slot reuse is race-free only below the ring
  if (lag && 3 * a.depth + 1 >= kResidentRing) return hipErrorInvalidValue;
  if (p.tr && (p.tc != 1 || !a.shard || a.own0 % 4 != 0 || a.own1 % 4 != 0 || a.ows < a.g.rows))
    return hipErrorInvalidValue;
#define PP2_RES_LAUNCH(CAPV, TCV, TRV)                                                           \
  do {                                                                                           \
    if (lag)                                                                                     \
      hipLaunchKernelGGL((k_loop_resident<CAPV, TCV, true, TRV>), dim3(p.ntiles),                \
                         dim3(p.threads), lds, st, h, tr);                                       \
    else                                                                                         \
      hipLaunchKernelGGL((k_loop_resident<CAPV, TCV, false, TRV>), dim3(p.ntiles),               \
                         dim3(p.threads), lds, st, h, tr);                                       \
  } while (0)
  const int ktc = resident_tc(p.tc, p.threads);
  if (a.n <= kResidentShortSteps) {
    Trajectory<kResidentShortSteps> tr{};
    std::memcpy(tr.uz, a.uz, (size_t)a.n);
    if (p.tr) PP2_RES_LAUNCH(kResidentShortSteps, 1, true);
    else if (ktc == 1) PP2_RES_LAUNCH(kResidentShortSteps, 1, false);
    else if (ktc == 2) PP2_RES_LAUNCH(kResidentShortSteps, 2, false);
    else PP2_RES_LAUNCH(kResidentShortSteps, 3, false);
  } else {
    Trajectory<kResidentMaxSteps> tr;
    std::memcpy(tr.uz, a.uz, sizeof tr.uz);
    if (p.tr) PP2_RES_LAUNCH(kResidentMaxSteps, 1, true);
    else if (ktc == 1) PP2_RES_LAUNCH(kResidentMaxSteps, 1, false);
    else if (ktc == 2) PP2_RES_LAUNCH(kResidentMaxSteps, 2, false);
    else PP2_RES_LAUNCH(kResidentMaxSteps, 3, false);
  }
#undef PP2_RES_LAUNCH
  return hipGetLastError();
}

size_t solve_lds_bytes(const Geom& g, int E, int rt) {
  return ((size_t)lds_span(rows_floats(E, true)) + 3 * (4 + (size_t)rt * (g.wp + 4)) + 32) *
         sizeof(float);
}

bool solve_plan(const Geom& g, int E, int ncus, ResidentPlan* p) {
  if (E <= 0 || g.rows <= 0 || g.wp % 256 != 0 || ncus <= 0) return false;
  const int rt = (g.rows + ncus - 1) / ncus;
  const long long threads = (long long)rt * (g.wp / 4);
  if (threads > 1024) return false;
  const size_t lds = solve_lds_bytes(g, E, rt);
  if (lds > kDictLdsMaxBytes) return false;
  static unsigned long long attr = 0;
  allow_lds(reinterpret_cast<const void*>(&k_sweep_resident), attr);
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sweep_resident, (int)threads, lds) !=
          hipSuccess ||
      nb < 1) {
    (void)hipGetLastError();
    return false;
  }
  p->rt = rt;
  p->ntiles = (g.rows + rt - 1) / rt;
  p->threads = (int)threads;
  p->lds = lds;
  // co-residency, checked before any launch: every tile must hold a CU slot
  // at once (the waits assume it).  1024-lane workgroups at these LDS sizes
  // get one slot per CU, so this is ntiles <= ncus; the guide's SGPR caveat
  // (one block fewer than the API answer) applies to 256-lane blocks at
  // several per CU, not here.
  return (long long)nb * ncus >= p->ntiles;
}

hipError_t launch_sweep_resident(hipStream_t st, const ResidentPlan& p, const SweepRun& a) {
  if ((a.nsweeps == 0 && a.max_blocks < 1) || a.nsweeps < 0 || a.ntiles != p.ntiles ||
      a.rt != p.rt || a.j_out == a.j_in)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_sweep_resident, dim3(p.ntiles), dim3(p.threads), p.lds, st, a);
  return hipGetLastError();
}

namespace {

// ---------------------------------------------------------------- shard boundary
// Row shards whose resident runs scaled their beliefs by different powers of
// two (k_loop_resident, shard mode) meet at the next halo exchange.  Each
// shard posts {owned mass, shift} into its slot of a 2 x nranks vector
// (zeros elsewhere), the vector is summed over the ranks (every slot has one
// non-zero contributor, so the sum is exact in any order), and every shard
// rebases its rows to the common shift C = min over the shards: a row that
// came from shard q is multiplied by 2^(C - shift_q) <= 1 (exact, unless the
// value drops below FLT_MIN relative to the largest shard's mass), and the
// global mass at that common scale is the rank-ordered sum of
// ldexp(m_q, C - shift_q) -- identical on every shard.
__global__ void k_shard_mass_vec(const float* __restrict__ partials, int n,
                                 const int* __restrict__ shift, float* __restrict__ vec,
                                 int nranks, int rank, const unsigned* __restrict__ err_word) {
  const float S = wave_reduce_partials(partials, n);  // k_sum_finalize's tree
  for (int i = threadIdx.x; i < kVecRec * nranks; i += 64)
    if (i / kVecRec != rank) vec[i] = 0.0f;
  if (threadIdx.x == 0) {
    float* r = vec + kVecRec * rank;
    r[0] = S;
    r[1] = shift ? (float)*shift : 0.0f;
    r[2] = err_word && ld_flag(err_word) != 0u ? 1.0f : 0.0f;
  }
}

__global__ void k_shard_rebase(const float* __restrict__ vec, int nranks, int rank,
                               float* __restrict__ b, int wp, int r0, int r1, int own_rows,
                               float* __restrict__ mass_out, unsigned* __restrict__ err_host) {
  int C = 0x7fffffff;
  bool lost = false;
  for (int q = 0; q < nranks; ++q) {
    C = min(C, (int)vec[kVecRec * q + 1]);
    lost = lost || vec[kVecRec * q + 2] != 0.0f;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && err_host && lost)
    __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (blockIdx.x == 0 && threadIdx.x == 0 && mass_out) {
    float M = 0.0f;
    for (int q = 0; q < nranks; ++q)
      M += __builtin_ldexpf(vec[kVecRec * q], C - (int)vec[kVecRec * q + 1]);
    *mass_out = M;
  }
  const int tpr = wp >> 2;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nq = (long long)(r1 - r0) * tpr;
  if (i >= nq) return;
  const int row = r0 + (int)(i / tpr), x = (int)(i % tpr) * 4;
  int q = row < 0 ? rank - 1 : row >= own_rows ? rank + 1 : rank;
  if (q < 0 || q >= nranks) q = rank;  // off the grid: zeros either way
  const int k = C - (int)vec[kVecRec * q + 1];
  if (k == 0) return;
  float* p = b + (long long)row * wp + x;
  f4a v = *reinterpret_cast<const f4a*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = __builtin_ldexpf(v[j], k);
  *reinterpret_cast<f4a*>(p) = v;
}

}  // namespace

hipError_t launch_shard_mass_vec(hipStream_t st, const float* partials, int n, const int* shift,
                                 float* vec, int nranks, int rank, const unsigned* err_word) {
  if (n < 0 || n % 4 != 0 || nranks < 1 || rank < 0 || rank >= nranks) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_shard_mass_vec, dim3(1), dim3(64), 0, st, partials, n, shift, vec, nranks,
                     rank, err_word);
  return hipGetLastError();
}

hipError_t launch_shard_rebase(hipStream_t st, const float* vec, int nranks, int rank, float* b,
                               int wp, int r0, int r1, int own_rows, float* mass_out,
                               unsigned* err_host) {
  if (wp % 4 != 0 || r1 < r0 || nranks < 1) return hipErrorInvalidValue;
  const long long nq = (long long)(r1 - r0) * (wp / 4);
  const int blocks = (int)std::max<long long>(1, (nq + 255) / 256);
  hipLaunchKernelGGL(k_shard_rebase, dim3(blocks), dim3(256), 0, st, vec, nranks, rank, b, wp, r0,
                     r1, own_rows, mass_out, err_host);
  return hipGetLastError();
}

}  // namespace pp2

#ifdef PP2_RES_TRACE
extern "C" int pp2_debug_resident_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pp2::g_rtrace), sizeof(pp2::g_rtrace)) == hipSuccess
             ? 0 : 2;
}
extern "C" int pp2_debug_resident_prologue(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pp2::g_rtrace_pro), sizeof(pp2::g_rtrace_pro)) ==
                 hipSuccess ? 0 : 2;
}
#endif
