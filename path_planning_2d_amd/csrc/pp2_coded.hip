// pp2_coded.hip -- the dictionary-coded model path (gfx950).
//
// The generated model is a function of each cell's 3x3 occupancy (SURVEY.md
// §8 a1: at most 257 distinct transition patterns), so the dense model --
// T 324 B + C 36 B + R 36 B + L 64 B per cell, the bulk of the north-star
// loop's HBM traffic -- is mostly repetition.  The coded path stores
//   * code  : uint16 per cell (rows -1..rows, same padded geometry), and
//   * dict  : one row per distinct per-cell (T, C, L) tuple (kDictRow
//             floats): [u][T_u0..T_u8, C_u] (90) | L[16] | pad.
// R (the POMDP stage reward) is left out: it also varies with the occupancy
// around an occupied cell (another 256 patterns), and only the rollout reads
// it, once per cell per slab for a whole chunk of copies, from its plane.
// built from the dense planes by exact tuple equality (hash on the GPU,
// first-appearance numbering on the host, then a bitwise verification pass
// over every cell; any mismatch leaves the context on the dense path).  A
// kernel stages the dictionary's T/C rows in LDS once per workgroup and reads
// only codes, beliefs and values from HBM.  Per-cell arithmetic is exactly
// the dense kernels' (same operands, same fmaf order), and the belief partial
// sums use the dense kernels' cell->block mapping and reduction tree, so the
// coded and dense paths give bit-identical beliefs, masses, values and actions.
#include "pp2_coded_dev.h"

namespace pp2 {

#ifdef PP2_PHASE_TRACE
// Diagnostic build only (tools/micro/phase_trace.sh): thread 0 of each
// workgroup records s_memrealtime (100 MHz) at the fused step's phase points.
__device__ unsigned long long g_phase[1024][8];
#define PP2_PHASE(i) \
  if (threadIdx.x == 0 && blockIdx.x < 1024) g_phase[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime()
#else
#define PP2_PHASE(i) (void)0
#endif

namespace {

constexpr int kQuarter = kBlock;  // a dense-kernel block: 256 threads, 1024 cells

// ---------------------------------------------------------------- build
__device__ __forceinline__ float tuple_value(const PlaneSet& T, const PlaneSet& C,
                                             const PlaneSet& R, const PlaneSet& L, int y,
                                             int x, int k) {
  if (k < 90) {
    const int u = k / 10, i = k % 10;
    return i < 9 ? T.p[(long long)y * T.rs + (long long)(9 * u + i) * T.ps + x]
                 : C.p[(long long)y * C.rs + (long long)u * C.ps + x];
  }
  if (k < kDictTuple) return L.p[(long long)y * L.rs + (long long)(k - 90) * L.ps + x];
  return 0.0f;
}

__device__ __forceinline__ uint64_t mix64(uint64_t h) {
  h ^= h >> 31;
  h *= 0x7fb5d329728ea185ull;
  h ^= h >> 27;
  h *= 0x81dadef4bc2dd44dull;
  h ^= h >> 33;
  return h;
}

// hash of the kDictTuple-value tuple of every cell in rows [-1, rows]
__global__ __launch_bounds__(kBlock) void k_dict_hash(Geom g, PlaneSet T, PlaneSet C,
                                                      PlaneSet R, PlaneSet L,
                                                      uint64_t* __restrict__ out) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long n = (long long)(g.rows + 2 * g.halo) * g.wp;
  if (i >= n) return;
  const int y = (int)(i / g.wp) - g.halo, x = (int)(i % g.wp);
  uint64_t h = 0x9e3779b97f4a7c15ull;
  for (int k = 0; k < kDictTuple; ++k) {
    const uint32_t w = __float_as_uint(tuple_value(T, C, R, L, y, x, k));
    h = mix64(h ^ (w + 0x632be59bd9b4e019ull * (uint64_t)(k + 1)));
  }
  out[i] = h;
}

__global__ __launch_bounds__(kBlock) void k_dict_gather(Geom g, PlaneSet T, PlaneSet C,
                                                        PlaneSet R, PlaneSet L,
                                                        const int* __restrict__ reps, int E,
                                                        float* __restrict__ dict) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= E * kDictRow) return;
  const int e = i / kDictRow, k = i % kDictRow;
  const int cell = reps[e];
  const int y = cell / g.wp - g.halo, x = cell % g.wp;
  dict[i] = tuple_value(T, C, R, L, y, x, k);
}

__global__ __launch_bounds__(kBlock) void k_dict_verify(Geom g, PlaneSet T, PlaneSet C,
                                                        PlaneSet R, PlaneSet L,
                                                        const uint16_t* __restrict__ code,
                                                        const float* __restrict__ dict,
                                                        int* __restrict__ bad) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long n = (long long)(g.rows + 2 * g.halo) * g.wp;
  if (i >= n) return;
  const int y = (int)(i / g.wp) - g.halo, x = (int)(i % g.wp);
  const float* d = dict + (long long)code[i] * kDictRow;
  int diff = 0;
  for (int k = 0; k < kDictTuple; ++k)
    diff |= __float_as_uint(tuple_value(T, C, R, L, y, x, k)) != __float_as_uint(d[k]);
  if (diff) atomicOr(bad, 1);
}


// Fused north-star step on the coded model (k_loop_step's semantics).  A
// workgroup of QPB x 256 threads covers QPB dense-kernel blocks per tile:
// lane (q, t) of tile tl is the dense kernel's thread t of block QPB*tl + q,
// with the same 4 cells, and writes that block's wave partial 4*d + wave, so
// masses -- and everything else -- are bit-identical to the dense path.  The
// first tile's codes and belief window are in flight while the dictionary
// stages; the value window is loaded after the belief update (its registers
// would not fit beside the belief's); no barrier follows the stores.
//   rows: dictionary rows in the LDS layout (E x Layout::row floats)
//   lz:   L_z column of the dictionary (E floats)
// NT: non-temporal b', J', A stores (they skip the L2 write-back at the end
// of the launch).  A value-row prefetch into LDS (the sweep's J window staged
// with the dictionary) measured slower: every workgroup's barrier then waits
// for an HBM round trip that the register path overlaps with the belief
// update (MI355X, 1024^2: 10.5 vs 9.3 us per step).
template <bool SPARSE, int QPB, int MINB, int U = -1, bool NT = false>
__global__ __launch_bounds__(QPB * kQuarter, MINB * QPB) void k_loop_step_coded(
    Geom g, float gamma, const uint16_t* __restrict__ code, const float* __restrict__ rows,
    const float* __restrict__ lz, const float* __restrict__ tu, int E,
    const float* __restrict__ b_in, float* __restrict__ b_out, int u,
    const float* __restrict__ in_partials, int in_n,
    const float* __restrict__ in_sum, float* __restrict__ in_sum_out,
    float* __restrict__ out_partials, int dense_blocks, const float* __restrict__ J_in,
    float* __restrict__ J_out, uint8_t* __restrict__ A, int own0, int own1, float scale) {
  using LY = Layout<SPARSE>;
  extern __shared__ float lds[];
  float* sTC = lds;
  float* sL = lds + lds_span(rows_floats(E, SPARSE));
  float* sTu = sL + lds_span(E);
  PP2_PHASE(0);
  const int q = threadIdx.x / kQuarter, tq = threadIdx.x % kQuarter;
  const int tpr = g.wp / 4;
  const int ntiles = (dense_blocks + QPB - 1) / QPB;
  const int tile0 = xcd_remap(blockIdx.x, gridDim.x);
  // cell of this lane in tile tl (lanes past the last row read row rows-1)
#define PP2_CELL(tl, y, x0, ok)                                        \
  const long long t_ = (long long)(QPB * (tl) + q) * kQuarter + tq;     \
  int y = (int)(t_ / tpr);                                              \
  const int x0 = (int)(t_ % tpr) * 4;                                   \
  const bool ok = y < g.rows;                                           \
  if (!ok) y = g.rows - 1
  PP2_CELL(tile0 < ntiles ? tile0 : 0, y, x0, ok);
  CodeWin6 cw;
  Win6 bw;
  load_codes6(code, g.wp, y, x0, cw);
  load_win6(b_in, g.wp, y, x0, x0 == 0, x0 + 4 == g.wp, bw);
  stage_rows(rows, rows_floats(E, SPARSE), sTC);
  stage_rows(lz, E, sL);
  stage_rows(tu, E * LY::tu, sTu);
  // pending input mass: wave 0 reduces the partials (k_sum_finalize's tree)
  // while the dictionary stages, and hands the sum over through LDS
  float* sS = sTu + lds_span(E * LY::tu);
  if (in_partials && threadIdx.x < 64) {
    const float S = wave_reduce_partials(in_partials, in_n);
    if (threadIdx.x == 0) {
      sS[0] = S;
      if (in_sum_out && blockIdx.x == 0) *in_sum_out = S;
    }
  } else if (!in_partials && in_sum_out && blockIdx.x == 0 && threadIdx.x == 0) {
    *in_sum_out = in_sum ? *in_sum : 1.0f;
  }
  // belief gather: LDS slot of T[.][u][i] inside the action-u block, or -1
  // when i is outside u's support on the sparse layout (T == 0 there)
  int slot[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    if constexpr (SPARSE) {
      slot[i] = -1;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < kSupN[u] && kSup[u][j] == i) slot[i] = j;
    } else {
      slot[i] = i;
    }
  }
  __syncthreads();
  const float S = in_partials ? sS[0] : in_sum ? *in_sum : 1.0f;
  const float inv = (1.0f / S) * scale;  // scale: a power of two (1 unsharded)
  PP2_PHASE(1);
  if (tile0 >= ntiles) return;
  {
    // compute only on lanes with a cell (a divergent region, as in the dense
    // kernel); unconditional compute with a guarded store spills heavily
    float local = 0.0f;
    if (ok) {
      belief_cells<SPARSE, U, NT>(g, sTu, sL, slot, inv, cw, bw, y, x0, b_out, local);
      const bool own = y >= own0 && y < own1;
      if (!own) local = 0.0f;
      PP2_PHASE(2);
      if (J_in) {  // (null: a belief update alone, pp2_belief_update)
        Win6 jw;
        load_win6(J_in, g.wp, y, x0, x0 == 0, x0 + 4 == g.wp, jw);
        sweep_cells<SPARSE, NT>(g, sTC, gamma, cw.m0[1], cw.m1[1], jw, y, x0, own, J_out, A);
      }
      PP2_PHASE(3);
    }
    const int d = QPB * tile0 + q;
    if (d < dense_blocks) write_wave_partial(local, out_partials, d);
  }
  // ---- further tiles (grids larger than the resident workgroups)
  for (int tl = tile0 + gridDim.x; tl < ntiles; tl += gridDim.x) {
    PP2_CELL(tl, yy, xx, okk);
    float local = 0.0f;
    if (okk) {
      CodeWin6 c2;
      Win6 w2;
      load_codes6(code, g.wp, yy, xx, c2);
      load_win6(b_in, g.wp, yy, xx, xx == 0, xx + 4 == g.wp, w2);
      belief_cells<SPARSE, U, NT>(g, sTu, sL, slot, inv, c2, w2, yy, xx, b_out, local);
      const bool own = yy >= own0 && yy < own1;
      if (!own) local = 0.0f;
      if (J_in) {
        load_win6(J_in, g.wp, yy, xx, xx == 0, xx + 4 == g.wp, w2);
        sweep_cells<SPARSE, NT>(g, sTC, gamma, c2.m0[1], c2.m1[1], w2, yy, xx, own, J_out, A);
      }
    }
    const int d = QPB * tl + q;
    if (d < dense_blocks) write_wave_partial(local, out_partials, d);
  }
#undef PP2_CELL
  PP2_PHASE(4);
}

template <bool SPARSE, int QPB, int MINB, bool NTS>
__global__ __launch_bounds__(QPB * kQuarter, MINB * QPB) void k_mdp_sweep_coded(
    Geom g, float gamma, const uint16_t* __restrict__ code, const float* __restrict__ rows,
    int E, const float* __restrict__ J_in, float* __restrict__ J_out,
    uint8_t* __restrict__ A) {
  constexpr int NT = QPB * kQuarter;
  extern __shared__ float lds[];
  const int tpr = g.wp / 4;
  const long long nthreads = (long long)g.rows * tpr;
  const int ntiles = (int)((nthreads + NT - 1) / NT);
  int tile = xcd_remap(blockIdx.x, gridDim.x);
  stage_rows(rows, rows_floats(E, SPARSE), lds);
  __syncthreads();
  for (; tile < ntiles; tile += gridDim.x) {
    const long long t = (long long)tile * NT + threadIdx.x;
    const int y = (int)(t / tpr);
    const int x0 = (int)(t % tpr) * 4;
    if (y >= g.rows) continue;
    const bool le = x0 == 0, re = x0 + 4 == g.wp;
    const long long off = (long long)y * g.wp + x0;
    const uint2 m = *reinterpret_cast<const uint2*>(code + off);
    const uint32_t cc[4] = {m.x & 0xffffu, m.x >> 16, m.y & 0xffffu, m.y >> 16};
    float jn[9][4];
    load_jn(J_in, g.wp, y, x0, le, re, jn);
    float best[4];
    uint32_t arg[4];
    coded_sweep4<SPARSE>(lds, cc, jn, gamma, best, arg);
    store_ja<NTS>(J_out, A, off, best, arg);
  }
}


// ---------------------------------------------------------------- step pairs
// Two fused loop steps of one normalisation block in ONE launch, with no
// communication between workgroups: a workgroup owns a 4096-cell tile (the
// dense kernel's 4 blocks).  Step 1 is computed over the tile plus one row
// and a quad on each side (tile + 2 wp + 8 cells) from HBM, into LDS; step 2
// reads its b and J windows from LDS and writes the tile.  Each launch saves
// one launch, one dictionary staging and one dependent HBM round trip per
// two steps for 2 wp + 8 recomputed cells per tile (1.5x step-1 work at
// 1024^2).  Step-1 cells outside rows [0, rows) are the zero halo.  Per cell
// the arithmetic is k_loop_step_coded's; the intermediate belief, values and
// actions are not stored (nobody reads them), the mass partials and actions
// are step 2's, in the dense kernel's cell -> (block, wave) mapping.
// Row shards launch it on a view extended by halo rows (pp2_runtime.cpp
// loop_pair): step 1 then also covers view rows -1 and rows (s1lo/s1hi,
// real neighbour rows read from the deep halo), and only the owned rows
// [own0, own1) store actions and add to the mass.
// 256-thread quarters per workgroup.  Two (2048-cell tiles, two workgroups
// per CU) measured slower: 1024^2 8.5 us/step against 7.7.
constexpr int kPQ = 4;
constexpr int kPTile = kPQ * kQuarter * 4;  // cells per tile
// step-1 region: the tile plus a row per side, plus a quad per side unless
// tiles are whole rows (then the x +- 1 neighbours at the tile ends are the
// zero grid edge)
__host__ __device__ constexpr int pair_region(int wp) {
  return kPTile + 2 * wp + (kPTile % wp == 0 ? 0 : 8);
}


__global__ __launch_bounds__(kPQ * kQuarter, 4) void k_loop_pair_coded(
    Geom g, float gamma, const uint16_t* __restrict__ code, const float* __restrict__ rows,
    const float* __restrict__ lz1, const float* __restrict__ lz2, const float* __restrict__ tu1,
    const float* __restrict__ tu2, int E, int u1, int u2, const float* __restrict__ b_in,
    float* __restrict__ b_out, const float* __restrict__ J_in, float* __restrict__ J_out,
    uint8_t* __restrict__ A, float* __restrict__ out_partials, const float* __restrict__ in_partials,
    int in_n, float* __restrict__ in_sum_out, const float* __restrict__ in_sum, float scale0,
    int dense_blocks, int own0, int own1, int s1lo, int s1hi) {
  using LY = Layout<true>;
  extern __shared__ float lds[];
  PP2_PHASE(0);
  const int nreg = pair_region(g.wp);
  float* sTC = lds;
  float* sL1 = sTC + lds_span(rows_floats(E, true));
  float* sL2 = sL1 + lds_span(E);
  float* sT1 = sL2 + lds_span(E);
  float* sT2 = sT1 + lds_span(E * LY::tu);
  float* sB = sT2 + lds_span(E * LY::tu);  // step-1 belief over the region
  float* sJ = sB + lds_span(nreg);         // step-1 values over the region
  float* sS = sJ + lds_span(nreg);         // the input mass (block-start launch)
  const int q = threadIdx.x / kQuarter;
  const int ntiles = (dense_blocks + kPQ - 1) / kPQ;
  stage_rows(rows, rows_floats(E, true), sTC);
  stage_rows(lz1, E, sL1);
  stage_rows(lz2, E, sL2);
  stage_rows(tu1, E * LY::tu, sT1);
  stage_rows(tu2, E * LY::tu, sT2);
  // block-start launch with the previous launch's mass still pending: wave 0
  // reduces its partials (k_sum_finalize's tree, so the mass is bit-identical
  // to a separately finalised one) while the dictionary stages
  if (in_partials && threadIdx.x < 64) {
    const float S = wave_reduce_partials(in_partials, in_n);
    if (threadIdx.x == 0) {
      sS[0] = S;
      if (blockIdx.x == 0 && in_sum_out) *in_sum_out = S;
    }
  }
  __syncthreads();
  const float inv0 = in_partials ? (1.0f / sS[0]) * scale0
                                 : in_sum ? (1.0f / *in_sum) * scale0 : scale0;
  PP2_PHASE(1);
  for (int tile = xcd_remap(blockIdx.x, gridDim.x); tile < ntiles; tile += gridDim.x) {
    const long long c0 = (long long)tile * kPTile;
    // flat cell of sB[0] / sJ[0] (a quad boundary)
    const long long r0 = c0 - g.wp - (kPTile % g.wp == 0 ? 0 : 4);
    // ---- step 1 over the region: quads of 4 cells, rows outside [s1lo, s1hi) are 0
    for (int qd = threadIdx.x; 4 * qd < nreg; qd += kPQ * kQuarter) {
      const long long f = r0 + 4LL * qd;
      const int y = (int)((f + 2LL * g.wp) / g.wp) - 2;
      const int x0 = (int)(f - (long long)y * g.wp);
      float p[4] = {0.0f, 0.0f, 0.0f, 0.0f}, best[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (y >= s1lo && y < s1hi) {
        const bool le = x0 == 0, re = x0 + 4 == g.wp;
        CodeWin6 cw;
        Win6 w;
        load_codes6(code, g.wp, y, x0, cw);
        load_win6(b_in, g.wp, y, x0, le, re, w);
        float local;
        belief_u(u1, g, sT1, sL1, inv0, cw, w, x0, p, local);
        load_win6(J_in, g.wp, y, x0, le, re, w);
        uint32_t arg[4];
        sweep_vals<false>(sTC, gamma, cw, w, best, arg);  // step 1 stores no actions
      }
      *reinterpret_cast<f4a*>(sB + 4 * qd) = f4a{p[0], p[1], p[2], p[3]};
      *reinterpret_cast<f4a*>(sJ + 4 * qd) = f4a{best[0], best[1], best[2], best[3]};
      if (qd == threadIdx.x) PP2_PHASE(2);
    }
    PP2_PHASE(3);
    __syncthreads();
    PP2_PHASE(4);
    // ---- step 2 over the tile (k_loop_step_coded's lane -> cell mapping)
    const long long t_ = (long long)(kPQ * tile) * kQuarter + threadIdx.x;
    const int y = (int)(t_ / (g.wp / 4));
    const int x0 = (int)(t_ % (g.wp / 4)) * 4;
    float local = 0.0f;
    if (y < g.rows) {
      const bool le = x0 == 0, re = x0 + 4 == g.wp;
      CodeWin6 cw;
      Win6 w;
      load_codes6(code, g.wp, y, x0, cw);
      region_win6(sB, g.wp, y, x0, r0, le, re, w);
      float p[4];
      belief_u(u2, g, sT2, sL2, 1.0f, cw, w, x0, p, local);
      const long long off = (long long)y * g.wp + x0;
      store4<true>(b_out + off, p);
      region_win6(sJ, g.wp, y, x0, r0, le, re, w);
      float best[4];
      uint32_t arg[4];
      sweep_vals(sTC, gamma, cw, w, best, arg);
      if (y >= own0 && y < own1) {
        store_ja<true>(J_out, A, off, best, arg);
      } else {  // a recomputed halo row of a row shard: no actions, no mass
        store4<true>(J_out + off, best);
        local = 0.0f;
      }
    }
    PP2_PHASE(5);
    const int d = kPQ * tile + q;
    if (d < dense_blocks) write_wave_partial(local, out_partials, d);
    __syncthreads();  // the region is rewritten by the next tile
  }
  PP2_PHASE(6);
}

// Per-device launch facts: the CU count (grid caps, loop_pair_fits) and which
// kernels were opted into the large dynamic LDS on that device.  A process may
// drive several devices (a shard group, several contexts).
constexpr int kMaxDevices = 64;
int g_num_cus[kMaxDevices];

int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
  if (g_num_cus[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    g_num_cus[dev] = n;
  }
  return g_num_cus[dev];
}

int coded_grid(int ntiles, int per_cu) {
  const int cap = device_cus() * per_cu;
  return ntiles < cap ? ntiles : cap;
}

}  // namespace

// Opt a kernel into more than the default dynamic LDS once per device (bit d
// of `done`).  A refusal is not fatal here: the launch itself reports an
// oversized request.
void allow_lds(const void* fn, unsigned long long& done) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
  if (done >> dev & 1ull) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDictLdsMaxBytes);
  (void)hipGetLastError();
  done |= 1ull << dev;
}

size_t coded_loop_lds_bytes(int E, bool sparse) {
  return ((size_t)lds_span(rows_floats(E, sparse)) + lds_span(E) +
          lds_span(E * tu_width(sparse)) + 4) * sizeof(float);
}

hipError_t launch_dict_hash(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet C, PlaneSet R,
                            PlaneSet L, uint64_t* out) {
  const long long n = (long long)(g.rows + 2 * g.halo) * g.wp;
  hipLaunchKernelGGL(k_dict_hash, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     st, g, T, C, R, L, out);
  return hipGetLastError();
}

hipError_t launch_dict_gather(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet C, PlaneSet R,
                              PlaneSet L, const int* reps, int E, float* dict) {
  const int n = E * kDictRow;
  hipLaunchKernelGGL(k_dict_gather, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, g, T,
                     C, R, L, reps, E, dict);
  return hipGetLastError();
}

hipError_t launch_dict_verify(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet C, PlaneSet R,
                              PlaneSet L, const uint16_t* code_all, const float* dict, int* bad) {
  const long long n = (long long)(g.rows + 2 * g.halo) * g.wp;
  hipLaunchKernelGGL(k_dict_verify, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     st, g, T, C, R, L, code_all, dict, bad);
  return hipGetLastError();
}

// Launch shapes (workgroups of QPB x 256 threads, MINB per CU; one lane = 4
// cells): the sparse loop kernel 2 x 512 threads (<= 128 VGPRs, 4 waves per
// SIMD, 2 x ~60 KB LDS), the sparse sweep 2 x 1024 (<= 64 VGPRs, 8 waves per
// SIMD); full rows (up to ~160 KB LDS) one 1024-thread workgroup per CU.
hipError_t launch_loop_step_coded(hipStream_t st, const Geom& g, float gamma,
                                  const uint16_t* code, const float* rows, const float* lz,
                                  const float* tu, int E, bool sparse, const float* b_in, float* b_out, int u,
                                  const float* in_partials, int in_n, const float* in_sum,
                                  float* in_sum_out, float* out_partials, const float* J_in,
                                  float* J_out, uint8_t* A, int own0, int own1, float scale) {
  const size_t lds = coded_loop_lds_bytes(E, sparse);
  const int dense_blocks = cells_grid(g, 4);
#define PP2_LOOPC(SP, Q, MB, UU, N)                                                              \
  do {                                                                                          \
    if (lds * MB > kDictLdsMaxBytes) return hipErrorInvalidValue;                               \
    static unsigned long long attr = 0;                                                         \
    allow_lds(reinterpret_cast<const void*>(&k_loop_step_coded<SP, Q, MB, UU, N>), attr);       \
    const int grid = coded_grid((dense_blocks + Q - 1) / Q, MB);                                \
    hipLaunchKernelGGL((k_loop_step_coded<SP, Q, MB, UU, N>), dim3(grid), dim3(Q * kQuarter),   \
                       lds, st,                                                                 \
                       g, gamma, code, rows, lz, tu, E, b_in, b_out, u, in_partials, in_n,      \
                       in_sum, in_sum_out, out_partials, dense_blocks, J_in, J_out, A, own0,    \
                       own1, scale);                                                            \
  } while (0)
#define PP2_LOOPV(UU) PP2_LOOPC(true, 2, 2, UU, true)
  // sparse rows: two 512-thread workgroups per CU (~60-76 KB LDS each, <= 128
  // VGPRs, 4 waves per SIMD), one kernel per action (its support terms
  // only); full rows: one 1024-thread workgroup per CU
  if (sparse) {
    switch (u) {
      case 0: PP2_LOOPV(0); break;
      case 1: PP2_LOOPV(1); break;
      case 2: PP2_LOOPV(2); break;
      case 3: PP2_LOOPV(3); break;
      case 4: PP2_LOOPV(4); break;
      case 5: PP2_LOOPV(5); break;
      case 6: PP2_LOOPV(6); break;
      case 7: PP2_LOOPV(7); break;
      default: PP2_LOOPV(8); break;
    }
  } else {
    PP2_LOOPC(false, 4, 1, -1, false);
  }
#undef PP2_LOOPV
#undef PP2_LOOPC
  return hipGetLastError();
}

size_t loop_pair_lds_bytes(int E, int wp) {
  return ((size_t)lds_span(rows_floats(E, true)) + 2 * lds_span(E) +
          2 * lds_span(E * tu_width(true)) + 2 * lds_span(pair_region(wp)) + 4) * sizeof(float);
}

bool loop_pair_fits(const Geom& g, int E, bool sparse) {
  // Sparse rows, LDS for one 1024-thread workgroup, step 1 over at most 1.6x
  // the tile's cells (MI355X, 2048^2: pairs at 2.0x ran 31.4 us/step against
  // 24.2 for single steps)
  return sparse && E > 0 && loop_pair_lds_bytes(E, g.wp) <= kDictLdsMaxBytes &&
         5 * pair_region(g.wp) <= 8 * kPTile;
}

bool loop_pair_pays(const Geom& g) {
  // a tile for every CU: on fewer tiles the per-step kernel's 2048-cell
  // workgroups keep more CUs busy (MI355X, 512^2: 6.1 us/step per-step vs 7.4
  // paired; 1024^2: 8.6 vs 7.7)
  return (cells_grid(g, 4) + kPQ - 1) / kPQ >= device_cus() * (4 / kPQ);
}

hipError_t launch_loop_pair_coded(hipStream_t st, const Geom& g, float gamma,
                                  const uint16_t* code, const float* rows, const float* lz1,
                                  const float* lz2, const float* tu1, const float* tu2, int E,
                                  int u1, int u2, const float* b_in, float* b_out,
                                  const float* J_in, float* J_out, uint8_t* A,
                                  float* out_partials, const float* in_partials, int in_n,
                                  float* in_sum_out, const float* in_sum, float scale,
                                  int own0, int own1, bool halo_step1) {
  if (!loop_pair_fits(g, E, true) || u1 < 0 || u1 > 8 || u2 < 0 || u2 > 8 ||
      (halo_step1 && g.halo < 2))
    return hipErrorInvalidValue;
  // step-1 rows: the view plus one row per side read from the deep halo, or
  // the view alone with a zero halo (the grid boundary)
  const int s1lo = halo_step1 ? -1 : 0, s1hi = halo_step1 ? g.rows + 1 : g.rows;
  const size_t lds = loop_pair_lds_bytes(E, g.wp);
  static unsigned long long attr = 0;
  allow_lds(reinterpret_cast<const void*>(&k_loop_pair_coded), attr);
  const int dense_blocks = cells_grid(g, 4);
  const int grid = coded_grid((dense_blocks + kPQ - 1) / kPQ, 4 / kPQ);
  hipLaunchKernelGGL(k_loop_pair_coded, dim3(grid), dim3(kPQ * kQuarter), lds, st, g, gamma,
                     code, rows, lz1, lz2, tu1, tu2, E, u1, u2, b_in, b_out, J_in, J_out, A,
                     out_partials, in_partials, in_n, in_sum_out, in_sum, scale, dense_blocks,
                     own0, own1, s1lo, s1hi);
  return hipGetLastError();
}

hipError_t launch_mdp_sweep_coded(hipStream_t st, const Geom& g, float gamma,
                                  const uint16_t* code, const float* rows, int E, bool sparse,
                                  const float* J_in, float* J_out, uint8_t* A) {
  const size_t lds = (size_t)lds_span(rows_floats(E, sparse)) * sizeof(float);
  const long long nthreads = (long long)g.rows * (g.wp / 4);
// Plain stores: non-temporal ones measured slower here (1024^2: 8.8 -> 9.9 us).
#define PP2_SWEEPC(SP, Q, MB)                                                                  \
  do {                                                                                         \
    if (lds * MB > kDictLdsMaxBytes) return hipErrorInvalidValue;                              \
    static unsigned long long attr = 0;                                                        \
    allow_lds(reinterpret_cast<const void*>(&k_mdp_sweep_coded<SP, Q, MB, false>), attr);      \
    const int nt = Q * kQuarter;                                                               \
    const int grid = coded_grid((int)((nthreads + nt - 1) / nt), MB);                          \
    hipLaunchKernelGGL((k_mdp_sweep_coded<SP, Q, MB, false>), dim3(grid), dim3(nt), lds, st, g, \
                       gamma, code, rows, E, J_in, J_out, A);                                  \
  } while (0)
  if (sparse) PP2_SWEEPC(true, 4, 2);
  else PP2_SWEEPC(false, 4, 1);
#undef PP2_SWEEPC
  return hipGetLastError();
}

}  // namespace pp2

#ifdef PP2_PHASE_TRACE
extern "C" int pp2_debug_phase_trace(unsigned long long* out, int nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pp2::g_phase),
                             sizeof(unsigned long long) * 8 * nblocks) == hipSuccess ? 0 : 2;
}

#endif
