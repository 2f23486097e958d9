// pp2_internal.h -- shared declarations between the C-ABI runtime
// (pp2_runtime.cpp) and the gfx950 kernels (pp2_kernels.hip).
//
// HBM layout (DESIGN.md "Data layout"): every per-cell tensor is a set of
// fp32 *planes*.  A plane holds one value per cell of the owned rows plus one
// halo row above and one below; rows are padded to `wp` cells (a multiple of
// 4, pad cells hold 0).  `PlaneSet.p` points at (row 0, plane 0, x 0); element
// (plane k, row y in [-1, rows], x) lives at p[y*rs + k*ps + x].  Row-major
// over planes ([y][k][x], rs = K*wp, ps = wp) is the default: one row of
// cells reads one contiguous K*wp*4-byte stretch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pp2 {

struct PlaneSet {
  float* p;        // (row 0, plane 0, x 0)
  long long rs;    // row stride in floats
  long long ps;    // plane stride in floats
};

struct Geom {
  int rows;        // owned rows of this shard
  int width;       // logical width W
  int wp;          // padded row stride in cells (multiple of 4)
  int row0;        // global index of owned row 0
  int grows;       // global height
  int halo;        // halo rows above and below the owned rows in every plane
};

// Number of workgroups a per-cell launch uses (256 threads, CPT cells each).
int cells_grid(const Geom& g, int cpt);
// Belief-mass partials a belief / loop launch writes: one per wave.
inline int mass_partials(const Geom& g, int cpt) { return 4 * cells_grid(g, cpt); }

// All launchers are asynchronous on `st`.
hipError_t launch_model_gen(hipStream_t st, const Geom& g, const uint8_t* map,
                            int gx, int gy, PlaneSet T, PlaneSet L, PlaneSet R,
                            PlaneSet C);
hipError_t launch_belief_update(hipStream_t st, const Geom& g, int cpt,
                                PlaneSet T, PlaneSet L, const float* b_in,
                                float* b_out, int u, int z,
                                const float* in_sum, float* partials);
hipError_t launch_mdp_sweep(hipStream_t st, const Geom& g, int cpt,
                            float gamma, PlaneSet T, PlaneSet C,
                            const float* J_in, float* J_out, uint8_t* A,
                            bool nt);
// Fused north-star step (belief update + Bellman sweep).  The input belief's
// mass comes from in_partials[0..in_n) (reduced in-kernel) or *in_sum; block
// 0 stores it to *in_sum_out if non-null.  out_partials gets one partial sum
// of the output belief per wave.  Rows [own0, own1) are the shard's own: only
// they add to the mass and store actions (the others are recomputed halo rows
// of an extended-domain launch).  The new belief is scaled by scale / mass
// (scale a power of two, 1 except at the start of a row-shard loop block).
hipError_t launch_loop_step(hipStream_t st, const Geom& g, int cpt, float gamma,
                            PlaneSet T, PlaneSet L, PlaneSet C, const float* b_in,
                            float* b_out, int u, int z, const float* in_partials,
                            int in_n, const float* in_sum, float* in_sum_out,
                            float* out_partials, const float* J_in, float* J_out,
                            uint8_t* A, bool nt, int own0, int own1, float scale = 1.0f);
// Mass of a belief from its n wave partials (n a multiple of 4).
hipError_t launch_sum_finalize(hipStream_t st, const float* partials, int n,
                               float* out);
// out = v[0] + v[1] + ... + v[n-1], in index order.
hipError_t launch_sum_ordered(hipStream_t st, const float* v, int n, float* out);
// sparse: every T row is +0.0 off its action's base-kernel support (the
// dictionary build's check, pp2_ctx::dict_sparse) -- same alphas, bit for bit.
hipError_t launch_fib_sweep(hipStream_t st, const Geom& g, float gamma,
                            PlaneSet T, PlaneSet L, PlaneSet R,
                            PlaneSet a_in, PlaneSet a_out, bool sparse = false);
hipError_t launch_absdiff_max(hipStream_t st, const Geom& g, int planes,
                              PlaneSet cur, PlaneSet snap, float* partials,
                              int* nparts);
hipError_t launch_sum_cells(hipStream_t st, const Geom& g, const float* b,
                            float* partials, int* nparts);
// dense[y*W + x)*K + k]  <->  planes (reference AoS layout <-> SoA planes);
// mass_out (optional) receives *divide_by
hipError_t launch_pack(hipStream_t st, const Geom& g, int K, PlaneSet src,
                       float* dense, const float* divide_by, float* mass_out = nullptr);
hipError_t launch_unpack(hipStream_t st, const Geom& g, int K,
                         const float* dense, PlaneSet dst);
hipError_t launch_pack_u8(hipStream_t st, const Geom& g, const uint8_t* src,
                          uint8_t* dense);

// QV-tree expansion: rewards_out[9] = sum_x b(x) R_a(x);
// stats_out[z][a][10] = {sum_x c, sum_x c*alpha_i}, c = (T_a^T b)(x) L_z(x).
// rpartials >= tiles*9 floats, spartials >= tiles*16*90 floats, P = 9 planes.
hipError_t launch_expand(hipStream_t st, const Geom& g, int cpt, PlaneSet T,
                         const float* b, PlaneSet R, PlaneSet L, PlaneSet F,
                         PlaneSet P, float* rpartials, float* spartials,
                         float* rewards_out, float* stats_out);
// out[0] = sum b, out[1+i] = sum b*alpha_i; partials >= tiles*10 floats;
// mass_out (optional) receives *mass
hipError_t launch_belief_dots(hipStream_t st, const Geom& g, int cpt,
                              const float* b, PlaneSet F, float* partials,
                              float* out, const float* mass = nullptr,
                              float* mass_out = nullptr);
hipError_t launch_scale(hipStream_t st, const Geom& g, float* b, const float* mass);

// Batched fp16 rollouts (pp2_rollout.cpp).  Beliefs: fp16 [copy][rows+2][wp],
// cstride halfs per copy, copy plane origin at row -1.  A chunk is a run of
// rollout_chunk() copies (indices copies[first ..]) sharing the step's action.
int rollout_waves(const Geom& g);       // partials per copy to allocate (>= both passes)
int rollout_step_waves(const Geom& g);  // partials per copy of one step launch
int rollout_leaf_waves(const Geom& g);  // partials per copy of the leaf pass
int rollout_chunk();      // copies per chunk (workgroup) of the selected variant
int rollout_min_chunk();  // smallest chunk of any variant (sizes chunk tables)
// Model source: the coded model (E > 0: code plane, tu_all = the per-action
// raw T tables [u][tstride] with tw floats per entry, sparse = support-only
// rows; dl = L transposed [z][es]) or E = 0 for the T/L planes.  R is always
// the R plane.  Writes bout, then stats_out[copy][3] (k_rollout_reduce).
// istride: halfs between consecutive copies' input planes (0: every copy
// reads the one plane at bin -- the first step, from the root image).
hipError_t launch_rollout_step(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet L,
                               PlaneSet R, const uint16_t* code, const float* tu_all,
                               long long tstride, int tw, const float* dl, int es, int E,
                               bool sparse, const void* bin, void* bout, long long cstride,
                               long long istride, int nchunks, const int* chunk_u, const int* chunk_first,
                               const int* copies, const uint8_t* zs, const float* in_stats,
                               float* partials, float* stats_out, int ncopies);
hipError_t launch_rollout_reduce(hipStream_t st, const float* partials, int nwaves,
                                 int ncopies, float* stats_out);
hipError_t launch_rollout_leaf(hipStream_t st, const Geom& g, PlaneSet F, const void* b,
                               long long cstride, int ncopies, float* partials, float* out);
// The leaf pass on the matrix cores (pp2_rollout_dev.hip): usable when
// rollout_leaf_mfma_ok (16-B aligned copy rows); scratch of
// rollout_leaf_scratch_bytes (B columns, scales, per-slab partials).  pack:
// rebuild B and the scales from F (false: the scratch holds them for F).
bool rollout_leaf_mfma_ok(const Geom& g, long long cstride);
size_t rollout_leaf_scratch_bytes(const Geom& g, int ncopies);
hipError_t launch_rollout_leaf_mfma(hipStream_t st, const Geom& g, PlaneSet F, const void* b,
                                    long long cstride, int ncopies, void* scratch, float* out,
                                    bool pack);

// Dictionary-coded model (pp2_coded.hip).  code: uint16 per cell over rows
// [-1, rows] (same geometry as a plane); dict: kDictRow floats per entry,
// [u][T_u0..T_u8, C_u] (kDictTC) | L[16] | pad.
constexpr int kDictTC = 90;
constexpr int kDictL = 90;       // offset of L[16]
constexpr int kDictTuple = 106;  // floats compared per cell
constexpr int kDictRow = 108;
constexpr size_t kDictLdsMaxBytes = 160 * 1024;
constexpr int kDictMax = 400;  // coded_loop_lds_bytes(kDictMax, false) <= kDictLdsMaxBytes
// Factored sweep rows (the "sparse" layout; generated models always qualify).
// Every T entry off action a's base-kernel support kSup[a][0 .. kSupN[a]) is
// +0.0 (occupied neighbours and traps only move mass to the centre, which is
// in every support), and across the dictionary action a takes at most kFactK
// distinct (gT support quad, C_a) pairs -- 9 on generated models: the 8
// occupancy patterns of its 3 non-centre support cells, and the goal.  The
// LDS image is
//   QT [9][kFactK] quads: gT = fl(gamma * T) at kSup[a][0..3] (zero-padded)
//   CT [9][kFactK] x 4 floats: C_a of the pair at .x (16-B stride, so that
//      one byte offset addresses both tables)
//   IW [E] x 4 uint32: byte a of the 16 = 16 * (pair index of action a)
// so a cell's backup reads one 16-B IW record, then per action one quad and
// one cost from 256-B tables whose 16 entries sit on 16 distinct bank quads
// (conflict-free gathers).  More than kFactK pairs for any action: full rows.
constexpr int kFactK = 16;
// Class tables of the tile-resident loop (pp2_resident.hip), one image at the
// start of its LDS: the pair classes above also fix the raw T support quad
// (the host keys them on it too), and the dictionary's L columns (16 values
// per entry, one per z) take at most kResLK distinct vectors (16 on the grid
// of a generated model, plus the zero vector of the halo rows and pads).
//   QR  [9][kFactK] quads: raw T at kSup[a][0..3] of the class (belief gather,
//       addressed by the same 16 * class byte offsets as QT / CT)
//   LT  [16 z][kResLK]: L_z of the L class
//   LX  [E] bytes (global only): 4 * L class of the entry
constexpr int kResLK = 32;
constexpr int kResQR = 0;
constexpr int kResLT = 9 * kFactK * 4;
constexpr int kResTab = kResLT + 16 * kResLK;  // floats of the LDS image
constexpr int kResLX = kResTab;                // byte table after it (global)
constexpr int kFactQT = 0;
constexpr int kFactCT = 9 * kFactK * 4;
constexpr int kFactIW = 2 * 9 * kFactK * 4;
__host__ __device__ constexpr int rows_floats(int entries, bool sparse) {
  return sparse ? kFactIW + 4 * entries : entries * kDictTC;
}
// Raw T_u floats per entry in the belief gather's LDS table: the support
// cells (sparse, 4) or all 9, padded to an odd stride so that two codes land
// on the same LDS bank only when they differ by a multiple of 64.
constexpr int tu_width(bool sparse) { return sparse ? 5 : 9; }
constexpr int kSupN[9] = {4, 4, 4, 4, 1, 4, 4, 4, 4};
constexpr int kSup[9][4] = {{0, 1, 3, 4}, {0, 1, 2, 4}, {1, 2, 4, 5}, {0, 3, 4, 6}, {4, 0, 0, 0},
                            {2, 4, 5, 8}, {3, 4, 6, 7}, {4, 6, 7, 8}, {4, 5, 7, 8}};
size_t coded_loop_lds_bytes(int entries, bool sparse);
// Opt kernel `fn` into kDictLdsMaxBytes of dynamic LDS on the current device,
// once per device (bit d of `done`).
void allow_lds(const void* fn, unsigned long long& done);
hipError_t launch_dict_hash(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet C, PlaneSet R,
                            PlaneSet L, uint64_t* out);
hipError_t launch_dict_gather(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet C, PlaneSet R,
                              PlaneSet L, const int* reps, int entries, float* dict);
hipError_t launch_dict_verify(hipStream_t st, const Geom& g, PlaneSet T, PlaneSet C, PlaneSet R,
                              PlaneSet L, const uint16_t* code_all, const float* dict, int* bad);
// code = code plane at (row 0, x 0); rows = LDS-layout dictionary rows (E x
// factored if sparse else E x kDictTC, T entries pre-multiplied by gamma); lz =
// the L_z column (E floats); tu = raw T of action u per entry (E x 4 sparse,
// E x 9 full).  Same contract as launch_loop_step (cpt 4).
hipError_t launch_loop_step_coded(hipStream_t st, const Geom& g, float gamma,
                                  const uint16_t* code, const float* rows, const float* lz,
                                  const float* tu, int entries, bool sparse, const float* b_in, float* b_out,
                                  int u, const float* in_partials, int in_n,
                                  const float* in_sum, float* in_sum_out, float* out_partials,
                                  const float* J_in, float* J_out, uint8_t* A, int own0,
                                  int own1, float scale = 1.0f);
// Two fused loop steps in one launch (pp2_coded.hip, sparse rows,
// unsharded): step 1 (u1, L_z1 column lz1, T_u1 table tu1) divides by the
// input mass times scale, step 2 (u2, lz2, tu2) by 1.  The input mass is the
// reduction of in_n pending partials in_partials (k_sum_finalize's tree,
// also stored to *in_sum_out when given), else *in_sum, else 1.  Only rows
// [own0, own1) store actions and add to the mass; halo_step1 (row shards on
// an extended view, g.halo >= 2) computes step 1 on view rows -1 and rows from
// the halo instead of taking them as zero.  Reads b_in /
// J_in, writes b_out / J_out / A and step 2's mass partials.  Returns
// hipErrorInvalidValue when loop_pair_fits is false.
constexpr int kPlaneGuard = 64;  // floats of guard before/after every plane allocation
bool loop_pair_fits(const Geom& g, int entries, bool sparse);
// Whether pairing is faster than single steps on this geometry (a tile per CU).
bool loop_pair_pays(const Geom& g);
hipError_t launch_loop_pair_coded(hipStream_t st, const Geom& g, float gamma,
                                  const uint16_t* code, const float* rows, const float* lz1,
                                  const float* lz2, const float* tu1, const float* tu2,
                                  int entries, int u1, int u2, const float* b_in, float* b_out,
                                  const float* J_in, float* J_out, uint8_t* A,
                                  float* out_partials, const float* in_partials, int in_n,
                                  float* in_sum_out, const float* in_sum, float scale,
                                  int own0, int own1, bool halo_step1);
hipError_t launch_mdp_sweep_coded(hipStream_t st, const Geom& g, float gamma,
                                  const uint16_t* code, const float* rows, int entries,
                                  bool sparse, const float* J_in, float* J_out, uint8_t* A);

// Tile-resident loop (pp2_resident.hip): n fused loop steps of a sparse-coded
// context in one launch, one tile of rt whole rows per CU kept in LDS,
// neighbour rows handed over as data-tagged granules, block-start masses
// behind an arrival counter.  Needs wp % 256 == 0, rt * wp / 4 <= 1024 lanes,
// a tile per CU and the whole dictionary in LDS (resident_plan).  A row
// shard runs it on a *view*: its owned rows extended by e halo rows per side
// (DESIGN.md §6).
constexpr int kResidentMaxSteps = 2048;  // steps per launch (kernel-argument trajectory)
constexpr int kResidentRing = 32;        // partial-mass slots (> 3 x block depth: lagged shard block starts)
constexpr int kResidentSyncArrive = 0;   // sync words: block-start arrivals,
constexpr int kResidentSyncErr = 2;      //   sticky timeout flag
constexpr int kResidentSyncWords = 16;
// Exchange granules per lane and side: 16 B each, four values whose bit 31
// carries the slot use's tag bit (every handed-over value is finite and
// >= +0), so every 4-B word validates itself.  The loop hands over b and J.
constexpr int kResidentGranules = 2;
// 2-D tiles (tc tile columns of tw = wp / tc cells): a tile's first and last
// column cross CUs too, one 8-B {b, j} side granule per row, at most
// kResidentMaxRt rows per tile (rt * tw / 4 <= 1024 lanes, tw >= 256).
constexpr int kResidentMaxRt = 16;
// Lagged shard block starts: a view's partials staged in LDS (<= this many).
constexpr int kResRedFloats = 4096;
struct ResidentPlan {
  int rt = 0, ntiles = 0, threads = 0;
  int tc = 1;  // tile columns (1: tiles of whole rows)
  bool tr = false;  // transposed tiles (shard views): the plan is of transposed_geom(view)
  size_t lds = 0;
};
struct ResidentHead {
  Geom g;                    // the launch's rows: the grid, or a shard's view
  float gamma;
  int E;                     // dictionary entries
  const uint16_t* code;      // code plane (view row 0, x 0)
  const float* rows;         // factored sweep rows
  const float* rfact;        // class tables: kResTab floats (QR, LT), then the LX bytes
  const float* b_in;         // step 0's input belief / value planes (view row 0)
  const float* j_in;
  float* b_out;              // the last step's output planes (never b_in / j_in:
  float* j_out;              //   a run that fails leaves its inputs intact)
  float* xch;                // exchange granules, resident_xch_floats(): [step & 1][tile][top, bottom][wave][kResidentGranules][lane] x 16 B
  uint8_t* A;                // actions (view row 0; owned rows stored)
  int n, kstep0, depth, rt, ntiles, nparts;
  int tc;                    // tile columns (ResidentPlan::tc)
  int own0, own1;            // owned view rows: only they store b', J', A and add to the mass
  int ows;                   // TR plans: the grid's row stride (a.g is the transposed view)
  int red_lds;               // shard mode 2: the lagged partials are staged in LDS
                             //   (kResRedFloats more dynamic LDS at launch)
  int shard;                 // 1: block starts inside the run scale by 2^k from the view's
                             //   mass (no cross-rank reduction), k summed into *scale_out;
                             // 2: the same, k chosen from the view's mass one block
                             //   earlier (lagged: no grid-wide wait at a block start)
  float bscale;              // block-start scale (2^96, or 1 for depth 1)
  const float* in_partials;  // step 0's pending input mass (block start), or null
  int in_n;
  float* in_sum_out;         // receives that mass (tile 0)
  const float* in_sum;       // step 0's finalised input mass when in_partials is null
  float* ring;               // kResidentRing x nparts partial slots
  float* out_partials;       // the last step's partials (never in_partials)
  unsigned* sync;            // kResidentSyncWords sync words
  unsigned* err_host;        // pinned host word: set with the sticky error word
  int* scale_out;            // shard: the run's total power-of-two shift (tile 0)
  unsigned arrive_base;      // arrival counter of earlier launches (epoch-tagged)
  unsigned slot_use[2];      // uses of exchange slots 0 / 1 by earlier launches
  int stall_tile;            // diagnostic (tests): this tile returns at once, -1 none
};
// Runs of at most kResidentShortSteps steps launch a kernel instance whose
// trajectory argument holds just that many steps: 256 B of kernel arguments
// instead of ~2.3 KB, about 3 us less host time per launch from an idle
// stream (tools/micro/kernarg_cost.hip).
constexpr int kResidentShortSteps = 24;
struct ResidentRun : ResidentHead {
  uint8_t uz[kResidentMaxSteps];  // u | z << 4 per step
};
// Resident MDP solve (pp2_mdp_solve): sweeps in blocks of kSolveBlock, a
// convergence check after each, at most max_blocks per launch.
constexpr int kSolveBlock = 100;
struct SweepRun {
  Geom g;
  float gamma;
  int E;
  const uint16_t* code;
  const float* rows;
  const float* j_in;   // the input values
  float* j_out;        // the last sweep's values (never j_in)
  float* snap;         // convergence snapshot (read at start, written at the end)
  uint8_t* A;
  float* xch;
  unsigned* sync;
  unsigned* err_host;  // pinned host word, set with the sticky error word
  float* tile_max;     // 2 x ntiles per-tile maxima
  int* res;            // {sweeps done, norm bits}
  unsigned arrive_base;
  unsigned slot_use[2];  // uses of exchange slots 0 / 1 by earlier launches
  int rt, ntiles;
  int max_blocks;      // blocks per launch
  int cap_blocks;      // stop after this many blocks (0: no cap)
  double thresh;       // stop when norm <= thresh
  int nsweeps;         // > 0: exactly this many sweeps, no convergence checks
  int stall_tile;      // diagnostic (tests): this tile returns at once, -1 none
};
size_t resident_lds_bytes(const Geom& g, int E, int rt, int tc);
// Plans fail (the caller falls back BEFORE launching) unless every tile can
// be resident at once: occupancy per CU x ncus >= tiles (one 1024-lane
// workgroup per CU at these LDS sizes).
bool solve_plan(const Geom& g, int E, int ncus, ResidentPlan* p);
hipError_t launch_sweep_resident(hipStream_t st, const ResidentPlan& p, const SweepRun& a);
inline size_t resident_xch_floats(const Geom& g, int ntiles) {
  // [step & 1][tile][top, bottom][wave of row][granule][lane] 16-B granules
  // (sized for whole-row tiles, the most), then the 2-D tiles' side granules
  // [step & 1][tile][left, right][row < kResidentMaxRt] x 8 B
  return (size_t)2 * ntiles * 2 * (g.wp / 256) * kResidentGranules * 64 * 4 +
         (size_t)2 * ntiles * 2 * kResidentMaxRt * 2;
}
// tc_pref: 0 = automatic (two tile columns when whole-row tiles would hold
// fewer than 4 rows and 2-D tiles hold 4 or more), 1 = whole rows, 2 = two
// tile columns whenever they fit (and whole rows do: else no plan changes),
// 3 = transposed tiles when allow_tr (a shard view) and they fit: the plan is
// then of transposed_geom(g).
bool resident_plan(const Geom& g, int E, int ncus, ResidentPlan* p, int tc_pref = 0,
                   bool allow_tr = false);
// The kernel geometry of transposed tiles over view g: rows = g's row stride
// (its columns), row stride = g.rows (its rows; a multiple of 256).
inline Geom transposed_geom(const Geom& g) {
  Geom t = g;
  t.rows = g.wp;
  t.width = g.rows;
  t.wp = g.rows;
  t.row0 = 0;
  t.grows = g.wp;
  t.halo = 0;
  return t;
}
hipError_t launch_loop_resident(hipStream_t st, const ResidentPlan& p, const ResidentRun& a);
// Row-shard boundary kernels (pp2_resident.hip).  vec holds one
// record of kVecRec floats per rank, {owned mass, shift, lost}: the mass of the
// n partials (k_sum_finalize's tree), (float) *shift (0 if shift is null) and,
// with err_word (an RCCL shard's sticky resident error word), 1 if the word is
// set, else 0.  Every other rank's record := 0, so that an all-reduce (sum)
// shares the records exactly -- or the records travel point to point
// (exchange_halos_k with records, grouped with the halo rows).
constexpr int kVecRec = 3;
hipError_t launch_shard_mass_vec(hipStream_t st, const float* partials, int n, const int* shift,
                                 float* vec, int nranks, int rank, const unsigned* err_word);
// After the all-reduce of vec: C = min over ranks of the shifts; rows [r0, r1)
// of plane b (row stride wp) are scaled by 2^(C - shift_q), q = the rank the
// row came from (rank - 1 above row 0, rank + 1 at rows >= own_rows), and
// *mass_out = sum over q in rank order of ldexp(m_q, C - shift_q).
// With err_host, a nonzero `lost` in any record (some rank lost a run) sets *err_host.
hipError_t launch_shard_rebase(hipStream_t st, const float* vec, int nranks, int rank,
                               float* b, int wp, int r0, int r1, int own_rows, float* mass_out,
                               unsigned* err_host);

}  // namespace pp2
