// pp2_ctx.h -- private: the context struct and helpers shared by the C-ABI
// translation units (pp2_runtime.cpp, pp2_tree.cpp).  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <initializer_list>
#include <mutex>
#include <string>
#include <vector>

#include "pp2.h"
#include "pp2_internal.h"

using pp2::Geom;
using pp2::PlaneSet;

namespace pp2rt {

int set_err(int code, const char* fmt, ...);

#define HIPCHK(expr)                                                        \
  do {                                                                      \
    hipError_t e_ = (expr);                                                 \
    if (e_ != hipSuccess)                                                   \
      return set_err(PP2_EHIP, "%s failed: %s (%s:%d)", #expr,              \
                     hipGetErrorString(e_), __FILE__, __LINE__);            \
  } while (0)

#define NCCLCHK(expr)                                                       \
  do {                                                                      \
    ncclResult_t r_ = (expr);                                               \
    if (r_ != ncclSuccess)                                                  \
      return set_err(PP2_ERCCL, "%s failed: %s", #expr,                     \
                     ncclGetErrorString(r_));                               \
  } while (0)

#define CHECK(expr)                 \
  do {                              \
    int s_ = (expr);                \
    if (s_ != PP2_OK) return s_;    \
  } while (0)

constexpr int kGuard = pp2::kPlaneGuard;  // floats of guard before/after each plane set
// Halo rows allocated per side in row-sharded contexts: the per-step paths
// exchange up to kMaxNormBlock of them per block, the resident shard runs up
// to all (one exchange per up to kShardHalo steps).
constexpr int kShardHalo = 128;
// ... but only the per-cell b / J planes and the code plane carry them: the
// dense model and FIB planes (568 of the 590 bytes per cell) keep
// kDenseHalo rows per side, all the per-step paths read (kdepth_max <=
// kMaxNormBlock); the model generation of a deeper shard writes the deep
// rows into a transient full-halo copy that only the code plane keeps
// (pp2_model_generate), so a 2048^2 8-shard group allocates < 10 % above
// the unsharded planes.
constexpr int kDenseHalo = 8;
// Loop normalisation blocks (row shards, and PP2_TUNE_NORM_BLOCK > 1) start
// by dividing the belief by its exact (global) mass and multiplying by 2^96
// (exact), then divide by 1: the stored belief decays by < 8 observation
// probabilities inside a block, and 2^96 keeps cells far above the
// flush-to-zero range (at P(z) >= 1e-3 per step, every normalised value above
// FLT_MIN stays representable), while normalised cells <= 1 times 2^96 stay
// far below FLT_MAX.  Reads divide by the true mass.
constexpr float kBlockScale = 79228162514264337593543950336.0f;  // 2^96
constexpr int kMaxNormBlock = 8;
// a lagged resident shard block (depth <= kMaxNormBlock) reuses mass ring
// slots race-free only while 3 depth + 1 < kResidentRing (launch_loop_resident)
static_assert(3 * kMaxNormBlock + 1 < pp2::kResidentRing, "normalisation block vs mass ring");

// A set of K planes over rows [-1, rows] (one halo row each side).
struct Planes {
  float* alloc = nullptr;
  size_t floats = 0;
  PlaneSet v{nullptr, 0, 0};
  int K = 0;
};

struct PbviState;  // pp2_pbvi.cpp

}  // namespace pp2rt

using pp2rt::Planes;
using pp2rt::set_err;

struct pp2_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  Geom g{};
  int32_t gx = 0, gy = 0;
  float gamma = 0.95f;
  int cpt = 4;
  bool nt_streams = true;   // non-temporal loads of the once-read T/C streams
  bool model_ready = false;

  uint8_t* d_map = nullptr;  // the map, indexed by global row (only rows [row0 - halo - 1,
                             // row0 + rows + halo + 1) exist: d_map_alloc)
  uint8_t* d_map_alloc = nullptr;
  Planes T, L, R, C;         // 81, 16, 9, 9 planes
  Planes b[2];               // belief ping-pong (1 plane)
  int bcur = 0;
  float* bsum = nullptr;     // device float[2]: mass of b[0], b[1]
  Planes J[2], Jsnap;        // value ping-pong + convergence snapshot
  int jcur = 0;
  uint8_t* A = nullptr;      // rows * wp actions
  Planes fib[2], fibsnap;    // FIB alphas (9 planes)
  int fcur = 0;
  unsigned fib_version = 1;  // bumped whenever the current alphas change (planner caches)
  unsigned pbvi_version = 1;  // bumped whenever the PBVI alpha vectors change (planner caches)
  int dense_halo = 1;         // halo rows of the dense model / FIB planes (min(g.halo, kDenseHalo))
  bool fib_finite = true;          // every FIB alpha finite: the sparse / LDS sweeps apply
  float* pbuf[2] = {nullptr, nullptr};  // per-block partial masses of b[0], b[1]
  bool pending[2] = {false, false};     // mass of b[i] still in pbuf[i]
  int pcount[2] = {0, 0};               // number of partials in pbuf[i]
  float* rpartials = nullptr;  // convergence-check partials
  int partials_cap = 0;
  // dictionary-coded model (pp2_coded.hip), rebuilt whenever the model changes
  uint16_t* code_alloc = nullptr;  // code plane allocation (guards + rows -1..rows)
  uint16_t* d_code = nullptr;      // code plane at (row 0, x 0)
  float* d_dict = nullptr;         // kDictMax * kDictRow floats
  float* d_rows = nullptr;         // LDS-layout rows, gamma*T (rows_floats: factored or kDictTC)
  float* d_dl = nullptr;           // L transposed: [z][entry]
  float* d_tu = nullptr;           // raw T per action: [u][entry][4 sparse | 9 full]
  float* d_rfact = nullptr;        // resident class tables (pp2_internal.h kRes*)
  int dict_n = 0;                  // entries; 0 = no dictionary (dense path only)
  bool dict_sparse = false;        // every T row is zero off the base-kernel support
  bool dict_t_finite = false;      // every dictionary T entry is finite
  bool dict_tl_nonneg = false;     // every dictionary T and L entry finite and >= +0
  bool dict_rfact = false;         // d_rfact valid: raw T and L by class (<= 16 each)
  // the sparse rows' T == 0 skip needs finite, non-negative beliefs (not -0):
  // false after a pp2_belief_set that breaks that, until the next one
  bool belief_sparse_ok = true;
  bool use_coded = true;           // PP2_TUNE_CODED_MODEL
  void* staging = nullptr;     // dense host-layout staging buffer
  size_t staging_bytes = 0;

  // Row-sharded loop blocks: halo rows are exchanged kdepth
  // rows deep every kdepth loop steps; only a block's first step normalises.
  int kdepth = 1;          // loop halo depth in use
  int kdepth_max = 1;      // min(g.halo, the smallest shard's rows)
  int kstep = 0;           // loop step within the current halo / normalisation block
  int norm_block = 8;      // unsharded loop: steps per exact normalisation (PP2_TUNE_NORM_BLOCK)

  // pp2_loop_run on an unsharded sparse-coded context fuses the steps of a
  // normalisation block in pairs (pp2::launch_loop_pair_coded)
  int step_pairs = 1;              // PP2_TUNE_STEP_PAIRS

  // pp2_loop_run's tile-resident loop (pp2_resident.hip), PP2_TUNE_RESIDENT
  int resident = 1;
  int ncus = 0;                    // CUs of the device
  int res_plan_e = -1;             // dictionary size the plan below was made for
  bool res_ok = false;
  pp2::ResidentPlan res_plan{};
  unsigned* res_sync = nullptr;    // sync words (flags, counters, error)
  float* res_ring = nullptr;       // kResidentRing slots of mass partials
  float* res_xch = nullptr;        // exchange rows
  unsigned res_slot[4] = {0, 0, 0, 0};  // uses of the exchange slots 0 / 1 (tag bits):
                                        // loop kernel's region, then the sweep kernel's
  unsigned res_arrive = 0;         // arrival counter (epoch-tagged)
  int sol_plan_e = -1;             // resident MDP solve (k_sweep_resident): plan for dict_n
  bool sol_ok = false;
  pp2::ResidentPlan sol_plan{};
  int res_ntiles = 0;              // tiles the sync words / exchange rows were sized for
  float* res_tmax = nullptr;       // 2 x ntiles per-tile convergence maxima
  int* res_out = nullptr;          // {sweeps, norm bits} of a resident solve launch
  // pinned words the kernels write: {sweeps, norm bits, solve error word, -},
  // then one error word per journalled launch
  unsigned* res_host = nullptr;
  int res_launches = 0, sol_launches = 0;  // pp2_resident_launches
  // Every resident launch is journalled until verified (resident_settle): its
  // inputs stay intact (outputs go to the other ping-pong buffers), and a
  // launch queued behind an unverified one exits at once if an earlier one
  // timed out (the device error word is sticky), so the first failed launch
  // and all later ones are re-run from the failed one's inputs with per-step
  // launches before anything reads their outputs.  Resident loop runs and
  // sweeps queue up to kResidentChain launches this way (no host sync between
  // back-to-back calls); every other entry point verifies first.
  struct ResidentJournal {
    int kind = 0;                  // 1 loop run, 2 sweeps, 3 shard loop run
    int n = 0;
    int bcur = 0, jcur = 0, kstep = 0, pcount[2] = {0, 0};
    bool pending[2] = {false, false};
    std::vector<uint8_t> us, zs;
  };
  static constexpr int kResidentChain = 16;
  static constexpr int kResHostChain = 4;  // res_host index of launch 0's error word
  std::vector<ResidentJournal> journal;    // unverified launches, oldest first
  int res_fallbacks = 0;           // launches re-run after a timeout (pp2_resident_status)
  int res_stall_tile = -1;         // PP2_TUNE_RESIDENT_STALL (tests)
  int res_cus = 0;                 // PP2_TUNE_RESIDENT_CUS: CUs the plans may use (0: all)
  int res_tc_pref = 0;             // PP2_TUNE_RESIDENT_TILE_COLS (0: automatic)
  long long agree_gen = 0;         // model builds + tuning calls (RCCL shards: equal on all ranks)
  long long agree_done = -1;       // agree_gen at the ranks' last agreement on agreed_e
  int agreed_e = 0;                // the resident halo depth all ranks agreed on (0: none)
  int res_loop_tc = 0;             // tile columns of the last loop launch (0: fresh buffers)
  // row shards on the resident loop: halo depth per resident
  // launch, the run's power-of-two shift and the {mass, shift} rank vector
  int res_halo = 0;                // PP2_TUNE_RESIDENT_HALO (0: the most the shards allow)
  int shard_lag = 0;               // PP2_TUNE_SHARD_LAG (resident shard block starts)
  int min_shard_rows = 0;          // smallest shard of the grid (comm init / group create)
  int res_view_e = -1;             // view extension the plan below was made for
  int res_e = 0, res_e_dict = -1;  // shard_resident_e's answer and the dictionary it is for
  int* d_shift = nullptr;          // int: the last shard-resident run's shift
  float* d_vec = nullptr;          // kVecRec x nranks floats: {mass, shift, lost} per rank
  bool shift_pending = false;      // the pending mass comes with *d_shift (rebase owed)
  // a shard-resident run timed out: belief / values unusable until set again
  bool lost_belief = false, lost_values = false;

  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  hipStream_t comm_stream = nullptr;  // RCCL operations when use_comm_stream (PP2_TUNE_COMM_STREAM)
  bool use_comm_stream = false;
  hipEvent_t ev_enter = nullptr, ev_leave = nullptr;
  // PP2_TUNE_COMM_TIMING: every RCCL round bracketed by timing events on the
  // stream it runs on (pp2_comm_rounds reads and clears them)
  static constexpr int kCommTimed = 256;
  bool comm_timing = false, comm_open = false;
  std::vector<hipEvent_t> comm_ev;  // 2 * kCommTimed (begin, end) pairs, made on demand
  int comm_nev = 0;                 // rounds recorded since the last pp2_comm_rounds
  long long comm_dropped = 0;       // rounds beyond kCommTimed (not timed)
  pp2_shard_group* group = nullptr;  // single-process shard group, if any
  int grank = 0;                     // rank (row-block order) inside the group
  int group_size = 0;                // shards in the group

  pp2rt::PbviState* pbvi = nullptr;  // PBVI belief set / alpha vectors (pp2_pbvi.cpp)
};

namespace pp2rt {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// halo < 0: the context's own (g.halo); the dense sets take c->dense_halo
int alloc_planes(pp2_ctx* c, Planes* P, int K, int halo = -1);
void free_planes(Planes* P);
int ensure_staging(pp2_ctx* c, size_t bytes);
int check_ctx(pp2_ctx* c);          // null check, resident_settle, lost shard state
int check_ctx_settled(pp2_ctx* c);  // null check, resident_settle
int check_model(pp2_ctx* c);
size_t owned_cells(const pp2_ctx* c);
int download_planes(pp2_ctx* c, const Planes& P, float* host, const float* divide_by);
int belief_update_impl(pp2_ctx* c, uint8_t u, uint8_t z, bool fuse_with_sweep);
int launch_belief(pp2_ctx* c, const float* b_in, float* b_out, uint8_t u, uint8_t z,
                  const float* mass, float* partials);
int loop_step_fused(pp2_ctx* c, uint8_t u, uint8_t z, bool eager_mass);
int ensure_mass(pp2_ctx* c);
void break_pipeline(pp2_ctx* c);
// One fused step over the owned rows extended by e rows each side (partials
// of the new belief into pbuf[bcur ^ 1]; *nparts = their count).
int loop_launch(pp2_ctx* c, int e, uint8_t u, uint8_t z, const float* in_partials, int in_n,
                const float* in_sum, float* in_sum_out, int* nparts, float scale = 1.0f);
int mdp_sweep_once(pp2_ctx* c);
int build_model_dict(pp2_ctx* c);
bool coded_active(const pp2_ctx* c);
// Step pairs (k_loop_pair_coded) on this context: sparse coded model, a
// block depth >= 2, a fitting geometry and (unless PP2_TUNE_STEP_PAIRS = 2
// forces it) a tile per CU.
bool pairs_apply(pp2_ctx* c);
// One pair launch on the view extended by e rows per side (pp2_runtime.cpp).
int pair_launch(pp2_ctx* c, int e, bool shard, uint8_t u1, uint8_t z1, uint8_t u2, uint8_t z2,
                const float* in_partials, int in_n, float* in_sum_out, const float* in_sum,
                float scale, int* nparts);
int fib_sweep_once(pp2_ctx* c);
int absdiff_local_max(pp2_ctx* c, const Planes& cur, const Planes& snap, float* out);

// Resident launches (pp2_runtime.cpp): verify the journalled launch, re-run
// it on per-step launches if it timed out (every entry point, via check_ctx).
int resident_settle(pp2_ctx* c);
// Row shards on the resident loop: the view extension of the
// shard's runs (0: not eligible), its plan and buffers, the {mass, shift}
// post into d_vec's slot `rank`, the rebase of rows [r0, r1) once d_vec holds
// every shard's slot, and one launch of m <= e steps.
int shard_resident_e(pp2_ctx* c);
bool shard_resident_ready(pp2_ctx* c, int e);
int shard_post_mass(pp2_ctx* c, int nranks, int rank);
int shard_rebase(pp2_ctx* c, int nranks, int rank, int r0, int r1);
int shard_resident_launch(pp2_ctx* c, int e, int m, const uint8_t* us, const uint8_t* zs);
int loop_run_launches(pp2_ctx* c, int n, const uint8_t* us, const uint8_t* zs);

// Halo-exchanged state of a shard.
enum HaloKind { HALO_BELIEF, HALO_VALUE, HALO_FIB };
const Planes& halo_planes(pp2_ctx* c, HaloKind k);
int upload_planes(pp2_ctx* c, Planes& P, const float* host);

// Reference text formats: "%15.8f" values, per_line to a line / "%u" per line.
int write_text(const std::string& path, const std::vector<float>& v, int per_line);
int read_text(const std::string& path, std::vector<float>& v);
int read_actions(const std::string& path, std::vector<uint8_t>& v);
std::string join(const char* dir, const char* name);

void pbvi_free(pp2_ctx* c);
// The context's PBVI alpha vectors (device rows of ld floats, Sp rows); ESTATE if none.
int pbvi_alphas(pp2_ctx* c, const float** alpha, int* S, int* Sp, int* ld);
// d_dots[i*S + k] = inner_product(belief i, alpha k) for n device rows of ld floats
int pbvi_eval_device(pp2_ctx* c, int n, const float* d_beliefs, int ld, float* d_dots);

}  // namespace pp2rt
