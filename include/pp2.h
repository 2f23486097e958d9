/*
 * pp2.h -- C ABI of libpp2_hip.so, the MI355X (gfx950) implementation of the
 * path_planning_2d planner's data-parallel core.
 *
 * Drop-in boundary.  The reference has no library API: its ROS node classes
 * call C++-linkage free functions and launch CUDA kernels on global device
 * pointers.  Every entry point below replaces one of those
 * functions / kernel launches; the replaced reference interface is cited as
 * path:line relative to /root/reference/path_planning_2d/.  INTEGRATION.md
 * shows the edits a maintainer makes in the catkin package to bind them.
 *
 * Conventions
 *  - Every function returns a pp2_status; nothing calls exit() (the
 *    reference's checkCudaErrors exits: helper_cuda.h:984-999).
 *    pp2_last_error() returns a message for the last failure on this thread.
 *  - A context is one grid (or one row shard of a grid) on one device; it
 *    owns all device memory.  Host pointers are caller-owned and only read or
 *    written during the call.  A context is not thread-safe.
 *  - All work is enqueued on the context's stream (its own, or one set with
 *    pp2_set_stream); functions that return host data synchronise it.
 *  - Host arrays use the reference's layouts: T[hw][9 u][9 s'],
 *    L[hw][16 z], R/C[hw][9 u], beliefs/values[hw] with idx = y*W + x.
 *  - Action u in 0..8 is the 3x3 raster with 4 = stay; observation z in 0..15
 *    is m3<<3|m2<<2|m1<<1|m0 (src/pomdp/path_planning_2d.cu:205-207).
 */
#ifndef PP2_H
#define PP2_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PP2_ABI_VERSION 3

typedef enum {
  PP2_OK = 0,
  PP2_EINVAL = 1,   /* bad argument / shape */
  PP2_EHIP = 2,     /* HIP runtime error */
  PP2_EIO = 3,      /* file I/O or parse error (text model/FIB formats) */
  PP2_ENOMEM = 4,   /* device or host allocation failed */
  PP2_ESTATE = 5,   /* call not valid in the current state */
  PP2_ERCCL = 6     /* RCCL error (sharded contexts) */
} pp2_status;

typedef struct pp2_ctx pp2_ctx;

int pp2_abi_version(void);
const char* pp2_status_string(int status);
const char* pp2_last_error(void);
int pp2_device_count(int* count);

/* ---------------------------------------------------------------- lifetime
 * Replaces allocateDeviceMemory(H,W) / freeDeviceMemory()
 * (src/mdp/path_planning_2d_cuda.cu:40-74), allocateDeviceMemoryOfModel /
 * freeDeviceMemoryOfModel (src/pomdp/model_generation_cuda.cu:41-72),
 * allocateDeviceMemoryOfFIB / freeDeviceMemoryOfFIB
 * (src/pomdp/fast_informed_bound_cuda.cu:54-94) and the dev_* / host_*
 * globals they fill.  `map` is the H*W occupancy grid (1 = occupied) that
 * loadMapFromFile() produces (src/pomdp/path_planning_2d.cu:243-257); it is
 * copied.  (goal_x, goal_y) and gamma are the node's goal_x/goal_y/
 * discount_factor parameters. */
int pp2_create(pp2_ctx** out, int device, uint32_t height, uint32_t width,
               const uint8_t* map, int32_t goal_x, int32_t goal_y, float gamma);
/* Row shard [row_begin, row_end) of a global_height x width grid (no
 * reference counterpart: the reference is single-GPU).  `global_map` is the
 * whole grid.  Once pp2_shard_comm_init has been called on every shard,
 * shards exchange halo rows over RCCL: loop steps k rows deep every k steps
 * (PP2_TUNE_HALO_DEPTH, or e rows per resident launch of up to e steps,
 * PP2_TUNE_RESIDENT_HALO), sweeps and belief-only updates one row per step. */
int pp2_create_shard(pp2_ctx** out, int device, uint32_t global_height,
                     uint32_t width, uint32_t row_begin, uint32_t row_end,
                     const uint8_t* global_map, int32_t goal_x, int32_t goal_y,
                     float gamma);
int pp2_destroy(pp2_ctx* ctx);
/* Enqueue on a caller stream (a hipStream_t, e.g. torch's current stream);
 * NULL restores the context's own stream. */
int pp2_set_stream(pp2_ctx* ctx, void* hip_stream);
int pp2_synchronize(pp2_ctx* ctx);
/* rows = owned rows, row_stride = padded cells per row in device planes. */
int pp2_get_geometry(pp2_ctx* ctx, uint32_t* rows, uint32_t* width,
                     uint32_t* row_stride, uint32_t* row_begin);
/* Tuning: cells per lane of the streaming kernels (1, 2 or 4; default 4). */
int pp2_set_cells_per_lane(pp2_ctx* ctx, int cpt);
/* Tuning knobs (results are identical for every setting):
 *  PP2_TUNE_CELLS_PER_LANE  1, 2 or 4
 *  PP2_TUNE_NT_STREAMS      1 (default) = non-temporal loads of the
 *                           once-read T/C streams (loop and sweep kernels,
 *                           CPT 4): -8 % time per loop step measured
 *  PP2_TUNE_CODED_MODEL     1 (default) = loop step and MDP sweep read the
 *                           dictionary-coded model (pp2_model_dict_info)
 *                           when one exists, and FIB sweeps skip the T
 *                           entries the dictionary proved zero; 0 = always
 *                           the dense planes and full sums */
#define PP2_TUNE_CELLS_PER_LANE 1
#define PP2_TUNE_NT_STREAMS 2
#define PP2_TUNE_CODED_MODEL 3
/*  PP2_TUNE_HALO_DEPTH      row shards (RCCL or shard group), launch-per-step
 *                           loop: steps per halo exchange = halo rows
 *                           exchanged, 1..8 (default: the most the smallest
 *                           shard allows) */
#define PP2_TUNE_HALO_DEPTH 4
/*  PP2_TUNE_COMM_STREAM     0 (default): RCCL calls are issued on the context's
 *                           stream; 1: on a dedicated stream entered and left
 *                           through events */
#define PP2_TUNE_COMM_STREAM 5
/*  PP2_TUNE_NORM_BLOCK      unsharded pp2_loop_step: 1 = divide by the exact
 *                           mass every step (bit-exact with per-step host
 *                           normalisation); k = 2..8 (default 8) = divide by
 *                           the exact mass times 2^96 at the first step of
 *                           every k and by 1 in between (beliefs equal to
 *                           rounding; values and actions unchanged) */
#define PP2_TUNE_NORM_BLOCK 6
/*  PP2_TUNE_STEP_PAIRS      1 (default): pp2_loop_run (and
 *                           pp2_shard_group_loop_run) on a context with a
 *                           sparse coded model runs two steps of a
 *                           normalisation / halo block per launch (the first
 *                           over the tile plus a one-row halo, kept in LDS)
 *                           where the grid has a 4096-cell tile per CU;
 *                           2 = pairs on any fitting grid (tests);
 *                           0 = one launch per step.  Results are
 *                           bit-identical either way. */
#define PP2_TUNE_STEP_PAIRS 7
/*  PP2_TUNE_RESIDENT        1 (default): pp2_loop_run on an unsharded context
 *                           with a sparse coded model whose grid fits one
 *                           tile of whole rows per CU (width padded to a
 *                           multiple of 256, rows * width <= 4096 * CUs, the
 *                           dictionary in LDS) runs the whole trajectory in
 *                           one launch (the tile-resident loop, up to 2048
 *                           steps per launch); 0 = step pairs / single steps.
 *                           pp2_mdp_solve and pp2_mdp_sweep(n >= 2) run as
 *                           resident sweeps under the same conditions.
 *                           Results are bit-identical either way.  A plan
 *                           whose tiles cannot all be resident at once is
 *                           never launched.  Resident launches of this
 *                           process run one at a time per device.  A launch
 *                           that still cannot get every tile onto the GPU
 *                           within 0.25 s (another process holding CUs) ends
 *                           early, leaves its inputs intact, and the next
 *                           call on the context re-runs it on per-step
 *                           launches before reading anything (same bits; the
 *                           context then stays on them: pp2_resident_status).
 *                           Consequence: a call after a resident launch
 *                           first waits for that launch to finish -- except
 *                           pp2_loop_run and pp2_mdp_sweep(n >= 2) taking
 *                           the resident path again, which queue behind up
 *                           to 16 unverified launches without a host sync
 *                           (a launch queued behind one that timed out does
 *                           nothing, and all of them are re-run). */
#define PP2_TUNE_RESIDENT 8
/*  PP2_TUNE_RESIDENT_HALO   row shards: the loop runs on the resident kernel
 *                           when a view of the owned rows plus e halo rows
 *                           per side fits one tile per CU; a run of n steps
 *                           is ceil(n / e) launches of up to e steps, each
 *                           after one exchange of e halo rows and one
 *                           {mass, shift} all-reduce.  Value
 *                           = the largest e to use (0, default: the most the
 *                           halo allocation of 128 rows, the smallest shard
 *                           and the CUs allow).  Values and actions are
 *                           bit-identical to the unsharded grid either way. */
#define PP2_TUNE_RESIDENT_HALO 9
/*  PP2_TUNE_RESIDENT_TILE_COLS  tiles of the resident loop: 0 (default) =
 *                           whole rows, or two tile columns (2-D tiles whose
 *                           first and last columns cross CUs as well) when
 *                           whole-row tiles would hold fewer than 4 rows and
 *                           2-D tiles hold 4 or more (a 256 x 2048 rank share
 *                           of the 2048^2 grid on its 512-row view); 1 = whole
 *                           rows always; 2 = two tile columns wherever they
 *                           fit; 3 = transposed tiles on a row shard's view
 *                           whose row count is a multiple of 256 (e and the
 *                           owned rows multiples of 4): a tile is a strip of
 *                           grid columns spanning the whole view, so only its
 *                           two side columns cross CUs (HBM keeps the row-major
 *                           layout; the launch reads and writes it
 *                           transposed).  Values and actions are bit-identical
 *                           either way, beliefs equal to rounding. */
#define PP2_TUNE_RESIDENT_TILE_COLS 12
/*  PP2_TUNE_SHARD_LAG       row shards' resident launches: 0 (default) = a
 *                           normalisation block start inside a launch scales
 *                           the view by the power of two chosen from the
 *                           previous step's mass, after every tile of the view
 *                           has arrived; 1 = from its mass one block earlier
 *                           (staged in LDS ahead of time: no grid-wide wait,
 *                           no barrier).  Measured on the 2-D tiles of the
 *                           config-4 rank share the waited block start costs
 *                           nothing visible and the lagged one's extra state
 *                           ~0.2 us per step, so it is off by default; on
 *                           transposed tiles it is the faster one.  Beliefs
 *                           equal each other to rounding (power-of-two scales
 *                           are exact); values and actions are bit-identical. */
#define PP2_TUNE_SHARD_LAG 13
/*  Diagnostics (tests):
 *  PP2_TUNE_RESIDENT_CUS    plan resident launches for at most this many CUs
 *                           (0: all); a grid whose tiles do not fit falls
 *                           back before launching
 *  PP2_TUNE_RESIDENT_STALL  tile index that returns at once (-1: none): the
 *                           other tiles' waits time out, exercising the
 *                           re-run of a failed resident launch */
#define PP2_TUNE_RESIDENT_CUS 10
#define PP2_TUNE_RESIDENT_STALL 11
/*  PP2_TUNE_COMM_TIMING     1 = bracket every RCCL round of the context (halo
 *                           exchanges, record groups, all-reduces) with timing
 *                           events on the stream it runs on; read with
 *                           pp2_comm_rounds.  0 (default) = no events. */
#define PP2_TUNE_COMM_TIMING 14
int pp2_set_tuning(pp2_ctx* ctx, int key, int value);
/* Measurement, no reference counterpart (the reference is single-GPU): the
 * RCCL rounds timed since PP2_TUNE_COMM_TIMING was set or the last call --
 * `rounds` timed rounds (at most 256 between calls; later ones are counted in
 * `untimed`, which may be NULL), the first max_rounds of their durations in
 * microseconds (begin event to end event on the issuing stream: the group's
 * own time plus any wait for the peers).  Synchronises; clears the record. */
int pp2_comm_rounds(pp2_ctx* ctx, int* rounds, long long* untimed, float* round_us,
                    int max_rounds);

/* ---------------------------------------------------------------- model
 * generateModelData (src/pomdp/model_generation_cuda.cu:349-368) and the MDP
 * cudaGenerateModelData launch (src/mdp/path_planning_2d.cu:93-106): builds
 * T, L, R (POMDP stage reward) and C (MDP stage cost) on the device. */
int pp2_model_generate(pp2_ctx* ctx);
/* Download in the reference layouts (any pointer may be NULL); replaces the
 * D2H copies into host_trans_prob/host_meas_prob/host_stage_reward
 * (model_generation_cuda.cu:370-375). */
int pp2_model_download(pp2_ctx* ctx, float* T, float* L, float* R, float* C);
/* Upload reference-layout tensors (any may be NULL = keep); the device half
 * of loadModelDataFromFile (model_generation_cuda.cu:150-156). */
int pp2_model_upload(pp2_ctx* ctx, const float* T, const float* L,
                     const float* R, const float* C);
/* Text formats of saveModelDataToFile / loadModelDataFromFile
 * (model_generation_cuda.cu:74-159): files model_data_trans_prob,
 * model_data_meas_prob, model_data_stage_reward in `dir` ("%15.8f"). */
int pp2_model_save(pp2_ctx* ctx, const char* dir);
int pp2_model_load(pp2_ctx* ctx, const char* dir);
/* Dictionary-coded model (no reference counterpart; a lossless re-encoding of
 * the arrays above).  Every call that sets the model (generate / upload /
 * load) rebuilds it: one uint16 code per cell plus one dictionary row per
 * distinct per-cell (T, C, L) tuple, checked bitwise against every cell.
 * entries = dictionary rows (0: more than the LDS budget allows, dense path
 * only); active = 1 when pp2_loop_step / pp2_mdp_sweep use it.  Results are
 * bit-identical either way. */
int pp2_model_dict_info(pp2_ctx* ctx, int* entries, int* active);

/* Loop steps pp2_loop_run fuses into one kernel launch on this context: 2048
 * for the tile-resident loop (PP2_TUNE_RESIDENT) on an unsharded grid, the
 * resident halo depth e on a row shard (PP2_TUNE_RESIDENT_HALO), 2 when it
 * runs the steps of a normalisation / halo block in pairs
 * (PP2_TUNE_STEP_PAIRS with a sparse coded model whose grid has a 4096-cell
 * tile per CU; unsharded, RCCL row shard or shard-group member), else 1.
 * A query: allocates nothing. */
int pp2_loop_steps_per_launch(pp2_ctx* ctx, int* steps);
/* The tiling of the tile-resident loop this context would launch (its grid,
 * or a row shard's view): tiles (one per CU), rows per tile and tile columns
 * (1: whole rows; 2: 2-D tiles, PP2_TUNE_RESIDENT_TILE_COLS; 3: transposed
 * tiles of a shard view, rows per tile = grid columns per tile); all 0 when the
 * loop does not run resident.  A query: allocates nothing. */
int pp2_resident_tiling(pp2_ctx* ctx, int* tiles, int* rows_per_tile, int* tile_cols);
/* Diagnostics: resident launches so far on this context -- tile-resident loop
 * launches (pp2_loop_run) and resident MDP-solve launches (pp2_mdp_solve);
 * either pointer may be NULL.  No reference counterpart. */
int pp2_resident_launches(pp2_ctx* ctx, int* loop_launches, int* solve_launches);
/* Resident launches re-run on per-step launches after a timeout, and whether
 * the resident kernels are still enabled on the context (either may be NULL). */
int pp2_resident_status(pp2_ctx* ctx, int* fallbacks, int* enabled);

/* ---------------------------------------------------------------- belief
 * The belief lives on the device with deferred normalisation: each update
 * applies the previous step's 1/sum and records its own sum on the device,
 * so no host round trip is needed per step.
 *
 * pp2_belief_set: root belief from a Belief message (msg->belief,
 * src/pomdp/path_planning_2d.cu:208), used as given. */
int pp2_belief_set(pp2_ctx* ctx, const float* belief);
/* Normalised belief b/sum (host renormalisation of search_tree_cuda.cu:
 * 608-612). */
int pp2_belief_get(pp2_ctx* ctx, float* belief);
/* cudaBayesBeliefUpdate (point_based_value_iteration_cuda.cu:88-133) +
 * renormalisation (search_tree_cuda.cu:601-612).  Asynchronous. */
int pp2_belief_update(pp2_ctx* ctx, uint8_t u, uint8_t z);
/* The stored (unnormalised) belief and its mass: belief_get == raw / mass.
 * Exposes the kernel output itself, for bit-exact parity checks. */
int pp2_belief_get_raw(pp2_ctx* ctx, float* belief, float* mass);
/* Unnormalised mass of the current belief (= p(z | b, u) after an update
 * from a normalised belief). Synchronises. */
int pp2_belief_mass(pp2_ctx* ctx, float* mass);

/* ---------------------------------------------------------------- MDP
 * J := 0, A := 0 (cudaMemset, src/mdp/path_planning_2d_cuda.cu:55-61). */
int pp2_mdp_reset(pp2_ctx* ctx);
/* n Bellman sweeps, cudaOneStepValueIteration
 * (src/mdp/path_planning_2d_cuda.cu:215-264). Asynchronous. */
int pp2_mdp_sweep(pp2_ctx* ctx, int n);
/* MdpPathPlanning2d::valueIteration (src/mdp/path_planning_2d.cu:207-269)
 * without the OpenCV windows: blocks of 100 sweeps until the inf-norm of the
 * change over a block is <= 1e-3*5/(1-gamma).  max_sweeps <= 0: no cap. */
int pp2_mdp_solve(pp2_ctx* ctx, int max_sweeps, int* sweeps,
                  double* final_norm);
/* D2H of dev_optimal_cost1 / dev_optimal_action
 * (src/mdp/path_planning_2d.cu:119-126).  Either may be NULL. */
int pp2_mdp_get(pp2_ctx* ctx, float* J, uint8_t* A);

/* ---------------------------------------------------------------- north star
 * One iteration of the benchmarked loop: one belief update (u, z) and one
 * Bellman sweep in one launch.  The stored belief is renormalised by its
 * exact mass every PP2_TUNE_NORM_BLOCK steps (power-of-two scaled in
 * between); reads always divide by the true mass.  Sharded contexts also
 * exchange halo rows and all-reduce the belief mass at each block start.
 * Asynchronous. */
int pp2_loop_step(pp2_ctx* ctx, uint8_t u, uint8_t z);
int pp2_loop_run(pp2_ctx* ctx, int n, const uint8_t* us, const uint8_t* zs);

/* ---------------------------------------------------------------- FIB
 * cudaFIBValueIteration sweeps (fast_informed_bound_cuda.cu:97-204) from the
 * current alphas (zero after create). Asynchronous. */
int pp2_fib_reset(pp2_ctx* ctx);
int pp2_fib_sweep(pp2_ctx* ctx, int n);
/* fastInformedBound driver (fast_informed_bound_cuda.cu:206-276): blocks of
 * 10 sweeps until the inf-norm of the change <= 0.01. */
int pp2_fib_solve(pp2_ctx* ctx, int max_sweeps, int* sweeps, float* final_norm);
/* host_fib_alphas layout [hw][9] (fast_informed_bound_cuda.cu:270-271). */
int pp2_fib_get(pp2_ctx* ctx, float* alphas);
int pp2_fib_set(pp2_ctx* ctx, const float* alphas);
/* saveFibDataToFile / loadFibDataFromFile (fast_informed_bound_cuda.cu:
 * 343-394): dir/fib_alphas (one cell per line, 9 "%15.8f" values) and
 * dir/fib_actions (the 9 actions, "%10u" per line).  dir NULL: ".". */
int pp2_fib_save(pp2_ctx* ctx, const char* dir);
int pp2_fib_load(pp2_ctx* ctx, const char* dir);

/* ---------------------------------------------------------------- PBVI
 * Point-based value iteration lower bound (src/pomdp/
 * point_based_value_iteration_cuda.cu), state kept in the context (unsharded
 * contexts only): the belief set B[S][hw], alpha vectors alphas[S][hw] and
 * their actions[S] (host_pbvi_alphas / host_pbvi_actions, :51-57).  The
 * reference's node uses S = 500 (src/pomdp/path_planning_2d.cu:122,140).
 *
 * generateBeliefSet (:165-295): S beliefs (1..4096) grown from b0 (hw
 * floats, used as given).  Three glibc rand() draws per (belief, action) and round from
 * srand(rand_seed) (the reference never seeds: 1); *rand_calls (may be NULL)
 * gets the number drawn, so a planner can continue the same stream.  Resets
 * the alphas to 0 (pointBasedValueIteration, :652-657). */
int pp2_pbvi_belief_set(pp2_ctx* ctx, const float* b0, uint32_t set_size,
                        uint32_t rand_seed, uint64_t* rand_calls);
/* Any S beliefs [S][hw] as the belief set (alphas reset to 0). */
int pp2_pbvi_set_beliefs(pp2_ctx* ctx, uint32_t set_size, const float* beliefs);
int pp2_pbvi_get_beliefs(pp2_ctx* ctx, float* beliefs);
/* backupAlphaVectors (:319-641): `iterations` synchronous point-based
 * backups from the current alphas; iterations <= 0 runs the reference's
 * ceil(log(1e-3/5) / log(gamma)) (:440-441).  Asynchronous. */
int pp2_pbvi_backup(pp2_ctx* ctx, int iterations);
/* pointBasedValueIteration (:643-676): belief set + zero alphas + backup. */
int pp2_pbvi_solve(pp2_ctx* ctx, const float* b0, uint32_t set_size,
                   uint32_t rand_seed, uint64_t* rand_calls);
/* S (0 before any PBVI call) and whether a belief set is present. */
int pp2_pbvi_info(pp2_ctx* ctx, uint32_t* set_size, int* has_beliefs);
/* alphas [S][hw] and actions [S]; either may be NULL. */
int pp2_pbvi_get(pp2_ctx* ctx, float* alphas, uint8_t* actions);
int pp2_pbvi_set(pp2_ctx* ctx, uint32_t set_size, const float* alphas,
                 const uint8_t* actions);
/* evaluatePbviCpu (:678-699) for n beliefs [n][hw]: values[i] = max over k
 * of inner_product(b_i, alpha_k) (x-ordered, multiply then add), actions[i]
 * = the action of the first maximising alpha.  Either output may be NULL. */
int pp2_pbvi_evaluate(pp2_ctx* ctx, int n, const float* beliefs, float* values,
                      uint8_t* actions);
/* savePbviDataToFile / loadPbviDataFromFile (:737-797): dir/pbvi_alphas (one
 * alpha vector per line, "%15.8f" per cell) and dir/pbvi_actions ("%10u" per
 * line; read back into uint8 storage, which the reference overflows). */
int pp2_pbvi_save(pp2_ctx* ctx, const char* dir);
int pp2_pbvi_load(pp2_ctx* ctx, const char* dir, uint32_t set_size);

/* ---------------------------------------------------------------- QV-tree
 * Online POMDP planner: QNode / VNode / SearchTree
 * (include/path_planning_2d/search_tree.h:31-165, src/pomdp/
 * search_tree_cuda.cu:161-626) driven like PomdpPathPlanning2d::beliefCallback
 * (src/pomdp/path_planning_2d.cu:199-241).  Tree logic runs on the host
 * exactly as the reference; every belief update, renormalisation and leaf
 * bound of one VNode::expand (9 actions x all observations) is one batched
 * device pass over the context's model (T, L, R) and FIB alphas (set them
 * with pp2_fib_solve / pp2_fib_set first).  Beliefs of expanded nodes stay
 * on the device; leaf children are scored without being materialised.
 *
 * Sampling follows the reference bit for bit in algorithm: 50 state samples
 * per QNode from glibc rand() over the fp32 prefix sum of the belief
 * (search_tree_cuda.cu:326-337), next state and observation from the cuRAND
 * XORWOW stream curand_init(1234, idx, 0) that every QNode re-creates
 * (:84-147, :318-323). */
typedef struct pp2_planner pp2_planner;

typedef struct {
  int32_t max_search_tree_depth;  /* launch default 50 */
  int32_t max_online_iteration;   /* launch default 15 */
  int32_t lower_bound_mode;       /* 0: constant -5/(1-gamma), the reference's
                                     commented fallback (search_tree_cuda.cu:382-383);
                                     1: PBVI, evaluatePbviCpu (:379) over the
                                     context's alpha vectors (pp2_pbvi_*) */
  uint32_t rand_seed;             /* glibc srand seed; reference never seeds: 1 */
  uint32_t sample_num;            /* observation samples per QNode (:176): 50 */
  uint64_t curand_seed;           /* curand_init seed (:90): 1234 */
  uint64_t rand_skip;             /* rand() draws already taken from the stream
                                     (the reference's generateBeliefSet runs
                                     first: pp2_pbvi_solve's *rand_calls) */
  int32_t reference_order;        /* 1 (default, the drop-in): every sum the
                                     reference runs on its host -- the QNode
                                     reward inner_product and the child
                                     renormalisation accumulate
                                     (search_tree_cuda.cu:168-173, :225-229),
                                     evaluateFibCpu / evaluatePbviCpu
                                     (fast_informed_bound_cuda.cu:278-297,
                                     point_based_value_iteration_cuda.cu:
                                     678-699) and the sampling cdf (:176-183)
                                     -- gives the result of the reference's
                                     x-ordered fp32 chain (multiply, then add;
                                     IEEE division), so bounds, rewards,
                                     weights and the tree equal the
                                     reference's arithmetic bit for bit.
                                     0 (opt-in fast variant, NOT bit-exact):
                                     grid-wide sums as parallel trees (fp64
                                     where the reference's fp32 chains lose
                                     digits); within rel 1e-4 of the
                                     reference, which can flip a near-tied
                                     expansion choice. */
} pp2_planner_params;

/* Snapshot of the root and its children, for inspection and parity tests. */
typedef struct {
  uint32_t depth;
  float root_upper_bound, root_lower_bound, root_heuristic;
  uint32_t n_root_children;  /* 0 (unexpanded) or 9 */
  float q_upper_bound[9], q_lower_bound[9], q_reward[9], q_heuristic[9];
  uint32_t q_depth[9], q_nchildren[9];
  uint8_t q_obs[9][16];
  float q_weight[9][16], v_upper_bound[9][16], v_lower_bound[9][16];
  uint32_t total_vnodes, total_qnodes, expansions;
} pp2_tree_info;

int pp2_planner_default_params(pp2_planner_params* p);
/* PomdpPathPlanning2d::initialize tail (src/pomdp/path_planning_2d.cu:145-155):
 * binds the planner to a context whose model and FIB alphas are ready. */
int pp2_planner_create(pp2_planner** out, pp2_ctx* ctx,
                       const pp2_planner_params* params);
int pp2_planner_destroy(pp2_planner* p);
/* One plan step = beliefCallback (:199-241): first call (or after reset)
 * builds the tree from `belief` (hw floats, used as given); later calls
 * re-root with (action, observation).  Expands while depth < max depth and
 * fewer than max_online_iteration expansions, then returns the action with
 * the largest Q upper bound. */
int pp2_planner_step(pp2_planner* p, uint8_t action, uint8_t observation,
                     const float* belief, uint8_t* new_action,
                     float* new_value);
/* resetSearchTreeCallback (:275-282). */
int pp2_planner_reset(pp2_planner* p);
int pp2_planner_info(pp2_planner* p, pp2_tree_info* info);
/* The 2*n curand_uniform draws the reference's cudaForwardSampling sees:
 * u1[i], u2[i] = first and second draw of curand_init(seed, i, 0). */
int pp2_curand_uniforms(uint64_t seed, int n, float* u1, float* u2);

/* ---------------------------------------------------------------- rollouts
 * Batched QV-tree rollouts (BASELINE configs[4]: 4096 copies x depth 5 at
 * 512x512): C copies of a root belief each follow their own (u_k, z_k),
 * k < depth.  Per copy and step: reward r_k = <b_k, R[:,u_k]> (QNode reward,
 * search_tree_cuda.cu:168-173), observation likelihood p_k = sum of the
 * unnormalised update, b_{k+1} = normalise(L_zk . T_uk^T b_k) (the
 * reference update + renormalisation); leaf: FIB bound max_i <b_depth,
 * alpha_i> (evaluateFibCpu); value = sum_k gamma^k r_k + gamma^depth * leaf.
 * Beliefs are stored as per-copy max-normalised fp16 (2 B per cell-copy),
 * arithmetic is fp32; expect ~1e-3 relative agreement with an fp32 rollout. */
typedef struct pp2_rollout pp2_rollout;
/* copies 1..131072, depth >= 1 */
int pp2_rollout_create(pp2_rollout** out, pp2_ctx* ctx, int copies, int depth);
int pp2_rollout_destroy(pp2_rollout* r);
/* root belief (hw floats): every copy starts from it (one fp16 image that
 * the first step of every run reads for all copies) */
int pp2_rollout_set_root(pp2_rollout* r, const float* belief);
/* us, zs: [depth][copies]; every run starts from the root.  Asynchronous. */
int pp2_rollout_run(pp2_rollout* r, const uint8_t* us, const uint8_t* zs);
/* rewards, obs_prob: [depth][copies]; leaf_upper, value: [copies]; any may be
 * NULL.  Synchronises. */
int pp2_rollout_results(pp2_rollout* r, float* rewards, float* obs_prob,
                        float* leaf_upper, float* value);
/* normalised fp32 belief of one copy after the run, or the root before any
 * run (hw floats) */
int pp2_rollout_get_belief(pp2_rollout* r, int copy, float* belief);

/* ---------------------------------------------------------------- shards
 * Two transports for row shards (no reference counterpart):
 *  - one process per GPU: RCCL (pp2_rccl_unique_id / pp2_shard_comm_init);
 *    then every per-context call exchanges its halos itself;
 *  - one process driving several shard contexts (one or more devices): a
 *    shard group, whose pp2_shard_group_* calls run each step phase-wise
 *    over all shards, moving halo rows and the belief mass with device
 *    copies.  Grouped contexts reject the per-context stepping calls. */
typedef struct pp2_shard_group pp2_shard_group;
/* ctxs[i] must be the shards of one grid in row order (pp2_create_shard). */
int pp2_shard_group_create(pp2_shard_group** out, pp2_ctx* const* ctxs, int n);
int pp2_shard_group_destroy(pp2_shard_group* g);
int pp2_shard_group_loop_step(pp2_shard_group* g, uint8_t u, uint8_t z);
/* n loop steps (pp2_loop_run's contract): pairs of steps of a halo block per
 * launch on every shard where PP2_TUNE_STEP_PAIRS applies, else single steps. */
int pp2_shard_group_loop_run(pp2_shard_group* g, int n, const uint8_t* us, const uint8_t* zs);
int pp2_shard_group_belief_update(pp2_shard_group* g, uint8_t u, uint8_t z);
int pp2_shard_group_mdp_sweep(pp2_shard_group* g, int n);
int pp2_shard_group_mdp_solve(pp2_shard_group* g, int max_sweeps, int* sweeps,
                              double* final_norm);
int pp2_shard_group_fib_sweep(pp2_shard_group* g, int n);
int pp2_shard_group_synchronize(pp2_shard_group* g);

/* RCCL bootstrap for row shards (no reference counterpart).  Rank 0 calls
 * pp2_rccl_unique_id, the 128 bytes are broadcast out of band, then every
 * rank calls pp2_shard_comm_init with its own shard context. */
#define PP2_RCCL_ID_BYTES 128
int pp2_rccl_unique_id(uint8_t id[PP2_RCCL_ID_BYTES]);
int pp2_shard_comm_init(pp2_ctx* ctx, const uint8_t id[PP2_RCCL_ID_BYTES],
                        int nranks, int rank);

#ifdef __cplusplus
}
#endif
#endif /* PP2_H */
