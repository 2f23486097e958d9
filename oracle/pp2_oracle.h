/*
 * pp2_oracle.h -- CPU restatement of path_planning_2d's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (path_planning_2d_amd/)
 * links, imports or calls this code; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg use it, as the checker / the timed CPU
 * baseline.
 *
 * Parity status: UNPINNED by the reference's own tests -- the reference
 * ships no tests, fixtures or golden vectors, and it cannot be
 * built here (nvcc, ROS, OpenCV, Boost, Eigen are absent).
 * The restatement follows the reference line by line (citations below, all
 * relative to /root/reference/path_planning_2d/), is cross-checked against an
 * independent numpy restatement of the simulator's scatter-form CPU filter
 * (dummy_simulator/src/dummy_simulator.cpp:440-773), and is frozen into
 * tests/golden/ fixtures.
 *
 * Layouts are the reference's: T[hw][9 u][9 s'], L[hw][16 z], R/C[hw][9 u],
 * cell idx = y*W + x.
 *
 * Arithmetic: the reference device code is built with nvcc --use_fast_math
 * (CMakeLists.txt:36), i.e. FTZ and a*b+c contracted to fma.  The device-side
 * functions here spell every contraction out with fmaf() and (optionally)
 * flush denormals; host-side functions (normalisation, leaf evaluation) use
 * plain separate multiply/add like the reference's x86 host code.  Build with
 * -ffp-contract=off so the compiler adds no contraction of its own.
 */
#ifndef PP2_ORACLE_H
#define PP2_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- model generation (a1) ------------------------------------------------ */
/* POMDP cudaGenerateModelData: src/pomdp/model_generation_cuda.cu:161-347 */
void orc_model_pomdp(int H, int W, const uint8_t* map, int gx, int gy,
                     float* T, float* L, float* R);
/* MDP cudaGenerateModelData: src/mdp/path_planning_2d_cuda.cu:76-213 */
void orc_model_mdp(int H, int W, const uint8_t* map, int gx, int gy,
                   float* T, float* C);
/* Model of one cell (same code path), for trajectory sampling. */
void orc_cell_model(int H, int W, const uint8_t* map, int x, int y, int gx,
                    int gy, float* T81, float* L16, float* R9, float* C9);

/* ---- belief update (a2) + renormalisation (a3) ----------------------------- */
/* cudaBayesBeliefUpdate: src/pomdp/point_based_value_iteration_cuda.cu:88-133
 * (gather form, output unnormalised). ftz!=0 flushes denormals like FTZ. */
void orc_belief_update(int H, int W, const float* T, const float* L,
                       const float* b_in, int u, int z, float* b_out, int ftz);
/* Row range [y0,y1) only (for threaded CPU baseline). */
void orc_belief_update_rows(int H, int W, const float* T, const float* L,
                            const float* b_in, int u, int z, float* b_out,
                            int ftz, int y0, int y1);
/* Host renormalisation, search_tree_cuda.cu:225-229 / :608-612:
 * sum = std::accumulate(b, 0.0f) (sequential fp32), then x /= sum. */
float orc_normalize_seq(size_t n, float* b);
/* Same with an fp64 sum (the accuracy reference at large grids). */
double orc_normalize_f64(size_t n, float* b);
double orc_sum_f64(size_t n, const float* b);
float orc_sum_seq(size_t n, const float* b);

/* ---- MDP Bellman backup (a4) ---------------------------------------------- */
/* cudaOneStepValueIteration: src/mdp/path_planning_2d_cuda.cu:215-264 */
void orc_mdp_sweep(int H, int W, float gamma, const float* T, const float* C,
                   const float* J_in, float* J_out, uint8_t* A);
/* CPU baseline: nsteps loop steps, rows split over nthreads pthreads. */
int orc_loop_run_mt(int H, int W, float gamma, const float* T, const float* L, const float* C,
                    float* b, float* bo, float* J, float* Jo, uint8_t* A, int nsteps,
                    const uint8_t* us, const uint8_t* zs, int nthreads);
void orc_mdp_sweep_rows(int H, int W, float gamma, const float* T,
                        const float* C, const float* J_in, float* J_out,
                        uint8_t* A, int y0, int y1);
/* MdpPathPlanning2d::valueIteration driver, src/mdp/path_planning_2d.cu:207-269:
 * blocks of 100 sweeps (50 ping-pong pairs), stop when the inf-norm of the
 * change over the block <= 1e-3*5/(1-gamma).  J, A are outputs (J starts at 0).
 * Returns the number of sweeps; *final_norm gets the last inf-norm.
 * max_sweeps<=0 means unlimited. */
int orc_mdp_solve(int H, int W, float gamma, const float* T, const float* C,
                  float* J, uint8_t* A, int max_sweeps, double* final_norm);

/* ---- FIB Bellman backup (a5) ----------------------------------------------- */
/* cudaFIBValueIteration: src/pomdp/fast_informed_bound_cuda.cu:97-204
 * alphas are [hw][9]. */
void orc_fib_sweep(int H, int W, float gamma, const float* T, const float* L,
                   const float* R, const float* a_in, float* a_out);
/* fastInformedBound driver :206-276 -- blocks of 10 sweeps, stop when the
 * inf-norm of the change over the block <= 0.01f. Returns sweeps. */
int orc_fib_solve(int H, int W, float gamma, const float* T, const float* L,
                  const float* R, float* alphas, int max_sweeps,
                  float* final_norm);

/* ---- leaf bounds / rewards (a7) --------------------------------------------- */
/* evaluateFibCpu: fast_informed_bound_cuda.cu:278-297 (alphas [hw][9]) */
void orc_fib_eval(size_t n, const float* b, const float* alphas, float* value,
                  uint8_t* action);
/* evaluatePbviCpu: point_based_value_iteration_cuda.cu:678-699 (alphas [S][hw]) */
void orc_pbvi_eval(size_t n, const float* b, int S, const float* alphas,
                   const uint8_t* actions, float* value, uint8_t* action);
/* QNode reward, search_tree_cuda.cu:168-173: inner_product(b, R[:,a], 0.0f) */
float orc_reward_dot(size_t n, const float* b, const float* R, int a);

/* ---- simulator scatter filter (independent cross-check) --------------------- */
/* DummySimulator::updateBelief(u), dummy_simulator.cpp:671-718 (+ normalise) */
void orc_sim_predict(int H, int W, const uint8_t* map, const float* b, int u,
                     float* out);
/* DummySimulator::updateBelief(meas), dummy_simulator.cpp:720-773 */
void orc_sim_correct(int H, int W, const uint8_t* map, const float* b, int z,
                     float* out);

/* ---- random number restatements (a8) ---------------------------------------- */
/* glibc rand() (TYPE_3 additive feedback, srand(seed)); reference never seeds,
 * so its sequence is seed 1. State is caller-owned (34 words + 2 indices). */
typedef struct { int32_t r[34]; int f, b; } orc_rand_state;
void orc_rand_seed(orc_rand_state* s, uint32_t seed);
int32_t orc_rand_next(orc_rand_state* s);
/* cuRAND XORWOW (CUDA 8 curand_kernel.h): curand_init(seed, subseq, offset)
 * followed by n curand() draws; writes the raw 32-bit outputs. */
void orc_curand_xorwow(uint64_t seed, uint64_t subsequence, uint64_t offset,
                       int n, uint32_t* out);
/* curand_uniform(x) = x * 2^-32 + 2^-33 in fp32 */
float orc_curand_uniform(uint32_t x);

/* ---- synthetic inputs -------------------------------------- */
uint64_t orc_splitmix64_next(uint64_t* s);
void orc_synth_map(int H, int W, uint64_t seed, double p_occ, uint8_t* map);
/* first free cell scanning left from (W-6, H-6), then upward */
int orc_synth_goal(int H, int W, const uint8_t* map, int* gx, int* gy);
/* seeded (u, z) trajectory of n steps (see DESIGN.md "Synthetic inputs") */
int orc_synth_trajectory(int H, int W, const uint8_t* map, int gx, int gy,
                         uint64_t seed, int n, uint8_t* us, uint8_t* zs,
                         int32_t* states);

/* ---- PBVI lower bound, pp2_oracle_pbvi.c -------------------------------------- */
/* generateBeliefSet (point_based_value_iteration_cuda.cu:165-295): b_set[S][hw]
 * from b0, drawing rand() from *rs (seed it with orc_rand_seed(rs, 1) for the
 * reference's unseeded glibc rand()). */
int orc_pbvi_belief_set(int H, int W, const float* T, const float* L, const float* b0,
                        int S, orc_rand_state* rs, float* b_set);
/* backupAlphaVectors (:319-641) from the given alphas[S][hw] (the driver
 * zeroes them, :652-657); iterations <= 0: the reference's count (:440-441).
 * Returns the iterations run. */
int orc_pbvi_backup(int H, int W, float gamma, const float* T, const float* L, const float* R,
                    int S, const float* b_set, float* alphas, uint8_t* actions, int iterations);
int orc_pbvi_iterations(float gamma);
/* indices sorted as the reference's partial_sort (:264-269) leaves them */
void orc_heap_sort_desc(size_t n, const float* key, size_t* idx);

/* ---- QV-tree online planner (a6-a8), pp2_oracle_tree.c ---------------------- */
typedef struct {
  uint32_t depth;
  float root_upper_bound, root_lower_bound, root_heuristic;
  uint32_t n_root_children;
  float q_upper_bound[9], q_lower_bound[9], q_reward[9], q_heuristic[9];
  uint32_t q_depth[9], q_nchildren[9];
  uint8_t q_obs[9][16];
  float q_weight[9][16], v_upper_bound[9][16], v_lower_bound[9][16];
  uint32_t total_vnodes, total_qnodes, expansions;
} orc_tree_info;
typedef struct orc_planner orc_planner;
/* T, L, R, alphas are borrowed (reference layouts; alphas [hw][9]).
 * accurate = 0: the reference's arithmetic (sequential fp32 sums);
 * accurate = 1: fp64 accumulation of normalisation sums, rewards and FIB
 *               dots -- the accuracy reference for the device tree sums. */
orc_planner* orc_planner_create(int H, int W, const float* T, const float* L,
                                const float* R, const float* alphas, float gamma,
                                int max_depth, int max_iter, uint32_t rand_seed,
                                uint32_t sample_num, uint64_t curand_seed,
                                int accurate);
int orc_planner_step(orc_planner* p, uint8_t a, uint8_t z, const float* belief,
                     uint8_t* new_action, float* new_value);
void orc_planner_reset(orc_planner* p);
/* VNode lower bounds from PBVI alphas [S][hw] (evaluatePbviCpu,
 * search_tree_cuda.cu:379) instead of the constant -5/(1-gamma); borrowed. */
void orc_planner_set_pbvi(orc_planner* p, int S, const float* alphas, const uint8_t* actions);
/* discard n rand() draws (the reference's generateBeliefSet runs first) */
void orc_planner_skip_rand(orc_planner* p, uint64_t n);
void orc_planner_info(orc_planner* p, orc_tree_info* info);
void orc_planner_destroy(orc_planner* p);

#ifdef __cplusplus
}
#endif
#endif
