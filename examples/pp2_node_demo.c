/*
 * pp2_node_demo.c -- the POMDP node's call sequence through the C ABI alone
 * (include/pp2.h), as a catkin node would make it:
 * create a context from an occupancy grid, generate the model, solve FIB and
 * PBVI, create the planner with PBVI leaf bounds, answer a few belief
 * messages, run the benchmarked belief-update + Bellman loop, and save the
 * reference text formats.  Plain C99, linked against libpp2_hip.so.
 *
 *   ./pp2_node_demo [out_dir]      exit status 0 on success
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "pp2.h"

#define CHECK(call)                                                                \
  do {                                                                             \
    int s_ = (call);                                                               \
    if (s_ != PP2_OK) {                                                            \
      fprintf(stderr, "%s: %s: %s\n", #call, pp2_status_string(s_), pp2_last_error()); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t H = 40, W = 60;
  uint8_t* map = (uint8_t*)calloc(H * W, 1);
  float* belief = (float*)malloc(sizeof(float) * H * W);
  float* J = (float*)malloc(sizeof(float) * H * W);
  uint8_t* A = (uint8_t*)malloc(H * W);
  if (!map || !belief || !J || !A) return 1;
  /* a walled room with two pillars; the goal near the far corner */
  for (uint32_t y = 0; y < H; ++y)
    for (uint32_t x = 0; x < W; ++x)
      map[y * W + x] = (x == 0 || y == 0 || x == W - 1 || y == H - 1 ||
                        (x >= 20 && x < 23 && y >= 10 && y < 30) ||
                        (x >= 40 && x < 43 && y >= 5 && y < 25));
  /* uniform initial belief over the free cells (src/pomdp/path_planning_2d.cu:99-107) */
  float free_cells = 0.0f;
  for (uint32_t i = 0; i < H * W; ++i) free_cells += 1.0f - map[i];
  for (uint32_t i = 0; i < H * W; ++i) belief[i] = (1.0f - map[i]) / free_cells;

  int ndev = 0;
  CHECK(pp2_device_count(&ndev));
  if (ndev < 1) {
    fprintf(stderr, "no GPU\n");
    return 2;
  }
  pp2_ctx* ctx = NULL;
  CHECK(pp2_create(&ctx, 0, H, W, map, 55, 35, 0.95f));
  CHECK(pp2_model_generate(ctx));
  int sweeps = 0;
  float fnorm = 0.0f;
  CHECK(pp2_fib_solve(ctx, 0, &sweeps, &fnorm));
  uint64_t draws = 0;
  CHECK(pp2_pbvi_solve(ctx, belief, 64, 1, &draws));
  float v0 = 0.0f;
  uint8_t a0 = 0;
  CHECK(pp2_pbvi_evaluate(ctx, 1, belief, &v0, &a0));

  pp2_planner_params prm;
  CHECK(pp2_planner_default_params(&prm));
  prm.max_search_tree_depth = 5;
  prm.lower_bound_mode = 1;
  prm.rand_skip = draws;
  pp2_planner* pl = NULL;
  CHECK(pp2_planner_create(&pl, ctx, &prm));
  uint8_t act = 0, obs = 0;
  float value = 0.0f;
  for (int k = 0; k < 4; ++k) {
    CHECK(pp2_planner_step(pl, act, obs, belief, &act, &value));
    if (act > 8) return 3;
    obs = (uint8_t)((k * 5) & 15);
  }
  pp2_tree_info info;
  CHECK(pp2_planner_info(pl, &info));

  /* the north-star loop: belief update + Bellman sweep per step */
  CHECK(pp2_belief_set(ctx, belief));
  CHECK(pp2_mdp_reset(ctx));
  uint8_t us[16], zs[16];
  for (int k = 0; k < 16; ++k) {
    us[k] = (uint8_t)(k % 9);
    zs[k] = (uint8_t)((3 * k) % 16);
  }
  CHECK(pp2_loop_run(ctx, 16, us, zs));
  CHECK(pp2_belief_get(ctx, belief));
  CHECK(pp2_mdp_get(ctx, J, A));
  double mass = 0.0;
  for (uint32_t i = 0; i < H * W; ++i) mass += belief[i];
  if (mass < 0.999 || mass > 1.001) {
    fprintf(stderr, "belief mass %f\n", mass);
    return 4;
  }
  if (argc > 1) {
    CHECK(pp2_model_save(ctx, argv[1]));
    CHECK(pp2_fib_save(ctx, argv[1]));
    CHECK(pp2_pbvi_save(ctx, argv[1]));
  }
  printf("pp2_node_demo ok: abi %d, FIB %d sweeps, PBVI S=64 (%llu rand draws) V(b0)=%.4f a=%u, "
         "plan action %u value %.4f depth %u, 16 loop steps, mass %.6f\n",
         pp2_abi_version(), sweeps, (unsigned long long)draws, v0, a0, act, value, info.depth,
         mass);
  CHECK(pp2_planner_destroy(pl));
  CHECK(pp2_destroy(ctx));
  free(map);
  free(belief);
  free(J);
  free(A);
  return 0;
}
