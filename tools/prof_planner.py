"""Closed-loop plan steps for rocprofv3 --kernel-trace --stats: kernels per
plan step and their time against the step's wall time.
  PP2_CASE=256   256^2 synthetic, depth 3 (bench plan_step; PP2_LB=1: PBVI
                 leaves, S = 500, bench plan_step_pbvi_lb)
  PP2_CASE=node  sparse_map_100x40, goal (95, 34), depth 50, PBVI leaves
                 S = 500 (bench node_plan_step)
PP2_REF: reference_order (default 1, the drop-in's mode); PP2_STEPS steps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    case = os.environ.get("PP2_CASE", "256")
    steps = int(os.environ.get("PP2_STEPS", "100"))
    if case == "node":
        grid = np.load(os.path.join(ROOT, "tests", "golden", "maps", "sparse_map_100x40.npy"),
                       allow_pickle=False)
        goal, depth, lb = (95, 34), 50, 1
    else:
        grid = S.synth_grid(256, 256, seed=256)
        goal, depth, lb = S.synth_goal(grid), 3, int(os.environ.get("PP2_LB", "0"))
    ctx = P.GridContext(grid, goal, gamma=0.95, device=0)
    ctx.model_generate()
    ctx.fib_solve()
    b0 = S.uniform_belief(grid)
    calls = 0
    if lb:
        calls = ctx.pbvi_belief_set(b0, 500)
        ctx.pbvi_backup(int(os.environ.get("PP2_ITERS", "0")))
    ref = int(os.environ.get("PP2_REF", "1"))

    def planner():
        return P.QVTreePlanner(ctx, max_search_tree_depth=depth, max_online_iteration=15,
                               lower_bound_mode=lb, rand_skip=calls, reference_order=ref)
    with planner() as pl:
        S.closed_loop(grid, b0, pl.step, 3)
    with planner() as pl:
        t0 = time.perf_counter()
        ms, _, _ = S.closed_loop(grid, b0, pl.step, steps)
        el = time.perf_counter() - t0
        info = pl.info()
    ctx.close()
    print(f"case {case} lb {lb} reference_order={ref}: {steps} plan steps: p50 "
          f"{np.percentile(ms, 50):.3f} ms, mean {ms.mean():.3f} ms, wall {el * 1e3:.1f} ms, "
          f"expansions {info['expansions']}", flush=True)


if __name__ == "__main__":
    main()
