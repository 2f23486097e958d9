"""Closed-loop plan steps at 256^2, depth 3 (bench.py's plan_step leg, no CPU
baseline) for rocprofv3 --kernel-trace --stats: kernels per plan step and
their time against the step's wall time."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import bench
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = int(os.environ.get("PP2_N", "256"))
    steps = int(os.environ.get("PP2_STEPS", "200"))
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    ctx = P.GridContext(grid, goal, gamma=0.95, device=0)
    ctx.model_generate()
    ctx.fib_solve()
    b0 = S.uniform_belief(grid)
    ref = int(os.environ.get("PP2_REF", "0"))  # 1: reference_order planner
    with P.QVTreePlanner(ctx, max_search_tree_depth=3, max_online_iteration=15,
                         reference_order=ref) as pl:
        bench.closed_loop(grid, b0, pl.step, 3, 1e9)
        pl.reset()
        t0 = time.perf_counter()
        ms = bench.closed_loop(grid, b0, pl.step, steps, 1e9)
        el = time.perf_counter() - t0
    ctx.close()
    print(f"reference_order={ref}: {steps} plan steps: p50 {np.percentile(ms, 50):.3f} ms, mean {ms.mean():.3f} ms, "
          f"wall {el * 1e3:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
