"""The bench's PBVI-leaf plan step alone (256^2 synthetic, S = 500 alphas,
depth 3, reference order): p50 over closed-loop plan steps, for same-box A/B
of library builds (PP2_LIBRARY).  The alphas come from a short PBVI solve
(PP2_ITERS backups) -- their values do not change the work."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import bench
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 256
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    ctx = P.GridContext(grid, goal, gamma=0.95, device=0)
    ctx.model_generate()
    ctx.fib_solve()
    b0 = S.uniform_belief(grid)
    ctx.pbvi_belief_set(b0, 500)
    ctx.pbvi_backup(int(os.environ.get("PP2_ITERS", "3")))
    with P.QVTreePlanner(ctx, max_search_tree_depth=3, max_online_iteration=15,
                         lower_bound_mode=1) as pl:
        bench.closed_loop(grid, b0, pl.step, 3, 1e9)
        pl.reset()
        ms = bench.closed_loop(grid, b0, pl.step, int(os.environ.get("PP2_STEPS", "40")), 1e9)
    ctx.close()
    print(f"{os.environ.get('PP2_LIBRARY', 'in-tree')}: PBVI-leaf plan step p50 "
          f"{np.percentile(ms, 50):.3f} ms, mean {ms.mean():.3f} ms", flush=True)


if __name__ == "__main__":
    main()
