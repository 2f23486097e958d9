"""Minimal driver for counter collection on the coded / dense MDP sweep and
loop kernels (rocprofv3 --pmc ... -- python3 tools/coded_sweep_driver.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = int(os.environ.get("PP2_N", "1024"))
    reps = int(os.environ.get("PP2_REPS", "20"))
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, reps, seed=42)
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.model_generate()
        if os.environ.get("PP2_DENSE"):
            ctx.set_tuning(ctx.TUNE_CODED_MODEL, 0)
        print("dict", ctx.model_dict_info(), flush=True)
        ctx.belief_set(S.uniform_belief(grid))
        ctx.mdp_reset()
        ctx.mdp_sweep(reps)
        ctx.loop_run(us, zs)
        ctx.synchronize()
        print("mass", float(ctx.belief_get().astype(np.float64).sum()))


if __name__ == "__main__":
    main()
