"""Rollout-only driver for rocprofv3 (per-kernel split of a batched rollout).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_roll -- \
        python3 tools/prof_rollout.py --copies 4096 --depth 5 --size 512
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = a.size
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    b0 = S.uniform_belief(grid)
    us, zs = S.rollout_trajectories(grid, b0, a.copies, a.depth, seed=13)
    ctx = P.GridContext(grid, goal, gamma=0.95, device=0)
    ctx.model_generate()
    ctx.fib_solve(max_sweeps=40)
    with P.BatchedRollout(ctx, a.copies, a.depth) as r:
        for i in range(a.reps + 1):
            r.set_root(b0)
            ctx.synchronize()
            t0 = time.perf_counter()
            r.run(us, zs)
            ctx.synchronize()
            dt = time.perf_counter() - t0
            print(f"rep {i}: {dt * 1e3:.3f} ms", flush=True)
        res = r.results()
    print("mean value", float(res["value"].mean()))
    ctx.close()


if __name__ == "__main__":
    main()
