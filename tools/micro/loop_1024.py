"""Per-step time of the unsharded 1024^2 tile-resident loop (one 200-step
pp2_loop_run after warm-up, median of 5) and per sweep of the resident MDP solve -- with PP2_LIBRARY pointing at a
diagnostic build (tools/micro/resident_nowait.sh) it times that build."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = int(os.environ.get("PP2_N", "1024"))
    k = 200
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, k + 16, seed=42)
    ctx = P.GridContext(grid, goal)
    ctx.model_generate()
    ctx.belief_set(S.uniform_belief(grid))
    ctx.mdp_reset()
    ts = []
    for rep in range(5):
        ctx.loop_run(us[:16], zs[:16])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.loop_run(us[16:], zs[16:])
        torch.cuda.synchronize()
        ts.append(1e6 * (time.perf_counter() - t0) / k)
    print(f"{N}^2 unsharded, tiling {ctx.resident_tiling()}: {np.median(ts):.3f} us/step "
          f"({', '.join(f'{t:.3f}' for t in ts)})", flush=True)
    # the MDP solve (resident sweeps) from J = 0, 300 sweeps
    ss = []
    for rep in range(5):
        ctx.mdp_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_sw, _ = ctx.mdp_solve(300)
        torch.cuda.synchronize()
        ss.append(1e6 * (time.perf_counter() - t0) / max(n_sw, 1))
    print(f"{N}^2 MDP solve: {np.median(ss):.3f} us/sweep ({n_sw} sweeps)", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
