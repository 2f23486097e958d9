"""A/B timing of loop-kernel tuning variants, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24): N rounds x variants, median/min."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = int(os.environ.get("PP2_N", "1024"))
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 64, seed=42)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = P.GridContext(grid, goal)
    ctx.set_stream(stream.cuda_stream)
    ctx.model_generate()
    ctx.belief_set(S.uniform_belief(grid))
    ctx.mdp_reset()
    variants = {"base": [], "nt": []}
    steps = 100
    for rnd in range(12):
        for name in variants:
            ctx.set_tuning(P.GridContext.TUNE_NT_STREAMS, 1 if name == "nt" else 0)
            ctx.loop_run(us[:8], zs[:8])
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for k in range(steps // 64 + 1):
                ctx.loop_run(us, zs)
            e1.record(stream)
            torch.cuda.synchronize()
            n = (steps // 64 + 1) * 64
            variants[name].append(e0.elapsed_time(e1) * 1e3 / n)
    for name, v in variants.items():
        v = np.array(v[2:])
        print(f"{name:6s} median {np.median(v):7.2f} us  min {v.min():7.2f} us  "
              f"-> {417 * N * N / (np.median(v) * 1e-6) / 1e12:.3f} TB/s algorithmic")


if __name__ == "__main__":
    main()
