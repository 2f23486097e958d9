"""Event-timed FIB sweeps (k_fib_sweep_sparse on generated models, and the
dense k_fib_sweep with the coded model switched off), alphas compared."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    for N in (256, 1024):
        grid = S.synth_grid(N, N, seed=N)
        goal = S.synth_goal(grid)
        stream = torch.cuda.Stream()
        res = {}
        for mode in ("sparse", "dense"):
            with P.GridContext(grid, goal, gamma=0.95) as ctx:
                ctx.set_stream(stream.cuda_stream)
                ctx.model_generate()
                if mode == "dense":
                    ctx.set_tuning(ctx.TUNE_CODED_MODEL, 0)
                ctx.fib_reset()
                ctx.fib_sweep(2)
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                reps = 20
                e0.record(stream)
                ctx.fib_sweep(reps)
                e1.record(stream)
                torch.cuda.synchronize()
                res[mode] = ctx.fib_get()
                print(f"{N} {mode:6s} {e0.elapsed_time(e1) / reps * 1e3:8.2f} us/sweep", flush=True)
        d = np.abs(res["sparse"].astype(np.float64) - res["dense"]).max()
        print(f"{N} max |sparse - dense| = {d:.3g}")


if __name__ == "__main__":
    main()
