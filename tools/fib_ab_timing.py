"""FIB sweeps at 1024^2 on the staged kernel (k_fib_sweep_lds), event-timed
over 20 sweeps after 2, for same-box A/B of library builds (PP2_LIBRARY):
prints us per sweep (median of 3) and a digest of the alphas, which every
build must reproduce bit for bit."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, seed=N)
    stream = torch.cuda.Stream()
    with P.GridContext(grid, S.synth_goal(grid), gamma=0.95) as ctx:
        ctx.set_stream(stream.cuda_stream)
        ctx.model_generate()
        ts = []
        for _ in range(3):
            ctx.fib_reset()
            ctx.fib_sweep(2)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            ctx.fib_sweep(20)
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        dig = hashlib.sha1(np.ascontiguousarray(ctx.fib_get()).tobytes()).hexdigest()[:12]
    lib = os.path.basename(os.environ.get("PP2_LIBRARY", "libpp2_hip.so"))
    print(f"{lib}: k_fib_sweep_lds {np.median(ts):.1f} us/sweep (runs "
          f"{', '.join(f'{t:.1f}' for t in ts)}), alphas sha1 {dig}", flush=True)


if __name__ == "__main__":
    main()
