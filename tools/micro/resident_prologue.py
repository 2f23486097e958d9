"""Prologue / epilogue times of the tile-resident loop (diagnostic build, see
resident_trace.sh): per launch of n steps, over all tiles, the spread of the
tiles' entry times (dispatch ramp), entry -> tables staged, staged -> loop
top, loop top -> outputs stored (n steps), relative to the first entry."""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ["PP2_LIBRARY"] = os.path.join(HERE, "_rtrace", "libpp2_rtrace.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def ctx_kstep(ctx):
    return "?"


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import _lib
    from path_planning_2d_amd import synthetic as S
    N = int(os.environ.get("PP2_N", "1024"))
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 2000, seed=42)
    lib = _lib.load()
    fn = lib.pp2_debug_resident_prologue
    fn.argtypes = [C.c_void_p]
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.model_generate()
        ctx.belief_set(S.uniform_belief(grid))
        ctx.mdp_reset()
        ctx.loop_run(us[:10], zs[:10])
        ctx.synchronize()
        nt = None
        for n in (2, 20, 20, 200):
            for rep in range(3):
                ctx.loop_run(us[:n], zs[:n])
                ctx.synchronize()
            buf = np.zeros((1024, 8), np.uint64)
            assert fn(buf.ctypes.data) == 0
            b = buf.astype(np.int64)
            if nt is None:
                nt = int((b[:, 0] > 0).sum())
            b = b[:nt]
            t0 = b[:, 0].min()
            x = (b - t0) / 100.0
            md = lambda v: np.median(v)  # noqa: E731
            print(f"n={n:4d} kstep0 {ctx_kstep(ctx)} tiles {nt}: entry spread {x[:, 0].max():6.2f} us  staged {md(x[:, 1] - x[:, 0]):5.2f}"
                  f"  planes {md(x[:, 4] - x[:, 1]):5.2f}  tile+publish {md(x[:, 5] - x[:, 4]):5.2f}"
                  f"  mass+sync {md(x[:, 2] - x[:, 5]):5.2f}  loop+store {md(x[:, 3] - x[:, 2]):8.2f}"
                  f" ({md(x[:, 3] - x[:, 2]) / n:5.2f}/step)  last end {x[:, 3].max():8.2f} us", flush=True)


if __name__ == "__main__":
    main()
