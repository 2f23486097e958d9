"""Per-step duration over a 64-step launch of the tile-resident loop
(diagnostic build, resident_trace.sh): median over tiles 1..15 of step t's
top -> step t+1's top for wave 0, t = 0 .. 62, to see whether the first
steps of a launch run slower than the rest (tile entry skew, cold caches)."""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ["PP2_LIBRARY"] = os.path.join(HERE, "_rtrace", "libpp2_rtrace.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import _lib
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 64, seed=42)
    lib = _lib.load()
    fn = lib.pp2_debug_resident_trace
    fn.argtypes = [C.c_void_p]
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.model_generate()
        ctx.belief_set(S.uniform_belief(grid))
        ctx.mdp_reset()
        for rep in range(3):
            ctx.loop_run(us, zs)
            ctx.synchronize()
        buf = np.zeros((16, 64, 4, 4), np.uint64)
        assert fn(buf.ctypes.data) == 0
    b = buf.astype(np.int64)[1:, :, 0, 0] / 100.0  # tiles 1..15, wave 0, step tops (us)
    d = np.median(b[:, 1:] - b[:, :-1], axis=0)
    print("step durations (us), t = 0..62:")
    print(" ".join(f"{v:.2f}" for v in d))
    print(f"steps 0-7 mean {d[:8].mean():.2f}, 8-62 mean {d[8:].mean():.2f}")


if __name__ == "__main__":
    main()
