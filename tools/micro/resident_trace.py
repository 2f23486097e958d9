"""Per-step phase times of the tile-resident loop (diagnostic build, see
resident_trace.sh): for tiles 1..15, wave 0 (the tile's first row: waits for
the tile above) and wave 5 (an interior row at 1024^2), the median over steps
8..63 of  top -> rows in hand -> computed+published -> after the barrier ->
next top.  PP2_RES_HX picks the hand-off variant."""
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
    N = int(os.environ.get("PP2_N", "1024"))
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
        ctx.loop_run(us, zs)
        ctx.synchronize()
        buf = np.zeros((16, 64, 4, 4), np.uint64)
        assert fn(buf.ctypes.data) == 0
    b = buf.astype(np.int64)
    tot = (b[1:, 56, 0, 0] - b[1:, 8, 0, 0]) / 100.0 / 48
    print(f"N={N} prio={os.environ.get('PP2_RES_PRIO', '1')}: us/step (tiles 1..15, steps 8..56, "
          f"block starts included) median {np.median(tot):.2f}")
    names = ["top->rows", "rows->done", "done->barrier", "barrier->top"]
    for w, role in ((0, "row 0 (top edge) wave 0"), (1, "row 1 (interior) wave 5"),
                    (2, "row 2 (interior) wave 9"), (3, "row 3 (bottom edge) wave 12")):
        x = b[1:, 8:63, w, :] / 100.0
        nxt = b[1:, 9:64, w, 0] / 100.0
        d = [x[..., 1] - x[..., 0], x[..., 2] - x[..., 1], x[..., 3] - x[..., 2], nxt - x[..., 3]]
        print("  " + role + ": " + "  ".join(f"{n} {np.median(v):.2f}" for n, v in zip(names, d)))


if __name__ == "__main__":
    main()
