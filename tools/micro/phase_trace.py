"""Per-workgroup phase times of one coded loop launch (diagnostic build, see
phase_trace.sh).  PP2_PAIR=1 (default): a k_loop_pair_coded launch (start ->
staged -> first step-1 quad -> step 1 done -> barrier -> step 2 done -> end);
PP2_PAIR=0: a k_loop_step_coded launch (start -> staged -> belief stored ->
sweep done -> end)."""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
os.environ["PP2_LIBRARY"] = os.path.join(HERE, "_trace", "libpp2_trace.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import _lib
    from path_planning_2d_amd import synthetic as S
    N = int(os.environ.get("PP2_N", "1024"))
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 12, seed=42)
    lib = _lib.load()
    fn = lib.pp2_debug_phase_trace
    fn.argtypes = [C.c_void_p, C.c_int]
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.model_generate()
        ctx.belief_set(S.uniform_belief(grid))
        ctx.mdp_reset()
        pair = os.environ.get("PP2_PAIR", "1") == "1"
        ctx.loop_run(us[:10], zs[:10])
        ctx.loop_run(us[10:12], zs[10:12]) if pair else ctx.loop_run(us[10:11], zs[10:11])
        ctx.synchronize()
        nb = 512
        buf = np.zeros((nb, 8), np.uint64)
        assert fn(buf.ctypes.data, nb) == 0
    used = buf[:, 0] > 0
    b = buf[used].astype(np.int64)
    t0 = b[:, 0].min()
    names = (["start", "staged", "s1quad", "s1done", "barrier", "s2done", "end"] if pair
             else ["start", "staged", "belief", "sweep", "end"])
    k = len(names)
    rel = (b[:, :k] - t0) / 100.0  # 100 MHz -> us
    print(f"{used.sum()} workgroups; times in us from the first start")
    for i, n in enumerate(names):
        col = rel[:, i]
        print(f"  {n:7s} min {col.min():7.2f}  p50 {np.median(col):7.2f}  max {col.max():7.2f}")
    d = np.diff(rel, axis=1)
    for i in range(k - 1):
        print(f"  {names[i]}->{names[i+1]:7s} p50 {np.median(d[:, i]):6.2f}  max {d[:, i].max():6.2f}")


if __name__ == "__main__":
    main()
