"""Closed-loop plan steps for rocprofv3 --kernel-trace --stats: kernels per
plan step and their time against the step's wall time.
  PP2_CASE=256   256^2 synthetic, depth 3 (bench plan_step; PP2_LB=1: PBVI
                 leaves, S = 500, bench plan_step_pbvi_lb)
  PP2_CASE=node  sparse_map_100x40, goal (95, 34), depth 50, PBVI leaves
                 S = 500 (bench node_plan_step)
PP2_REF: reference_order (default 1, the drop-in's mode); PP2_STEPS steps.
PP2_FC_STATS=1: the chain-set drivers' counters per set kind over the timed
steps (pp2_debug_fc_stats)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    case = os.environ.get("PP2_CASE", "256")
    steps = int(os.environ.get("PP2_STEPS", "100"))
    if case == "node":
        grid = np.load(os.path.join(ROOT, "tests", "golden", "maps", "sparse_map_100x40.npy"),
                       allow_pickle=False)
        goal, depth, lb = (95, 34), 50, 1
    else:
        grid = S.synth_grid(256, 256, seed=256)
        goal, depth, lb = S.synth_goal(grid), 3, int(os.environ.get("PP2_LB", "0"))
    ctx = P.GridContext(grid, goal, gamma=0.95, device=0)
    ctx.model_generate()
    ctx.fib_solve()
    b0 = S.uniform_belief(grid)
    calls = 0
    if lb:
        calls = ctx.pbvi_belief_set(b0, 500)
        ctx.pbvi_backup(int(os.environ.get("PP2_ITERS", "0")))
    ref = int(os.environ.get("PP2_REF", "1"))

    def planner():
        return P.QVTreePlanner(ctx, max_search_tree_depth=depth, max_online_iteration=15,
                               lower_bound_mode=lb, rand_skip=calls, reference_order=ref)
    with planner() as pl:
        S.closed_loop(grid, b0, pl.step, 3)
    stats = None
    if os.environ.get("PP2_FC_STATS") == "1":
        import ctypes as C
        from path_planning_2d_amd import _lib
        stats = _lib.load().pp2_debug_fc_stats
        stats.argtypes = [C.c_void_p, C.c_int]
        stats.restype = C.c_int
        assert stats(None, 1) == 0
        buf = np.zeros(256, np.int32)
        stats(buf.ctypes.data, 0)  # (clears the warm-up's counts)
    with planner() as pl:
        t0 = time.perf_counter()
        ms, _, _ = S.closed_loop(grid, b0, pl.step, steps)
        el = time.perf_counter() - t0
        info = pl.info()
    if stats is not None:
        assert stats(buf.ctypes.data, 0) == 0
        names = ["row", "row x9", "child", "child x9", "list", "list x9", "-", "-"]
        for kind in range(8):
            c = buf[32 * kind:32 * kind + 32].view(np.uint32).astype(np.int64)  # (wrapping sums)
            if c[7]:
                print(f"set {names[kind]:8s}: chains {c[7]}, per chain: iterations {c[0] / c[7]:.1f}, "
                      f"fallbacks {c[1] / c[7]:.1f}, exact rounds {c[2] / c[7]:.1f}, stash hits "
                      f"{c[3] / c[7]:.1f}; us: flags {c[4] / c[7] / 100:.2f}, stash {c[5] / c[7] / 100:.2f}, "
                      f"walk {c[6] / c[7] / 100:.2f}; fallbacks: no entry {c[8] / c[7]:.1f}, other "
                      f"binade {c[9] / c[7]:.1f}, crossing {c[10] / c[7]:.1f}; s_memtime per chain: steps "
                      f"{c[11] / c[7]:.0f}, fetches {c[12] / c[7]:.0f}, exact {c[13] / c[7]:.0f}, "
                      f"chunk 0 {c[14] / c[7]:.0f}; longest chain {c[15] / 100:.2f} us (exact chunks {c[16]}, "
                      f"rounds {c[17]}, slow steps {c[18]}, stash hits {c[19]}, chunks {c[20]}, "
                      f"group {c[21]}); tables: {c[22] / c[7]:.1f} plans per chain, "
                      f"{c[23] / max(c[22], 1):.0f} cycles each", flush=True)
    ctx.close()
    print(f"case {case} lb {lb} reference_order={ref}: {steps} plan steps: p50 "
          f"{np.percentile(ms, 50):.3f} ms, mean {ms.mean():.3f} ms, wall {el * 1e3:.1f} ms, "
          f"expansions {info['expansions']}", flush=True)


if __name__ == "__main__":
    main()
