"""The reference node's plan step (sparse_map_100x40, goal (95, 34), depth 50,
PBVI S = 500 leaves, reference order) with its small-grid chain sets walked
by k_chain_walk2 (PP2_CHAIN_WALK=2: terms formed beside the walk) against
k_chain_walk (the default: all terms formed first), alternated on one
box; p50 over PP2_STEPS closed-loop steps, actions and value bits compared."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    steps = int(os.environ.get("PP2_STEPS", "60"))
    grid = np.load(os.path.join(ROOT, "tests", "golden", "maps", "sparse_map_100x40.npy"),
                   allow_pickle=False)
    ctx = P.GridContext(grid, (95, 34), gamma=0.95, device=0)
    ctx.model_generate()
    ctx.fib_solve()
    b0 = S.uniform_belief(grid)
    calls = ctx.pbvi_belief_set(b0, 500)
    ctx.pbvi_backup(0)
    res = {}
    for rep in range(3):
        for mode in ("2", "1"):
            os.environ["PP2_CHAIN_WALK"] = mode
            with P.QVTreePlanner(ctx, max_search_tree_depth=50, max_online_iteration=15,
                                 lower_bound_mode=1, rand_skip=calls) as pl:
                S.closed_loop(grid, b0, pl.step, 3)
            with P.QVTreePlanner(ctx, max_search_tree_depth=50, max_online_iteration=15,
                                 lower_bound_mode=1, rand_skip=calls) as pl:
                ms, acts, vals = S.closed_loop(grid, b0, pl.step, steps)
            res.setdefault(mode, []).append((float(np.percentile(ms, 50)), acts, vals))
    ctx.close()
    names = {"2": "k_chain_walk2 (PP2_CHAIN_WALK=2)", "1": "k_chain_walk (default)"}
    for mode in ("2", "1"):
        print(f"node 100x40 depth 50: {names[mode]}: p50 " +
              " / ".join(f"{r[0]:.3f}" for r in res[mode]) + " ms", flush=True)
    same = all(np.array_equal(res["2"][k][1], res["1"][k][1]) and
               np.array_equal(res["2"][k][2].view(np.uint32), res["1"][k][2].view(np.uint32))
               for k in range(3))
    print(f"actions and values identical across the walks: {same}", flush=True)


if __name__ == "__main__":
    main()
