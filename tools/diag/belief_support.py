"""Diagnostic: how many cells carry belief mass along the bench's closed
loops (bench plan_step_pbvi_lb: 256^2 synthetic, depth 3; node_plan_step:
sparse_map_100x40) -- the support every reference-order chain of an
expansion walks.  A second context filters the same (action, observation)
messages the planner receives (pp2_belief_update) and counts the nonzero
cells after each message, and the cells within one step of them (the
predictions' support, a superset of every child's)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    steps = int(os.environ.get("PP2_STEPS", "200"))
    node = np.load(os.path.join(ROOT, "tests", "golden", "maps", "sparse_map_100x40.npy"),
                   allow_pickle=False)
    g256 = S.synth_grid(256, 256, seed=256)
    for label, grid, goal, depth in (("256x256", g256, S.synth_goal(g256), 3),
                                     ("node 100x40", node, (95, 34), 50)):
        ctx = P.GridContext(grid, goal, gamma=0.95, device=0)
        ctx.model_generate()
        ctx.fib_solve()
        filt = P.GridContext(grid, goal, gamma=0.95, device=0)
        filt.model_generate()
        b0 = S.uniform_belief(grid)
        filt.belief_set(b0)
        sup, dil = [], []

        def count():
            b = filt.belief_get().reshape(grid.shape)
            nz = b != 0
            d = nz.copy()
            d[1:, :] |= nz[:-1, :]
            d[:-1, :] |= nz[1:, :]
            d2 = d.copy()
            d2[:, 1:] |= d[:, :-1]
            d2[:, :-1] |= d[:, 1:]
            sup.append(int(nz.sum()))
            dil.append(int(d2.sum()))

        with P.QVTreePlanner(ctx, max_search_tree_depth=depth, max_online_iteration=15,
                             lower_bound_mode=0) as pl:
            def step(a, z, b):
                if b is None:
                    filt.belief_update(int(a), int(z))
                count()
                return pl.step(a, z, b)
            S.closed_loop(grid, b0, step, steps)
        n = grid.size
        sup, dil = np.array(sup), np.array(dil)
        for q in (10, 50, 90):
            print(f"{label}: cells {n}: support p{q} {np.percentile(sup, q):.0f}, "
                  f"one-step dilation p{q} {np.percentile(dil, q):.0f}", flush=True)
        print(f"{label}: steps with dilation <= n/2: {(dil <= n // 2).sum()} of {len(dil)}; "
              f"first 12 supports {sup[:12].tolist()}", flush=True)
        ctx.close()
        filt.close()


if __name__ == "__main__":
    main()
