"""The bench's PBVI-leaf plan steps alone, reference order, with the PBVI
leaf dots as one chain per lane with the rows by DPP broadcast
(k_pair_dot_bq, PP2_PAIR_DOT=3, the default), packed two-chain lanes
(k_pair_dot_pk, =1), one chain per lane from LDS (k_pair_dot_1, =2), the lookahead
k_pair_seq (=0) and, with PP2_AB_FC=1, FC_LIST candidate chain sets
(PP2_PBVI_FCHAIN=1), alternated on one box:
  * 256^2 synthetic, S = 500 alphas, depth 3 (bench plan_step_pbvi_lb);
  * sparse_map_100x40, goal (95, 34), depth 50 (bench node_plan_step).
The alphas come from the full PBVI solve (PP2_ITERS backups, 0 = the
reference's 167): the tree and so the work depend on them.  p50 over
PP2_STEPS closed-loop plan steps; PP2_PBVI_STATS=1 prints the candidate
chains per row (pp2_tree.cpp) when a planner closes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    steps = int(os.environ.get("PP2_STEPS", "40"))
    g256 = S.synth_grid(256, 256, seed=256)
    node = np.load(os.path.join(ROOT, "tests", "golden", "maps", "sparse_map_100x40.npy"),
                   allow_pickle=False)
    cases = [("256x256 depth 3", g256, S.synth_goal(g256), 3),
             ("node 100x40 depth 50", node, (95, 34), 50)]
    for label, grid, goal, depth in cases:
        ctx = P.GridContext(grid, goal, gamma=0.95, device=0)
        ctx.model_generate()
        ctx.fib_solve()
        b0 = S.uniform_belief(grid)
        calls = ctx.pbvi_belief_set(b0, 500)
        ctx.pbvi_backup(int(os.environ.get("PP2_ITERS", "0")))
        res = {}
        modes = [("bq", "0", "3"), ("pk", "0", "1"), ("one", "0", "2"), ("seq", "0", "0")]
        if os.environ.get("PP2_AB_FC") == "1":
            modes.append(("fc", "1", "1"))
        for rep in range(2):
            for mode, fc, sq in modes:
                os.environ["PP2_PBVI_FCHAIN"] = fc
                os.environ["PP2_PAIR_DOT"] = sq
                with P.QVTreePlanner(ctx, max_search_tree_depth=depth, max_online_iteration=15,
                                     lower_bound_mode=1, rand_skip=calls) as pl:
                    S.closed_loop(grid, b0, pl.step, 3)
                with P.QVTreePlanner(ctx, max_search_tree_depth=depth, max_online_iteration=15,
                                     lower_bound_mode=1, rand_skip=calls) as pl:
                    ms, acts, vals = S.closed_loop(grid, b0, pl.step, steps)
                res.setdefault(mode, []).append((float(np.percentile(ms, 50)), acts, vals))
        ctx.close()
        names = {"bq": "k_pair_dot_bq (default)", "pk": "k_pair_dot_pk (PP2_PAIR_DOT=1)",
                 "one": "k_pair_dot_1 (PP2_PAIR_DOT=2)",
                 "seq": "k_pair_seq (PP2_PAIR_DOT=0)",
                 "fc": "FC_LIST candidate chain sets (PP2_PBVI_FCHAIN=1)"}
        for mode, _, _ in modes:
            name = names[mode]
            p50 = [r[0] for r in res[mode]]
            print(f"{label}: {name}: p50 {p50[0]:.3f} / {p50[1]:.3f} ms", flush=True)
        same = all(np.array_equal(res[m][k][1], res["seq"][k][1]) and
                   np.array_equal(res[m][k][2].view(np.uint32), res["seq"][k][2].view(np.uint32))
                   for k in range(2) for m, _, _ in modes)
        print(f"{label}: actions and values identical across the modes: {same}", flush=True)


if __name__ == "__main__":
    main()
