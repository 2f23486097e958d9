"""Diagnostic: how many of the PBVI alphas (S = 500, full solve) are exact
duplicates, and for a few beliefs how many alphas' dots lie within the
candidate bound of the maximum (pp2_fchain.hip k_pbvi_cands) -- distinct
alpha vectors and distinct fp64 dot values among them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    g256 = S.synth_grid(256, 256, seed=256)
    node = np.load(os.path.join(ROOT, "tests", "golden", "maps", "sparse_map_100x40.npy"),
                   allow_pickle=False)
    for label, grid, goal in (("256", g256, S.synth_goal(g256)), ("node", node, (95, 34))):
        with P.GridContext(grid, goal, gamma=0.95, device=0) as ctx:
            ctx.model_generate()
            b0 = S.uniform_belief(grid)
            ctx.pbvi_solve(b0, 500)
            al, act = ctx.pbvi_get()
            B = ctx.pbvi_get_beliefs()
        n = grid.size
        u = np.unique(al.view(np.uint32), axis=0)
        print(f"{label}: {al.shape[0]} alphas, {u.shape[0]} distinct; actions {np.bincount(act, minlength=9)}")
        c = (n + 1100) * 2.0 ** -24
        for k in (0, 1, 7, 100, 300, 499):
            b = B[k].astype(np.float64)
            d = al.astype(np.float64) @ b
            lo = (d - c * np.abs(d)).max()
            cand = np.nonzero(d + c * np.abs(d) >= lo)[0]
            dv = np.unique(d[cand])
            sup = b > 0
            ua = np.unique(al[cand][:, sup].view(np.uint32), axis=0)
            print(f"  belief {k}: max dot {d.max():.4f}, bound {c * abs(d.max()):.4f}, candidates "
                  f"{cand.size}, distinct dots {dv.size}, distinct on support {ua.shape[0]}, "
                  f"support {sup.sum()}; spread of the 10 best: "
                  f"{np.sort(d)[::-1][:10] - d.max()}")


if __name__ == "__main__":
    main()
