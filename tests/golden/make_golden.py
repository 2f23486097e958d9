"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (the only place /root/reference exists):

    python tests/golden/make_golden.py

What is frozen, and where it comes from:

* ``maps/*.npy`` -- the reference's own map images
  (/root/reference/path_planning_2d/maps/*.png), decoded with PIL and
  thresholded like PathPlanning2dBase::loadMapFromFile (pixel <= 250 ->
  occupied; src/pomdp/path_planning_2d.cu:243-257).  Data, not code.
* ``glibc_rand.npy`` -- the first 2000 values of the real glibc ``rand()`` from
  the default seed (the reference never seeds; search_tree_cuda.cu:332),
  captured through ctypes: pins the oracle's rand() restatement.
* ``model_<map>.npz``, ``belief_<map>.npz``, ``mdp_<map>.npz``,
  ``fib_<map>.npz``, ``pbvi_<map>.npz`` -- outputs of the CPU oracle (oracle/pp2_oracle.c), the
  restatement of the reference kernels.  The reference itself cannot be built
  or run here, so these are "parity unpinned" vectors that
  freeze the oracle and feed the GPU tests (which may not read
  /root/reference).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from path_planning_2d_amd import maps as M  # noqa: E402
from path_planning_2d_amd import synthetic as S  # noqa: E402

REF_MAPS = "/root/reference/path_planning_2d/maps"
GAMMA = np.float32(0.95)

# (name, goal) -- goals from the launch files (launch/*.launch:2-9) and
# SURVEY.md §8(d) for the 64x64 tile.
MAP_GOALS = {
    "map_3x3": (1, 1),
    "map_5x5": (3, 2),
    "map_10x10": (8, 8),
    "map_100x40": (95, 34),
    "sparse_map_100x40": (95, 34),
    "tile64_sparse_map_100x40": (58, 58),
}


def save_maps():
    os.makedirs(os.path.join(HERE, "maps"), exist_ok=True)
    grids = {}
    for name in ["map_3x3", "map_5x5", "map_10x10", "map_100x40",
                 "sparse_map_100x40"]:
        g = M.load_map(os.path.join(REF_MAPS, name + ".png"))
        np.save(os.path.join(HERE, "maps", name + ".npy"), g)
        grids[name] = g
    t = M.tile_map(grids["sparse_map_100x40"], 64, 64)
    np.save(os.path.join(HERE, "maps", "tile64_sparse_map_100x40.npy"), t)
    grids["tile64_sparse_map_100x40"] = t
    return grids


def free_goal(grid, goal):
    gx, gy = goal
    if grid[gy, gx] == 0:
        return goal
    ys, xs = np.nonzero(grid == 0)
    k = int(np.argmin((xs - gx) ** 2 + (ys - gy) ** 2))
    return int(xs[k]), int(ys[k])


def main():
    grids = save_maps()
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    np.save(os.path.join(HERE, "glibc_rand.npy"),
            np.array([libc.rand() for _ in range(2000)], np.int32))

    goals = {}
    for name, grid in grids.items():
        goal = free_goal(grid, MAP_GOALS[name])
        goals[name] = goal
        H, W = grid.shape
        T, L, R = O.model_pomdp(grid, goal)
        T2, Cc = O.model_mdp(grid, goal)
        assert np.array_equal(T, T2), "MDP T must equal POMDP T"
        np.savez_compressed(os.path.join(HERE, f"model_{name}.npz"), T=T, L=L,
                            R=R, C=Cc, goal=np.array(goal, np.int32))

        # belief trajectory: uniform start, 64 seeded (u, z) steps, each the
        # reference step "kernel + sequential fp32 renormalisation"
        if name in ("map_10x10", "sparse_map_100x40",
                    "tile64_sparse_map_100x40"):
            us, zs, st = S.synth_trajectory(grid, 64, seed=42)
            b = S.uniform_belief(grid)
            keep = {}
            for k in range(64):
                b = O.belief_step(H, W, T, L, b, us[k], zs[k], mode="seq")
                if (k + 1) in (1, 2, 4, 8, 16, 32, 64):
                    keep[f"b{k + 1}"] = b.copy()
            np.savez_compressed(os.path.join(HERE, f"belief_{name}.npz"),
                                us=us, zs=zs, states=st,
                                b0=S.uniform_belief(grid), **keep)

        if name in ("map_10x10", "sparse_map_100x40",
                    "tile64_sparse_map_100x40"):
            J, A, n, nrm = O.mdp_solve(H, W, GAMMA, T, Cc)
            J7 = np.zeros(H * W, np.float32)
            for _ in range(7):
                J7, A7 = O.mdp_sweep(H, W, GAMMA, T, Cc, J7)
            np.savez_compressed(os.path.join(HERE, f"mdp_{name}.npz"), J=J, A=A,
                                sweeps=np.int32(n), norm=np.float64(nrm),
                                J7=J7, A7=A7)
            print(f"{name}: MDP converged after {n} sweeps (norm {nrm:.6f})")

        if name in ("map_10x10", "sparse_map_100x40"):
            a, n, nrm = O.fib_solve(H, W, GAMMA, T, L, R)
            np.savez_compressed(os.path.join(HERE, f"fib_{name}.npz"), alphas=a,
                                sweeps=np.int32(n), norm=np.float32(nrm))
            print(f"{name}: FIB converged after {n} sweeps (norm {nrm:.6f})")
    print("goals:", goals)


def save_pbvi():
    """PBVI (point_based_value_iteration_cuda.cu): generateBeliefSet from the
    uniform belief with the reference's unseeded rand() (seed 1), then
    backupAlphaVectors from zero alphas -- all 167 backups on 10x10 at
    S = 32, 2 backups on 100x40 at S = 48.  Needs only the committed maps:
    ``python tests/golden/make_golden.py pbvi``."""
    for name, S_, iters in (("map_10x10", 32, 0), ("sparse_map_100x40", 48, 2)):
        grid = np.load(os.path.join(HERE, "maps", name + ".npy"), allow_pickle=False)
        goal = tuple(np.load(os.path.join(HERE, f"model_{name}.npz"))["goal"])
        H, W = grid.shape
        T, L, R = O.model_pomdp(grid, goal)
        b0 = S.uniform_belief(grid)
        B, _ = O.pbvi_belief_set(H, W, T, L, b0, S_)
        al, act, n = O.pbvi_backup(H, W, GAMMA, T, L, R, B, iterations=iters)
        np.savez_compressed(os.path.join(HERE, f"pbvi_{name}.npz"), beliefs=B, alphas=al,
                            actions=act, iterations=np.int32(n))
        print(f"{name}: PBVI S={S_}, {n} backups")


if __name__ == "__main__":
    if sys.argv[1:] == ["pbvi"]:
        save_pbvi()
    else:
        main()
        save_pbvi()
