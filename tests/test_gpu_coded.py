"""GPU: the dictionary-coded model path (pp2_coded.hip) against the dense
kernels and the oracle.

The coded kernels compute every cell with the dense kernels' operands and fmaf
order, and reduce the belief mass over the same cell->block map and tree, so
the bar is bit equality with the dense path -- raw beliefs, masses, values and
actions -- after every step, on golden maps, ragged synthetic grids and the
1024x1024 bench grid.  Parity with the reference then follows from the dense
path's parity (test_gpu_parity.py), and is re-checked here against the oracle.
"""
import numpy as np
import pytest

from conftest import GAMMA, assert_rel_close, golden, golden_map

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pp2():
    import path_planning_2d_amd as P
    assert P.device_count() >= 1, "no GPU visible"
    return P


def ctx_pair(pp2, grid, goal):
    a = pp2.GridContext(grid, goal, gamma=float(GAMMA))
    b = pp2.GridContext(grid, goal, gamma=float(GAMMA))
    a.model_generate()
    b.model_generate()
    b.set_tuning(b.TUNE_CODED_MODEL, 0)
    ea, aa = a.model_dict_info()
    eb, ab = b.model_dict_info()
    assert aa and ea > 0 and ea == eb and not ab
    return a, b


def grids():
    from path_planning_2d_amd import synthetic as S
    out = []
    for name in ("map_3x3", "map_10x10", "sparse_map_100x40", "tile64_sparse_map_100x40"):
        out.append((name, golden_map(name), tuple(golden("model", name)["goal"])))
    for H, W, seed in ((97, 131, 3), (1, 7, 1), (5, 1, 2), (256, 256, 256), (33, 1030, 9)):
        g = S.synth_grid(H, W, seed)
        g[0, 0] = 0
        out.append((f"synth_{H}x{W}", g, (0, 0)))
    return out


GRIDS = grids()


@pytest.mark.parametrize("name,grid,goal", GRIDS, ids=[g[0] for g in GRIDS])
def test_dictionary_covers_model(pp2, name, grid, goal):
    with pp2.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        entries, active = ctx.model_dict_info()
    # 3x3 occupancy determines the tuple: <= 256 free-centre patterns, 16
    # trapped (L depends on 4 neighbours), the goal and the zero cell
    assert active and 1 <= entries <= 256 + 16 + 2


@pytest.mark.parametrize("name,grid,goal", GRIDS, ids=[g[0] for g in GRIDS])
def test_loop_coded_equals_dense_bit_exact(pp2, name, grid, goal):
    from path_planning_2d_amd import synthetic as S
    steps = 6
    us, zs, _ = S.synth_trajectory(grid, steps, seed=7)
    b0 = S.uniform_belief(grid)
    a, b = ctx_pair(pp2, grid, goal)
    with a, b:
        for c in (a, b):
            c.belief_set(b0)
            c.mdp_reset()
        for k in range(steps):
            a.loop_step(int(us[k]), int(zs[k]))
            b.loop_step(int(us[k]), int(zs[k]))
            ra, ma = a.belief_get_raw()
            rb, mb = b.belief_get_raw()
            np.testing.assert_array_equal(ra, rb, err_msg=f"raw belief, step {k}")
            assert np.float32(ma) == np.float32(mb), (k, ma, mb)
            Ja, Aa = a.mdp_get()
            Jb, Ab = b.mdp_get()
            np.testing.assert_array_equal(Ja, Jb, err_msg=f"J, step {k}")
            np.testing.assert_array_equal(Aa, Ab, err_msg=f"A, step {k}")


def test_loop_1024_coded_equals_dense(pp2):
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 4, seed=42)
    b0 = S.uniform_belief(grid)
    a, b = ctx_pair(pp2, grid, goal)
    with a, b:
        for c in (a, b):
            c.belief_set(b0)
            c.mdp_reset()
            c.loop_run(us, zs)
        np.testing.assert_array_equal(a.belief_get(), b.belief_get())
        Ja, Aa = a.mdp_get()
        Jb, Ab = b.mdp_get()
        np.testing.assert_array_equal(Ja, Jb)
        np.testing.assert_array_equal(Aa, Ab)


@pytest.mark.parametrize("name", ["map_10x10", "sparse_map_100x40", "tile64_sparse_map_100x40"])
def test_mdp_coded_matches_golden(pp2, name):
    """Coded sweeps reproduce the reference's values/actions bit for bit."""
    grid = golden_map(name)
    m = golden("model", name)
    g = golden("mdp", name)
    with pp2.GridContext(grid, tuple(m["goal"]), gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        assert ctx.model_dict_info()[1]
        ctx.mdp_reset()
        ctx.mdp_sweep(7)
        J, A = ctx.mdp_get()
        np.testing.assert_array_equal(J, g["J7"])
        np.testing.assert_array_equal(A, g["A7"])


def test_mdp_solve_coded_equals_dense(pp2, oracle):
    from path_planning_2d_amd import synthetic as S
    N = 256
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    a, b = ctx_pair(pp2, grid, goal)
    with a, b:
        ra = a.mdp_solve()
        rb = b.mdp_solve()
        assert ra == rb
        Ja, Aa = a.mdp_get()
        Jb, Ab = b.mdp_get()
        np.testing.assert_array_equal(Ja, Jb)
        np.testing.assert_array_equal(Aa, Ab)
    T, _, _ = oracle.model_pomdp(grid, goal)
    _, Cc = oracle.model_mdp(grid, goal)
    Jo = np.zeros(N * N, np.float32)
    for _ in range(25):
        Jo, Ao = oracle.mdp_sweep(N, N, GAMMA, T, Cc, Jo)
    with pp2.GridContext(grid, goal, gamma=float(GAMMA)) as c:
        c.model_generate()
        c.mdp_reset()
        c.mdp_sweep(25)
        J, A = c.mdp_get()
    np.testing.assert_array_equal(J, Jo)
    np.testing.assert_array_equal(A, Ao)


def test_toggling_paths_mid_run(pp2):
    """Pending partial masses hand over between the coded and dense kernels."""
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(64, 72, 5)
    grid[0, 0] = 0
    us, zs, _ = S.synth_trajectory(grid, 8, seed=3)
    b0 = S.uniform_belief(grid)
    a, b = ctx_pair(pp2, grid, (0, 0))
    with a, b:
        for c in (a, b):
            c.belief_set(b0)
            c.mdp_reset()
        for k in range(8):
            a.set_tuning(a.TUNE_CODED_MODEL, k % 2)
            a.loop_step(int(us[k]), int(zs[k]))
            b.loop_step(int(us[k]), int(zs[k]))
        np.testing.assert_array_equal(a.belief_get(), b.belief_get())
        np.testing.assert_array_equal(a.mdp_get()[0], b.mdp_get()[0])


def test_irregular_model_falls_back_to_dense(pp2):
    """A model with more distinct cells than the LDS dictionary holds runs on
    the dense kernels (and a regular one re-enables the coded path)."""
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(40, 48, 11)
    grid[0, 0] = 0
    with pp2.GridContext(grid, (0, 0), gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        T, L, R, Cc = ctx.model_download()
        e0, _ = ctx.model_dict_info()
        rng = np.random.default_rng(0)
        Tn = (T * (1.0 + 1e-3 * rng.random(T.shape))).astype(np.float32)
        ctx.model_upload(Tn, L, R, Cc)
        assert ctx.model_dict_info() == (0, False)
        b0 = S.uniform_belief(grid)
        ctx.belief_set(b0)
        ctx.belief_update(1, 3)
        assert np.isfinite(ctx.belief_get()).all()
        ctx.model_upload(T, L, R, Cc)
        assert ctx.model_dict_info() == (e0, True)
        # perturbing one cell whose tuple is shared adds exactly one entry
        tup = np.concatenate([T.reshape(len(T), -1), Cc, L], axis=1)
        _, inv, cnt = np.unique(tup, axis=0, return_inverse=True, return_counts=True)
        cell = int(np.nonzero(cnt[inv.reshape(-1)] >= 2)[0][0])
        T1 = T.copy()
        T1[cell, 0, 0] = np.float32(0.3)
        ctx.model_upload(T1, L, R, Cc)
        e1, act = ctx.model_dict_info()
        assert act and e1 == e0 + 1


def test_model_upload_on_whole_grid_shard(pp2):
    """pp2_model_upload on a rows=(0, H) shard context (round-5 ADVICE): its
    dense planes keep only kDenseHalo halo rows while the dictionary build
    walks the deep shard halo, so the upload builds the dictionary from a
    transient full-halo copy.  The shard's coded dictionary equals the
    unsharded context's, and an uploaded (perturbed) model runs the same
    loop steps bit for bit on both."""
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(96, 128, 5)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 6, seed=3)
    b0 = S.uniform_belief(grid)
    with pp2.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            pp2.GridContext(grid, goal, gamma=float(GAMMA), rows=(0, grid.shape[0])) as sh:
        sh.shard_comm_init(pp2.GridContext.rccl_unique_id(), 1, 0)
        ref.model_generate()
        T, L, R, Cc = ref.model_download()
        T1 = T.copy()
        T1[5 * 128 + 7, 4, 4] = np.float32(0.5)  # one more dictionary entry
        for c in (ref, sh):
            c.model_upload(T1, L, R, Cc)
        assert sh.model_dict_info() == ref.model_dict_info()
        assert ref.model_dict_info()[1]
        for c in (ref, sh):
            c.belief_set(b0)
            c.mdp_reset()
        for k in range(6):
            ref.loop_step(int(us[k]), int(zs[k]))
            sh.loop_step(int(us[k]), int(zs[k]))
        np.testing.assert_array_equal(sh.mdp_get()[0], ref.mdp_get()[0])
        np.testing.assert_array_equal(sh.mdp_get()[1], ref.mdp_get()[1])
        assert_rel_close(sh.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=1e-30,
                         msg="belief on the uploaded model")


def test_off_support_model_uses_full_rows(pp2):
    """A T entry outside its action's base-kernel support rules out the
    sparse LDS rows; the full-row coded kernels must still match dense."""
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(48, 60, 21)
    grid[0, 0] = 0
    us, zs, _ = S.synth_trajectory(grid, 5, seed=8)
    us[:] = 4  # the stay action reads the off-support entry below
    b0 = S.uniform_belief(grid)
    a, b = ctx_pair(pp2, grid, (0, 0))
    with a, b:
        T, L, R, Cc = a.model_download()
        cell = 17 * 60 + 23
        T[cell, 4, 0] = np.float32(0.25)  # stay action: support is {4} only
        for c in (a, b):
            c.model_upload(T, L, R, Cc)
            c.belief_set(b0)
            c.mdp_reset()
        assert a.model_dict_info()[1] and not b.model_dict_info()[1]
        for k in range(5):
            a.loop_step(int(us[k]), int(zs[k]))
            b.loop_step(int(us[k]), int(zs[k]))
        np.testing.assert_array_equal(a.belief_get_raw()[0], b.belief_get_raw()[0])
        np.testing.assert_array_equal(a.mdp_get()[0], b.mdp_get()[0])
        np.testing.assert_array_equal(a.mdp_get()[1], b.mdp_get()[1])
        a.mdp_sweep(9)
        b.mdp_sweep(9)
        np.testing.assert_array_equal(a.mdp_get()[0], b.mdp_get()[0])


@pytest.mark.parametrize("block", [8, 5, 3])
@pytest.mark.parametrize("H,W", [(1024, 1024), (1000, 1100), (1024, 1022)])
def test_step_pairs_equal_single_steps(pp2, H, W, block):
    """pp2_loop_run fuses two steps of a normalisation block per launch
    (k_loop_pair_coded: step 1 over the tile plus a one-row halo in LDS) on
    grids with a 4096-cell tile per CU.  Raw beliefs, masses, values and
    actions equal the one-launch-per-step path bit for bit, across odd chunk
    lengths and block boundaries."""
    from path_planning_2d_amd import synthetic as S
    wp = (W + 3) // 4 * 4
    assert 5 * (2 * wp + 8) <= 3 * 4096 and (-(-H * wp // 1024) + 3) // 4 >= 256
    grid = S.synth_grid(H, W, H + W)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 13, seed=3)
    b0 = S.uniform_belief(grid)
    a = pp2.GridContext(grid, goal, gamma=float(GAMMA))
    b = pp2.GridContext(grid, goal, gamma=float(GAMMA))
    with a, b:
        b.set_tuning(b.TUNE_STEP_PAIRS, 0)
        for c in (a, b):
            c.set_tuning(c.TUNE_RESIDENT, 0)  # pairs, not the resident loop (test_gpu_resident.py)
            c.model_generate()
            assert c.model_dict_info()[1]
            c.set_tuning(c.TUNE_NORM_BLOCK, block)
            c.belief_set(b0)
            c.mdp_reset()
        # the pair kernel really runs on a (every gate of loop_pair_fits holds)
        assert a.loop_steps_per_launch() == 2 and b.loop_steps_per_launch() == 1
        for lo, hi in ((0, 3), (3, 4), (4, 13)):
            a.loop_run(us[lo:hi], zs[lo:hi])
            b.loop_run(us[lo:hi], zs[lo:hi])
            ra, ma = a.belief_get_raw()
            rb, mb = b.belief_get_raw()
            np.testing.assert_array_equal(ra, rb, err_msg=f"raw belief after {hi} steps")
            assert np.float32(ma) == np.float32(mb), (hi, ma, mb)
            Ja, Aa = a.mdp_get()
            Jb, Ab = b.mdp_get()
            np.testing.assert_array_equal(Ja, Jb, err_msg=f"J after {hi} steps")
            np.testing.assert_array_equal(Aa, Ab, err_msg=f"A after {hi} steps")


def _bits(x):
    return np.ascontiguousarray(x, np.float32).view(np.uint32)


@pytest.mark.parametrize("bad", ["neg_zero", "negative", "inf", "nan", "huge"])
def test_cost_precondition_keeps_coded_equal_dense(pp2, oracle, bad):
    """The sparse rows drop T == 0 terms of the Bellman backup, which equals
    the dense fmaf chain only for finite costs >= +0 (pp2_runtime.cpp
    build_model_dict).  An uploaded model with a -0, negative, infinite, NaN
    or overflowing cost must leave the coded path bit-identical to dense
    (values compared as bit patterns, so -0 != +0)."""
    from path_planning_2d_amd import synthetic as S
    grid = golden_map("sparse_map_100x40")
    goal = (95, 34)
    T, L, R = oracle.model_pomdp(grid, goal)
    _, Cc = oracle.model_mdp(grid, goal)
    Cc = Cc.copy()
    free = np.flatnonzero(grid.reshape(-1) == 0)
    cells = free[::37]
    val = {"neg_zero": -0.0, "negative": -2.5, "inf": np.inf, "nan": np.nan,
           "huge": 3.0e38}[bad]
    Cc[cells, 4] = np.float32(val)
    Cc[cells[::2], 1] = np.float32(val)
    us, zs, _ = S.synth_trajectory(grid, 6, seed=11)
    b0 = S.uniform_belief(grid)
    a, b = ctx_pair(pp2, grid, goal)
    with a, b:
        for c in (a, b):
            c.model_upload(T, L, R, Cc)
            c.belief_set(b0)
            c.mdp_reset()
        assert a.model_dict_info()[1] and not b.model_dict_info()[1]
        for k in range(6):
            a.loop_step(int(us[k]), int(zs[k]))
            b.loop_step(int(us[k]), int(zs[k]))
            np.testing.assert_array_equal(_bits(a.mdp_get()[0]), _bits(b.mdp_get()[0]),
                                          err_msg=f"J bits, step {k}")
            np.testing.assert_array_equal(a.mdp_get()[1], b.mdp_get()[1])
        a.mdp_sweep(25)
        b.mdp_sweep(25)
        np.testing.assert_array_equal(_bits(a.mdp_get()[0]), _bits(b.mdp_get()[0]))
        np.testing.assert_array_equal(a.mdp_get()[1], b.mdp_get()[1])
        np.testing.assert_array_equal(_bits(a.belief_get_raw()[0]), _bits(b.belief_get_raw()[0]))


@pytest.mark.parametrize("bad", ["neg_zero", "negative", "inf"])
def test_belief_precondition_keeps_coded_equal_dense(pp2, bad):
    """The sparse belief gather drops T == 0 terms: exact only for finite
    beliefs >= +0.  A belief set with a -0, negative or infinite entry moves
    the context to the dense kernels until the next valid belief_set."""
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(64, 72, 5)
    grid[0, 0] = 0
    us, zs, _ = S.synth_trajectory(grid, 5, seed=3)
    b0 = S.uniform_belief(grid)
    val = {"neg_zero": -0.0, "negative": -1e-3, "inf": np.inf}[bad]
    bb = b0.copy()
    bb[np.flatnonzero(grid.reshape(-1) == 0)[::11]] = np.float32(val)
    a, b = ctx_pair(pp2, grid, (0, 0))
    with a, b:
        for c in (a, b):
            c.belief_set(bb)
            c.mdp_reset()
        for k in range(5):
            a.loop_step(int(us[k]), int(zs[k]))
            b.loop_step(int(us[k]), int(zs[k]))
            ra, ma = a.belief_get_raw()
            rb, mb = b.belief_get_raw()
            np.testing.assert_array_equal(_bits(ra), _bits(rb), err_msg=f"raw belief, step {k}")
            assert _bits(np.float32(ma)) == _bits(np.float32(mb))
