"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle
and the golden fixtures.

Bar (BASELINE.json north_star): beliefs and values within 1e-5 relative fp32,
cell indices / argmax actions bit-exact.  Where the device computes the same
fp32 operation sequence as the reference (model tensors, Bellman sweeps, FIB
sweeps, the unnormalised belief kernel output) the tests demand bit equality;
the normalised belief differs from the reference only by the order of the
normalising sum (deferred, tree-reduced on device vs sequential on host), so
it is held to rel 1e-5 with an FLT_MIN floor (FTZ).
"""
import numpy as np
import pytest

from conftest import GAMMA, assert_rel_close, golden, golden_map

pytestmark = pytest.mark.gpu

SMALL = ["map_3x3", "map_5x5", "map_10x10", "map_100x40", "sparse_map_100x40",
         "tile64_sparse_map_100x40"]


@pytest.fixture(scope="module")
def pp2():
    import path_planning_2d_amd as P
    assert P.device_count() >= 1, "no GPU visible"
    return P


def make_ctx(pp2, grid, goal, cpt=4):
    ctx = pp2.GridContext(grid, goal, gamma=float(GAMMA))
    ctx.set_cells_per_lane(cpt)
    ctx.model_generate()
    return ctx


@pytest.mark.parametrize("name", SMALL)
def test_model_generation_bit_exact(pp2, name):
    g = golden("model", name)
    with make_ctx(pp2, golden_map(name), tuple(g["goal"])) as ctx:
        T, L, R, C = ctx.model_download()
    np.testing.assert_array_equal(T, g["T"])
    np.testing.assert_array_equal(L, g["L"])
    np.testing.assert_array_equal(R, g["R"])
    np.testing.assert_array_equal(C, g["C"])


@pytest.mark.parametrize("H,W,seed", [(256, 256, 256), (97, 131, 3), (1, 7, 1),
                                      (5, 1, 2)])
def test_model_generation_synthetic(pp2, oracle, H, W, seed):
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(H, W, seed)
    grid[0, 0] = 0
    goal = (0, 0)
    T, L, R = oracle.model_pomdp(grid, goal)
    _, C = oracle.model_mdp(grid, goal)
    with make_ctx(pp2, grid, goal) as ctx:
        Td, Ld, Rd, Cd = ctx.model_download()
    np.testing.assert_array_equal(Td, T)
    np.testing.assert_array_equal(Ld, L)
    np.testing.assert_array_equal(Rd, R)
    np.testing.assert_array_equal(Cd, C)


@pytest.mark.parametrize("cpt", [1, 2, 4])
@pytest.mark.parametrize("name", ["map_10x10", "sparse_map_100x40",
                                  "tile64_sparse_map_100x40"])
def test_belief_kernel_bit_exact_one_step(pp2, oracle, name, cpt):
    """cudaBayesBeliefUpdate output (unnormalised) is bit-identical."""
    grid = golden_map(name)
    H, W = grid.shape
    m = golden("model", name)
    bt = golden("belief", name)
    with make_ctx(pp2, grid, tuple(m["goal"]), cpt) as ctx:
        for u in range(9):
            for z in (0, 5, 15):
                ctx.belief_set(bt["b8"])
                ctx.belief_update(u, z)
                raw, mass = ctx.belief_get_raw()
                want = oracle.belief_update(H, W, m["T"], m["L"], bt["b8"], u, z)
                np.testing.assert_array_equal(raw, want)
                assert_rel_close(mass, oracle.lib().orc_sum_f64(want.size, want),
                                 rel=2e-6, msg="mass")


@pytest.mark.parametrize("cpt", [1, 4])
@pytest.mark.parametrize("name", ["map_10x10", "sparse_map_100x40",
                                  "tile64_sparse_map_100x40"])
def test_belief_trajectory_matches_golden(pp2, name, cpt):
    grid = golden_map(name)
    m = golden("model", name)
    bt = golden("belief", name)
    with make_ctx(pp2, grid, tuple(m["goal"]), cpt) as ctx:
        ctx.belief_set(bt["b0"])
        for k in range(64):
            ctx.belief_update(bt["us"][k], bt["zs"][k])
            if f"b{k + 1}" in bt:
                got = ctx.belief_get()
                assert_rel_close(got, bt[f"b{k + 1}"], rel=1e-5,
                                 msg=f"{name} step {k + 1}")
                assert abs(float(got.astype(np.float64).sum()) - 1.0) < 1e-5


@pytest.mark.parametrize("name", ["map_10x10", "sparse_map_100x40",
                                  "tile64_sparse_map_100x40"])
@pytest.mark.parametrize("cpt", [1, 2, 4])
def test_mdp_sweeps_bit_exact(pp2, name, cpt):
    grid = golden_map(name)
    m = golden("model", name)
    g = golden("mdp", name)
    with make_ctx(pp2, grid, tuple(m["goal"]), cpt) as ctx:
        ctx.mdp_reset()
        ctx.mdp_sweep(7)
        J, A = ctx.mdp_get()
        np.testing.assert_array_equal(J, g["J7"])
        np.testing.assert_array_equal(A, g["A7"])
        sweeps, norm = ctx.mdp_solve()
        J, A = ctx.mdp_get()
    assert sweeps == int(g["sweeps"])
    np.testing.assert_array_equal(J, g["J"])
    np.testing.assert_array_equal(A, g["A"])


def test_mdp_256_bit_exact_vs_oracle(pp2, oracle):
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(256, 256, 256)
    goal = S.synth_goal(grid)
    T, Cc = oracle.model_mdp(grid, goal)
    J = np.zeros(256 * 256, np.float32)
    for _ in range(40):
        J, A = oracle.mdp_sweep(256, 256, GAMMA, T, Cc, J)
    with make_ctx(pp2, grid, goal) as ctx:
        ctx.mdp_reset()
        ctx.mdp_sweep(40)
        Jd, Ad = ctx.mdp_get()
    np.testing.assert_array_equal(Jd, J)
    np.testing.assert_array_equal(Ad, A)


@pytest.mark.parametrize("name", ["map_10x10", "sparse_map_100x40"])
def test_fib_bit_exact(pp2, oracle, name):
    grid = golden_map(name)
    H, W = grid.shape
    m = golden("model", name)
    g = golden("fib", name)
    a = np.zeros((H * W, 9), np.float32)
    for _ in range(3):
        a = oracle.fib_sweep(H, W, GAMMA, m["T"], m["L"], m["R"], a)
    with make_ctx(pp2, grid, tuple(m["goal"])) as ctx:
        ctx.fib_reset()
        ctx.fib_sweep(3)
        np.testing.assert_array_equal(ctx.fib_get(), a)
        sweeps, norm = ctx.fib_solve()
        got = ctx.fib_get()
    assert sweeps == int(g["sweeps"])
    np.testing.assert_array_equal(got, g["alphas"])


@pytest.mark.parametrize("cpt", [1, 4])
def test_loop_step_matches_separate_ops(pp2, oracle, cpt):
    """The fused north-star step == belief update + Bellman sweep."""
    name = "tile64_sparse_map_100x40"
    grid = golden_map(name)
    H, W = grid.shape
    m = golden("model", name)
    bt = golden("belief", name)
    g = golden("mdp", name)
    with make_ctx(pp2, grid, tuple(m["goal"]), cpt) as ctx:
        ctx.belief_set(bt["b0"])
        ctx.mdp_reset()
        ctx.loop_run(bt["us"][:7], bt["zs"][:7])
        J, A = ctx.mdp_get()
        np.testing.assert_array_equal(J, g["J7"])
        np.testing.assert_array_equal(A, g["A7"])
        ctx.loop_run(bt["us"][7:8], bt["zs"][7:8])
        assert_rel_close(ctx.belief_get(), bt["b8"], rel=1e-5, msg="loop belief")


def test_loop_1024_properties(pp2, oracle):
    """Full bench size: belief stays a distribution, matches the fp64-normalised
    oracle to 1e-5 relative after a few steps, values match bit-exactly."""
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 3, seed=42)
    b0 = S.uniform_belief(grid)
    T, L, R = oracle.model_pomdp(grid, goal)
    b = b0
    for k in range(3):
        b = oracle.belief_step(N, N, T, L, b, us[k], zs[k], mode="f64")
    del R
    with make_ctx(pp2, grid, goal) as ctx:
        ctx.belief_set(b0)
        ctx.mdp_reset()
        ctx.loop_run(us, zs)
        got = ctx.belief_get()
        J, A = ctx.mdp_get()
    assert (got >= 0).all()
    assert abs(got.astype(np.float64).sum() - 1.0) < 1e-5
    assert_rel_close(got, b, rel=1e-5, msg="1024 belief vs fp64 oracle")
    _, Cc = oracle.model_mdp(grid, goal)
    Jo = np.zeros(N * N, np.float32)
    for _ in range(3):
        Jo, Ao = oracle.mdp_sweep(N, N, GAMMA, T, Cc, Jo)
    np.testing.assert_array_equal(J, Jo)
    np.testing.assert_array_equal(A, Ao)


def test_model_roundtrip_text_format(pp2, tmp_path):
    name = "map_10x10"
    m = golden("model", name)
    with make_ctx(pp2, golden_map(name), tuple(m["goal"])) as ctx:
        ctx.model_save(str(tmp_path))
        lines = open(tmp_path / "model_data_trans_prob").read().splitlines()
        assert len(lines) == 100 * 9 and len(lines[0]) == 9 * 15
    with pp2.GridContext(golden_map(name), tuple(m["goal"])) as ctx2:
        ctx2.model_load(str(tmp_path))
        T, L, R, C = ctx2.model_download()
    # "%15.8f" keeps 8 decimals: the reload is within 5e-9 absolute
    assert np.abs(T - m["T"]).max() <= 5e-9
    assert np.abs(L - m["L"]).max() <= 5e-9
    assert np.abs(R - m["R"]).max() <= 5e-9


def test_errors_surface_as_exceptions(pp2):
    grid = golden_map("map_10x10")
    with pp2.GridContext(grid, (8, 7)) as ctx:
        with pytest.raises(pp2.Pp2Error):
            ctx.belief_update(0, 0)  # model not generated yet
        ctx.model_generate()
        with pytest.raises(pp2.Pp2Error):
            ctx.belief_update(9, 0)
        with pytest.raises(pp2.Pp2Error):
            ctx.model_load("/nonexistent-dir")


@pytest.mark.parametrize("block", [1, 2, 5, 8])
@pytest.mark.parametrize("cpt", [1, 4])
def test_loop_normalisation_blocks(pp2, oracle, block, cpt):
    """PP2_TUNE_NORM_BLOCK: the stored belief is divided by its exact mass
    every `block` steps (x 2^96, exact) and by 1 in between.  Over the 64-step
    golden trajectory every read belief matches the reference's per-step
    normalised sequence to rel 1e-5 (FTZ floor), at every block phase; values
    and actions are untouched (bit-exact).  block 1 is per-step division."""
    name = "sparse_map_100x40"
    grid = golden_map(name)
    m = golden("model", name)
    bt = golden("belief", name)
    with make_ctx(pp2, grid, tuple(m["goal"]), cpt) as ctx:
        ctx.set_tuning(ctx.TUNE_NORM_BLOCK, block)
        ctx.belief_set(bt["b0"])
        ctx.mdp_reset()
        done = 0
        for k in (1, 2, 4, 8, 16, 32, 64):
            ctx.loop_run(bt["us"][done:k], bt["zs"][done:k])
            done = k
            assert_rel_close(ctx.belief_get(), bt[f"b{k}"], rel=1e-5, abs_floor=1e-30,
                             msg=f"block {block}, step {k}")
            if k == 8:
                J, A = ctx.mdp_get()
                g = golden("mdp", name)
                Jr = np.zeros_like(J)
                with make_ctx(pp2, grid, tuple(m["goal"]), cpt) as ref:
                    ref.mdp_reset()
                    ref.mdp_sweep(8)
                    Jr, Ar = ref.mdp_get()
                np.testing.assert_array_equal(J, Jr)
                np.testing.assert_array_equal(A, Ar)
                del g
        with pytest.raises(pp2.Pp2Error):
            ctx.set_tuning(ctx.TUNE_NORM_BLOCK, 9)


def test_loop_blocks_equal_across_paths(pp2):
    """Coded and dense loops under the default normalisation blocks stay
    bit-identical (raw beliefs and masses) through block boundaries."""
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(96, 130, 4)
    grid[0, 0] = 0
    us, zs, _ = S.synth_trajectory(grid, 19, seed=5)
    b0 = S.uniform_belief(grid)
    a = pp2.GridContext(grid, (0, 0), gamma=float(GAMMA))
    b = pp2.GridContext(grid, (0, 0), gamma=float(GAMMA))
    with a, b:
        for c in (a, b):
            c.model_generate()
            c.belief_set(b0)
            c.mdp_reset()
        b.set_tuning(b.TUNE_CODED_MODEL, 0)
        for k in range(19):
            a.loop_step(int(us[k]), int(zs[k]))
            b.loop_step(int(us[k]), int(zs[k]))
            ra, ma = a.belief_get_raw()
            rb, mb = b.belief_get_raw()
            np.testing.assert_array_equal(ra, rb, err_msg=f"step {k}")
            assert np.float32(ma) == np.float32(mb)


@pytest.mark.parametrize("H,W,force", [(1024, 1024, ""), (1025, 700, ""), (301, 333, "1"),
                                       (257, 1030, "1"), (1, 700, "1"), (256, 256, "0")])
def test_fib_lds_equals_dense_geometries(pp2, monkeypatch, H, W, force):
    """The likelihood-staging FIB kernel (2-row x 256-column blocks, L rows
    y0-1 .. y0+2 in LDS; chosen from 1024 blocks up, PP2_FIB_LDS forces it)
    on grids whose rows and widths do not fill its blocks, and the sparse
    kernel it replaces: alphas equal the dense k_fib_sweep's bit for bit."""
    from path_planning_2d_amd import synthetic as S
    monkeypatch.setenv("PP2_FIB_LDS", force)
    grid = S.synth_grid(H, W, seed=H + 3 * W)
    goal = S.synth_goal(grid)
    with make_ctx(pp2, grid, goal) as a, make_ctx(pp2, grid, goal) as b:
        b.set_tuning(b.TUNE_CODED_MODEL, 0)
        assert a.model_dict_info()[1], "sparse (LDS) FIB path not selected"
        for c in (a, b):
            c.fib_reset()
            c.fib_sweep(3)
        np.testing.assert_array_equal(a.fib_get(), b.fib_get())


def test_fib_nonfinite_alphas_take_full_sums(pp2):
    """Uploaded alphas with an infinity: the support-only kernels' dropped
    terms are fmaf(0 * L, alpha, s), which is NaN, not s, for alpha = inf --
    the context then sweeps with the full 9-term sums, so it still equals
    the dense kernel bit for bit (NaNs included)."""
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(64, 64, seed=7)
    goal = S.synth_goal(grid)
    with make_ctx(pp2, grid, goal) as a, make_ctx(pp2, grid, goal) as b:
        b.set_tuning(b.TUNE_CODED_MODEL, 0)
        a.fib_reset()
        a.fib_sweep(5)
        al = a.fib_get()
        al.reshape(-1)[1000] = -np.inf
        for c in (a, b):
            c.fib_set(al)
            c.fib_sweep(2)
        np.testing.assert_array_equal(a.fib_get().view(np.uint32), b.fib_get().view(np.uint32))


@pytest.mark.parametrize("name", ["map_10x10", "sparse_map_100x40", "tile64_sparse_map_100x40"])
def test_fib_sparse_equals_dense(pp2, name):
    """k_fib_sweep_sparse (support-only terms, observation-outer loads) gives
    the dense k_fib_sweep's alphas bit for bit, sweep by sweep and solved."""
    grid = golden_map(name)
    m = golden("model", name)
    with make_ctx(pp2, grid, tuple(m["goal"])) as a, make_ctx(pp2, grid, tuple(m["goal"])) as b:
        b.set_tuning(b.TUNE_CODED_MODEL, 0)
        for c in (a, b):
            c.fib_reset()
        for k in range(4):
            a.fib_sweep(1)
            b.fib_sweep(1)
            np.testing.assert_array_equal(a.fib_get(), b.fib_get(), err_msg=f"sweep {k}")
        ra, rb = a.fib_solve(), b.fib_solve()
        assert ra == rb
        np.testing.assert_array_equal(a.fib_get(), b.fib_get())
