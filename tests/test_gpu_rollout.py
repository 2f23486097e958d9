"""GPU: batched fp16 QV-tree rollouts (BASELINE configs[4]) against an fp32
rollout restated with the oracle kernels.

Per copy and step the reference math is: reward <b_k, R[:,u]>, observation
likelihood p_k = sum(L_z . T_u^T b_k), b_{k+1} = normalise(...); leaf FIB
bound max_i <b_D, alpha_i>.  The device stores beliefs as per-copy
max-normalised fp16 (rounding 2^-11 per step), so the tolerance here is the
fp16 one: rewards / likelihoods / bounds / values within rel 3e-3, beliefs
within rel 5e-3 of each cell plus 1e-4 of the copy's peak (fp16 subnormal
range)."""
import numpy as np
import pytest

from conftest import GAMMA, golden, golden_map

pytestmark = pytest.mark.gpu


def oracle_rollout(O, grid, T, L, R, alphas, b0, us, zs, copies_idx):
    H, W = grid.shape
    D = us.shape[0]
    out = {}
    for c in copies_idx:
        b = b0.astype(np.float32)
        rw, pr = [], []
        for k in range(D):
            u, z = int(us[k, c]), int(zs[k, c])
            rw.append(float(np.dot(b.astype(np.float64), R[:, u])))
            nb = O.belief_update(H, W, T, L, b, u, z)
            p = float(nb.astype(np.float64).sum())
            pr.append(p)
            b = (nb.astype(np.float64) / p).astype(np.float32)
        dots = b.astype(np.float64) @ alphas.astype(np.float64)
        ub = float(dots.max())
        v = sum(float(GAMMA) ** k * rw[k] for k in range(D)) + float(GAMMA) ** D * ub
        out[c] = (np.array(rw), np.array(pr), ub, v, b)
    return out


def close(a, b, rel):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= rel * np.abs(b) + 1e-7)


def check(res, oc, r, rel=3e-3, check_beliefs=True):
    for c, (rw, pr, ub, v, b) in oc.items():
        assert close(res["rewards"][:, c], rw, rel), f"copy {c} rewards"
        assert close(res["obs_prob"][:, c], pr, rel), f"copy {c} obs_prob"
        assert close(res["leaf_upper"][c], ub, rel), f"copy {c} leaf"
        assert close(res["value"][c], v, rel), f"copy {c} value"
        if check_beliefs:
            got = r.belief(c).astype(np.float64)
            err = np.abs(got - b)
            assert np.all(err <= 5e-3 * np.abs(b) + 1e-4 * b.max()), f"copy {c} belief"


def test_rollout_small_all_copies(oracle):
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    name = "tile64_sparse_map_100x40"
    grid = golden_map(name)
    m = golden("model", name)
    H, W = grid.shape
    copies, depth = 96, 5
    b0 = S.uniform_belief(grid)
    us, zs = S.rollout_trajectories(grid, b0, copies, depth, seed=11)
    with P.GridContext(grid, tuple(m["goal"]), gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.fib_solve()
        alphas = ctx.fib_get()
        with P.BatchedRollout(ctx, copies, depth) as r:
            r.set_root(b0)
            r.run(us, zs)
            res = r.results()
            oc = oracle_rollout(oracle, grid, m["T"], m["L"], m["R"], alphas, b0, us, zs,
                                range(copies))
            check(res, oc, r)


def test_rollout_config5_512_4096x5(oracle):
    """BASELINE configs[4]: 512x512, 4096 copies x depth 5, fp16 beliefs."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N, copies, depth = 512, 4096, 5
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    b0 = S.uniform_belief(grid)
    us, zs = S.rollout_trajectories(grid, b0, copies, depth, seed=13)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.fib_solve(max_sweeps=40)
        alphas = ctx.fib_get()
        with P.BatchedRollout(ctx, copies, depth) as r:
            r.set_root(b0)
            r.run(us, zs)
            res = r.results()
            assert np.isfinite(res["value"]).all()
            assert ((res["obs_prob"] > 0) & (res["obs_prob"] <= 1.0 + 1e-3)).all()
            T, L, R = oracle.model_pomdp(grid, goal)
            pick = [0, 1, 777, 2048, 4095]
            oc = oracle_rollout(oracle, grid, T, L, R, alphas, b0, us, zs, pick)
            check(res, oc, r)


@pytest.mark.parametrize("H,W,copies,depth", [(37, 53, 61, 4), (128, 128, 300, 5)])
def test_rollout_coded_equals_dense(H, W, copies, depth):
    """The coded-model rollout (T_u / R_u / L from the LDS dictionary) gives
    bit-identical results and beliefs to the dense-plane rollout."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(H, W, seed=H * W)
    goal = S.synth_goal(grid)
    b0 = S.uniform_belief(grid)
    us, zs = S.rollout_trajectories(grid, b0, copies, depth, seed=5)
    out = []
    for coded in (1, 0):
        with P.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
            ctx.model_generate()
            ctx.set_tuning(ctx.TUNE_CODED_MODEL, coded)
            assert ctx.model_dict_info()[1] == bool(coded)
            ctx.fib_solve(max_sweeps=20)
            with P.BatchedRollout(ctx, copies, depth) as r:
                r.set_root(b0)
                r.run(us, zs)
                res = r.results()
                beliefs = [r.belief(c) for c in (0, copies // 2, copies - 1)]
        out.append((res, beliefs))
    (ra, ba), (rb, bb) = out
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)
    for x, y in zip(ba, bb):
        np.testing.assert_array_equal(x, y)


def test_rollout_runs_restart_from_root():
    """Every run starts from the root image set by set_root (its first step
    reads the one image for all copies): a second run after one set_root
    equals a fresh set_root + run bit for bit, and before any run every copy
    reads back as the root."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(96, 128, seed=9)
    goal = S.synth_goal(grid)
    b0 = S.uniform_belief(grid)
    copies, depth = 40, 3
    us1, zs1 = S.rollout_trajectories(grid, b0, copies, depth, seed=1)
    us2, zs2 = S.rollout_trajectories(grid, b0, copies, depth, seed=2)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.fib_solve(max_sweeps=20)
        with P.BatchedRollout(ctx, copies, depth) as r:
            r.set_root(b0)
            for c in (0, copies - 1):
                got = r.belief(c).astype(np.float64)
                assert np.all(np.abs(got - b0) <= 1e-3 * b0.max())
            r.run(us1, zs1)
            r.run(us2, zs2)
            again = r.results()
            b_again = r.belief(copies // 2)
            r.set_root(b0)
            r.run(us2, zs2)
            fresh = r.results()
            b_fresh = r.belief(copies // 2)
    for k in fresh:
        np.testing.assert_array_equal(again[k], fresh[k], err_msg=k)
    np.testing.assert_array_equal(b_again, b_fresh)


@pytest.mark.parametrize("H,W,copies,scale", [(40, 64, 96, 1.0), (40, 64, 96, -3e5),
                                              (300, 200, 130, 1e25), (300, 200, 130, -1e-20),
                                              (37, 50, 61, 1.0), (37, 50, 61, -3e5)])
def test_rollout_leaf_dots(H, W, copies, scale):
    """The leaf FIB bound max_i <b_D, alpha_i> (fast_informed_bound_cuda.cu:
    278-297) against float64 dots of the same stored fp16 beliefs, for alpha
    planes of magnitude |scale| (random per plane and cell, so that the
    argmax plane varies by copy): within rel 1e-5.  40 x 64 and 300 x 200
    (8 slabs of cells, 130 copies: a partial 64-copy group) take the MFMA
    pass (copy rows 16-B aligned, wp % 8 == 0), whose per-plane power-of-two
    scaling and fp16 hi + lo split these magnitudes exercise; 37 x 50 (wp 52)
    the fmaf pass."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(H, W, seed=H + W)
    goal = S.synth_goal(grid)
    b0 = S.uniform_belief(grid)
    us, zs = S.rollout_trajectories(grid, b0, copies, 3, seed=3)
    rng = np.random.default_rng(H * W)
    alphas = (scale * (0.5 + rng.random((H * W, 9)))).astype(np.float32)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.fib_set(alphas)
        with P.BatchedRollout(ctx, copies, 3) as r:
            r.set_root(b0)
            r.run(us, zs)
            res = r.results()
            a64 = alphas.astype(np.float64)
            winners = set()
            for c in range(copies):
                b = r.belief(c).astype(np.float64)
                dots = (b @ a64) / b.sum()
                winners.add(int(np.argmax(dots)))
                ub = float(dots.max())
                got = float(res["leaf_upper"][c])
                assert abs(got - ub) <= 1e-5 * abs(ub), (c, got, ub)
            assert len(winners) >= 3, winners


def test_rollout_leaf_follows_fib():
    """The MFMA leaf pass keeps the packed alpha columns between runs while
    the context's FIB alphas are unchanged, and repacks them after fib_set /
    fib_sweep: a second run repeats the bound bit for bit, alphas x 2 (exact)
    give exactly twice the bound, and after a FIB sweep the bound follows the
    new alphas."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    H, W, copies = 40, 64, 70
    grid = S.synth_grid(H, W, seed=77)
    goal = S.synth_goal(grid)
    b0 = S.uniform_belief(grid)
    us, zs = S.rollout_trajectories(grid, b0, copies, 2, seed=4)
    rng = np.random.default_rng(5)
    alphas = (-20.0 * (0.5 + rng.random((H * W, 9)))).astype(np.float32)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.fib_set(alphas)
        with P.BatchedRollout(ctx, copies, 2) as r:
            def leaf():
                r.set_root(b0)
                r.run(us, zs)
                return r.results()["leaf_upper"].copy()
            l1 = leaf()
            np.testing.assert_array_equal(leaf(), l1)
            ctx.fib_set(2.0 * alphas)
            np.testing.assert_array_equal(leaf(), 2.0 * l1)
            ctx.fib_sweep(1)
            l3 = leaf()
            a = ctx.fib_get().astype(np.float64)
            for c in (0, copies - 1):
                b = r.belief(c).astype(np.float64)
                ub = float(((b @ a) / b.sum()).max())
                assert abs(l3[c] - ub) <= 1e-5 * abs(ub), (c, l3[c], ub)
