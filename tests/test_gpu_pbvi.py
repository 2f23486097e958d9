"""GPU parity of the PBVI lower bound (pp2_pbvi_*) against the oracle's
restatement of point_based_value_iteration_cuda.cu.

* Belief set (generateBeliefSet :165-295): bit-exact.  Both draw the
  reference's glibc rand() stream; the device batches the samples, updates,
  normalisations and L1 distances of a round but keeps their arithmetic.
  Checked up to the reference node's own size, S = 500 on the 100x40 map.
* Backup (backupAlphaVectors :319-641): alpha vectors and actions bit-exact.
  The Sgemm's summation order belongs to cuBLAS and is not published; both
  sides pin it as the x-ordered fmaf chain (the MFMA f32 GEMM computes exactly
  that), so this parity is with the oracle, unpinned against cuBLAS.
* evaluatePbviCpu (:678-699): bit-exact.
At S = 500 on 100x40 (the reference's configuration) the backup is checked by
properties: valid actions, finite values, below the FIB upper bound.
"""
import os

import numpy as np
import pytest

from conftest import GAMMA, golden, golden_map

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pp2():
    import path_planning_2d_amd as P
    assert P.device_count() >= 1, "no GPU visible"
    return P


def setup(pp2, oracle, name):
    from path_planning_2d_amd import synthetic as S
    g = golden_map(name)
    goal = tuple(golden("model", name)["goal"])
    H, W = g.shape
    ctx = pp2.GridContext(g, goal, gamma=float(GAMMA))
    ctx.model_generate()
    T, L, R = oracle.model_pomdp(g, goal)
    return ctx, (H, W, T, L, R), S.uniform_belief(g)


def rand_draws(S):
    n, sizes = 1, []
    while n < S:
        sizes.append(n)
        n = min(S, n + (n if n < 100 else 100))
    return 27 * sum(sizes)


@pytest.mark.parametrize("name,S", [("map_10x10", 150), ("map_10x10", 7),
                                    ("sparse_map_100x40", 130)])
def test_belief_set_bit_exact(pp2, oracle, name, S):
    ctx, (H, W, T, L, R), b0 = setup(pp2, oracle, name)
    with ctx:
        calls = ctx.pbvi_belief_set(b0, S)
        B = ctx.pbvi_get_beliefs()
    Bo, rs = oracle.pbvi_belief_set(H, W, T, L, b0, S)
    assert calls == rand_draws(S)
    np.testing.assert_array_equal(B, Bo)
    # the streams end in the same state
    nxt = oracle.RandState(1)
    for _ in range(calls):
        nxt.next()
    assert nxt.next() == rs.next()


def test_belief_set_reference_size(pp2, oracle):
    """S = 500 on the 100x40 map: the reference node's own belief set."""
    ctx, (H, W, T, L, R), b0 = setup(pp2, oracle, "sparse_map_100x40")
    with ctx:
        ctx.pbvi_belief_set(b0, 500)
        B = ctx.pbvi_get_beliefs()
    Bo, _ = oracle.pbvi_belief_set(H, W, T, L, b0, 500)
    np.testing.assert_array_equal(B, Bo)


@pytest.mark.parametrize("name,S,iters", [("map_10x10", 32, 0), ("map_10x10", 130, 4),
                                          ("sparse_map_100x40", 24, 3)])
def test_backup_bit_exact(pp2, oracle, name, S, iters):
    ctx, (H, W, T, L, R), b0 = setup(pp2, oracle, name)
    Bo, _ = oracle.pbvi_belief_set(H, W, T, L, b0, S)
    al_o, act_o, n = oracle.pbvi_backup(H, W, GAMMA, T, L, R, Bo, iterations=iters)
    if iters == 0:
        assert n == oracle.pbvi_iterations(GAMMA) == 167
    with ctx:
        ctx.pbvi_set_beliefs(Bo)
        ctx.pbvi_backup(iters)
        al, act = ctx.pbvi_get()
        v, a = ctx.pbvi_evaluate(Bo[:9])
    np.testing.assert_array_equal(act, act_o)
    np.testing.assert_array_equal(al, al_o)
    for i in range(9):
        vo, ao = oracle.pbvi_eval(Bo[i], al_o, act_o)
        assert np.float32(vo) == v[i] and ao == a[i], i


def test_solve_equals_set_then_backup(pp2, oracle):
    ctx, (H, W, T, L, R), b0 = setup(pp2, oracle, "map_10x10")
    with ctx:
        calls = ctx.pbvi_solve(b0, 40)
        al, act = ctx.pbvi_get()
    Bo, _ = oracle.pbvi_belief_set(H, W, T, L, b0, 40)
    al_o, act_o, _ = oracle.pbvi_backup(H, W, GAMMA, T, L, R, Bo)
    assert calls == rand_draws(40)
    np.testing.assert_array_equal(act, act_o)
    np.testing.assert_array_equal(al, al_o)


def test_evaluate_batch_matches_oracle(pp2, oracle):
    """evaluatePbviCpu on beliefs outside the set, with alphas set by hand."""
    ctx, (H, W, T, L, R), b0 = setup(pp2, oracle, "sparse_map_100x40")
    rng = np.random.default_rng(5)
    S, hw = 37, H * W
    al = rng.uniform(-40, 0, (S, hw)).astype(np.float32)
    act = rng.integers(0, 9, S).astype(np.uint8)
    beliefs = rng.random((11, hw)).astype(np.float32)
    beliefs /= beliefs.sum(1, keepdims=True)
    with ctx:
        ctx.pbvi_set(al, act)
        v, a = ctx.pbvi_evaluate(beliefs)
    for i in range(len(beliefs)):
        vo, ao = oracle.pbvi_eval(beliefs[i], al, act)
        assert np.float32(vo) == v[i] and ao == a[i], i


@pytest.mark.parametrize("mode", ["3", "1", "2", "0"])
def test_evaluate_dot_shapes_bit_exact(pp2, oracle, monkeypatch, mode):
    """The leaf-dot kernels (PP2_PAIR_DOT 3: one chain per lane, rows by DPP
    broadcast; 1: packed two-chain lanes; 2: one chain per lane from LDS; 0:
    k_pair_seq) against evaluatePbviCpu's x-ordered chain
    on adversarial rows: an odd number of beliefs (a packed pair with no
    partner row), zeros, subnormal and huge terms, mixed-sign alphas, a
    ragged S."""
    monkeypatch.setenv("PP2_PAIR_DOT", mode)
    ctx, (H, W, T, L, R), b0 = setup(pp2, oracle, "sparse_map_100x40")
    rng = np.random.default_rng(11)
    S, hw = 53, H * W
    al = rng.uniform(-40, 5, (S, hw)).astype(np.float32)
    al[3, ::7] = 3e38
    al[4, ::5] = -1e-30
    act = rng.integers(0, 9, S).astype(np.uint8)
    beliefs = (rng.random((19, hw)) * (rng.random((19, hw)) < 0.6)).astype(np.float32)
    beliefs[2, 1::3] = np.float32(1e-42)  # subnormal terms
    beliefs[5] = 0.0
    beliefs[5, hw - 1] = 1.0
    beliefs[7, ::11] = 7e-39
    with ctx:
        ctx.pbvi_set(al, act)
        v, a = ctx.pbvi_evaluate(beliefs)
    for i in range(len(beliefs)):
        vo, ao = oracle.pbvi_eval(beliefs[i], al, act)
        assert np.float32(vo).view(np.uint32) == np.float32(v[i]).view(np.uint32) and ao == a[i], i


def test_reference_configuration_properties(pp2):
    """S = 500, 100x40, the reference's iteration count: every belief's
    action is valid, values are finite and below the FIB upper bound (within
    the gamma^167 tail of the zero start)."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    name = "sparse_map_100x40"
    g = golden_map(name)
    goal = tuple(golden("model", name)["goal"])
    b0 = S.uniform_belief(g)
    with P.GridContext(g, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.fib_solve()
        fib = ctx.fib_get()
        ctx.pbvi_solve(b0, 500)
        al, act = ctx.pbvi_get()
        B = ctx.pbvi_get_beliefs()
        v, a = ctx.pbvi_evaluate(B)
    assert al.shape == (500, g.size) and np.isfinite(al).all()
    assert act.max() <= 8
    ub = (B @ fib.astype(np.float64)).max(axis=1)
    assert np.all(v <= ub + 0.05), float((v - ub).max())
    assert np.all(v < 0) and np.all(v > -5.0 / (1.0 - 0.95) - 1e-3)


def test_pbvi_text_round_trip(pp2, oracle, tmp_path):
    """savePbviDataToFile / loadPbviDataFromFile formats."""
    ctx, (H, W, T, L, R), b0 = setup(pp2, oracle, "map_10x10")
    with ctx:
        ctx.pbvi_solve(b0, 20)
        al, act = ctx.pbvi_get()
        ctx.pbvi_save(str(tmp_path))
        lines = open(tmp_path / "pbvi_alphas").read().splitlines()
        assert len(lines) == 20 and len(lines[0]) == 15 * H * W
        want = np.array([[float(lines[i][15 * k:15 * k + 15]) for k in range(H * W)]
                         for i in range(20)], np.float32)
        np.testing.assert_allclose(want, al, atol=1e-7)
        acts = open(tmp_path / "pbvi_actions").read().splitlines()
        assert [int(s) for s in acts] == act.tolist() and all(len(s) == 10 for s in acts)
        with pp2.GridContext(golden_map("map_10x10"), ctx.goal, gamma=float(GAMMA)) as c2:
            c2.model_generate()
            c2.pbvi_load(str(tmp_path), 20)
            al2, act2 = c2.pbvi_get()
        np.testing.assert_array_equal(al2, want)
        np.testing.assert_array_equal(act2, act)
        with pytest.raises(pp2.Pp2Error):
            ctx.pbvi_load(str(tmp_path), 21)  # too few lines: "Data dimension is not set properly"


def test_fib_text_round_trip(pp2, tmp_path):
    name = "map_10x10"
    g = golden_map(name)
    goal = tuple(golden("model", name)["goal"])
    with pp2.GridContext(g, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.fib_solve()
        al = ctx.fib_get()
        ctx.fib_save(str(tmp_path))
        rows = open(tmp_path / "fib_alphas").read().splitlines()
        assert len(rows) == g.size and all(len(r) == 15 * 9 for r in rows)
        acts = open(tmp_path / "fib_actions").read().split()
        assert acts == [str(u) for u in range(9)]
        ctx.fib_reset()
        ctx.fib_load(str(tmp_path))
        np.testing.assert_allclose(ctx.fib_get(), al, atol=1e-7)


def test_pbvi_rejects_sharded_and_unset(pp2):
    from path_planning_2d_amd import synthetic as S
    g = S.synth_grid(16, 12, 3)
    with pp2.GridContext(g, (0, 0), gamma=float(GAMMA)) as ctx:
        with pytest.raises(pp2.Pp2Error):
            ctx.pbvi_backup(1)  # no model / no set
        ctx.model_generate()
        with pytest.raises(pp2.Pp2Error):
            ctx.pbvi_backup(1)  # no belief set
        with pytest.raises(pp2.Pp2Error):
            ctx.pbvi_belief_set(S.uniform_belief(g), 0)
        with pytest.raises(pp2.Pp2Error):
            ctx.pbvi_belief_set(S.uniform_belief(g), 4097)
    with pp2.GridContext(g, (0, 0), gamma=float(GAMMA), rows=(0, 8)) as sh:
        sh.model_generate()
        with pytest.raises(pp2.Pp2Error):
            sh.pbvi_belief_set(np.ones(sh.cells, np.float32) / sh.cells, 4)


@pytest.mark.parametrize("name", ["map_10x10", "sparse_map_100x40"])
def test_pbvi_matches_golden(pp2, name):
    """Belief set, alphas and actions equal the frozen oracle fixtures
    (tests/golden/pbvi_<map>.npz) bit for bit."""
    from path_planning_2d_amd import synthetic as S
    g = golden_map(name)
    p = golden("pbvi", name)
    with pp2.GridContext(g, tuple(golden("model", name)["goal"]), gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.pbvi_belief_set(S.uniform_belief(g), p["beliefs"].shape[0])
        np.testing.assert_array_equal(ctx.pbvi_get_beliefs(), p["beliefs"])
        ctx.pbvi_backup(int(p["iterations"]))
        al, act = ctx.pbvi_get()
    np.testing.assert_array_equal(al, p["alphas"])
    np.testing.assert_array_equal(act, p["actions"])


@pytest.mark.parametrize("case", ["map_3x3", "row_1x9", "col_7x1", "single_belief"])
def test_pbvi_edge_shapes(pp2, oracle, case):
    """Tiny and degenerate grids and S = 1: belief set and 5 backups equal the
    oracle bit for bit; an empty evaluation batch is a no-op."""
    from path_planning_2d_amd import synthetic as S
    if case == "map_3x3":
        g = golden_map("map_3x3")
        goal = tuple(golden("model", "map_3x3")["goal"])
        Sn = 20
    elif case == "row_1x9":
        g = np.zeros((1, 9), np.uint8)
        g[0, 4] = 1
        goal, Sn = (8, 0), 9
    elif case == "col_7x1":
        g = np.zeros((7, 1), np.uint8)
        goal, Sn = (0, 6), 5
    else:
        g = golden_map("map_10x10")
        goal = tuple(golden("model", "map_10x10")["goal"])
        Sn = 1
    H, W = g.shape
    T, L, R = oracle.model_pomdp(g, goal)
    b0 = S.uniform_belief(g)
    Bo, _ = oracle.pbvi_belief_set(H, W, T, L, b0, Sn)
    al_o, act_o, _ = oracle.pbvi_backup(H, W, GAMMA, T, L, R, Bo, iterations=5)
    with pp2.GridContext(g, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.pbvi_belief_set(b0, Sn)
        np.testing.assert_array_equal(ctx.pbvi_get_beliefs(), Bo)
        ctx.pbvi_backup(5)
        al, act = ctx.pbvi_get()
        v, a = ctx.pbvi_evaluate(np.zeros((0, H * W), np.float32))
        assert v.size == 0 and a.size == 0
    np.testing.assert_array_equal(al, al_o)
    np.testing.assert_array_equal(act, act_o)
