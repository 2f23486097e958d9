"""GPU: the tile-resident loop (pp2_resident.hip) -- pp2_loop_run's whole
trajectory in one launch, one tile of whole rows per CU kept in LDS,
neighbour rows handed over by per-wave flags, block-start masses behind an
arrival counter.

The bar is bit equality with the one-launch-per-step path (which equals the
dense path and the oracle: test_gpu_coded.py, test_gpu_parity.py): raw
beliefs, masses, values and actions after every run, across runs of odd and
even length (the last step's partials land in the input's buffer on even
runs with a pending mass), block boundaries inside and across launches,
normalisation blocks 1..8, partial last tiles, padded widths and runs longer
than one launch (2048 steps).
"""
import numpy as np
import pytest

from conftest import GAMMA

pytestmark = pytest.mark.gpu

RESIDENT_STEPS = 2048


@pytest.fixture(scope="module")
def pp2():
    import path_planning_2d_amd as P
    assert P.device_count() >= 1, "no GPU visible"
    return P


def _pair(pp2, H, W, block, seed):
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(H, W, seed)
    goal = S.synth_goal(grid)
    a = pp2.GridContext(grid, goal, gamma=float(GAMMA))
    b = pp2.GridContext(grid, goal, gamma=float(GAMMA))
    b.set_tuning(b.TUNE_RESIDENT, 0)
    b.set_tuning(b.TUNE_STEP_PAIRS, 0)
    b0 = S.uniform_belief(grid)
    for c in (a, b):
        c.model_generate()
        assert c.model_dict_info()[1]
        c.set_tuning(c.TUNE_NORM_BLOCK, block)
        c.belief_set(b0)
        c.mdp_reset()
    return grid, a, b


def _same(a, b, what):
    ra, ma = a.belief_get_raw()
    rb, mb = b.belief_get_raw()
    np.testing.assert_array_equal(ra.view(np.uint32), rb.view(np.uint32),
                                  err_msg=f"raw belief {what}")
    assert np.float32(ma).view(np.uint32) == np.float32(mb).view(np.uint32), (what, ma, mb)
    Ja, Aa = a.mdp_get()
    Jb, Ab = b.mdp_get()
    np.testing.assert_array_equal(Ja.view(np.uint32), Jb.view(np.uint32), err_msg=f"J {what}")
    np.testing.assert_array_equal(Aa, Ab, err_msg=f"A {what}")


# (H, W): the 1024^2 bench grid (4 rows per tile), 2-row and 1-row tiles, a
# partial last tile (700 rows over 256 CUs: 3-row tiles), a padded width
GEOMS = [(1024, 1024), (512, 512), (256, 1024), (700, 768), (1024, 1022), (300, 256)]


@pytest.mark.parametrize("block", [8, 5, 1])
@pytest.mark.parametrize("H,W", GEOMS)
def test_resident_equals_single_steps(pp2, H, W, block):
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, H, W, block, H * 7 + W)
    with a, b:
        assert a.loop_steps_per_launch() == RESIDENT_STEPS, "resident loop not selected"
        assert b.loop_steps_per_launch() == 1
        us, zs, _ = S.synth_trajectory(grid, 40, seed=5)
        # chunks: even and odd lengths, starting on and off block boundaries
        launches = 0
        for lo, hi in ((0, 2), (2, 5), (5, 6), (6, 16), (16, 40)):
            a.loop_run(us[lo:hi], zs[lo:hi])
            b.loop_run(us[lo:hi], zs[lo:hi])
            a.synchronize()
            launches += hi - lo >= 2  # a one-step run takes the single-step launch
            assert a.resident_launches()[0] == launches and b.resident_launches() == (0, 0)
            _same(a, b, f"after {hi} steps")


# 2-D tiles (two tile columns, PP2_TUNE_RESIDENT_TILE_COLS): the automatic
# choice on 512 x 2048 (the view of a 256-row rank share of config 4's 2048^2
# grid: 4 x 1024 tiles instead of 2 x 2048), and forced on a partial last tile
# row (301 rows in 3-row tiles), a padded width (200 x 1022) and 256 x 2048
GEOMS_2D = [(512, 2048, 0), (301, 1024, 2), (200, 1022, 2), (256, 2048, 2)]


@pytest.mark.parametrize("block", [8, 1])
@pytest.mark.parametrize("H,W,tc", GEOMS_2D)
def test_resident_2d_tiles_equal_single_steps(pp2, H, W, tc, block):
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, H, W, block, H * 5 + W)
    with a, b:
        if tc:
            a.set_tuning(a.TUNE_RESIDENT_TILE_COLS, tc)
        tiles, rt, cols = a.resident_tiling()
        assert cols == 2 and tiles <= 256, (tiles, rt, cols)
        us, zs, _ = S.synth_trajectory(grid, 40, seed=6)
        launches = 0
        for lo, hi in ((0, 2), (2, 5), (5, 6), (6, 16), (16, 40)):
            a.loop_run(us[lo:hi], zs[lo:hi])
            b.loop_run(us[lo:hi], zs[lo:hi])
            a.synchronize()
            launches += hi - lo >= 2
            assert a.resident_launches()[0] == launches
            assert a.resident_status()[0] == 0, "a resident launch fell back"
            _same(a, b, f"after {hi} steps")


def test_resident_tiling_switch_same_tile_count(pp2):
    """256 x 2048 runs 256 tiles either way (1 x 2048 whole rows, 2 x 1024 2-D
    tiles): switching the tiling between runs on one context clears the
    exchange rows (their stale granules would carry matching tag bits)."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 256, 2048, 8, 17)
    with a, b:
        us, zs, _ = S.synth_trajectory(grid, 60, seed=4)
        for k, (lo, hi) in enumerate(((0, 7), (7, 20), (20, 33), (33, 60))):
            a.set_tuning(a.TUNE_RESIDENT_TILE_COLS, 1 + k % 2)
            assert a.resident_tiling() == (256, 1 + k % 2, 1 + k % 2)
            a.loop_run(us[lo:hi], zs[lo:hi])
            b.loop_run(us[lo:hi], zs[lo:hi])
            a.synchronize()
            assert a.resident_status()[0] == 0, "a resident launch fell back"
            _same(a, b, f"after {hi} steps")


def test_resident_interleaved_with_other_ops(pp2):
    """Single loop steps, belief-only updates, sweeps and a belief_set between
    resident runs: the context's pipeline state (pending masses, block phase,
    ping-pong parities) stays consistent."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 1024, 1024, 8, 11)
    with a, b:
        us, zs, _ = S.synth_trajectory(grid, 40, seed=9)
        for c in (a, b):
            c.loop_run(us[:7], zs[:7])
            c.loop_step(int(us[7]), int(zs[7]))
            c.loop_run(us[8:12], zs[8:12])
            c.belief_update(int(us[12]), int(zs[12]))
            c.loop_run(us[13:20], zs[13:20])
            c.mdp_sweep(3)
            c.loop_run(us[20:30], zs[20:30])
        assert a.resident_launches()[0] == 4 and b.resident_launches()[0] == 0
        _same(a, b, "after mixed ops")
        b0 = S.uniform_belief(grid)
        for c in (a, b):
            c.belief_set(b0)
            c.loop_run(us[30:40], zs[30:40])
        _same(a, b, "after belief_set")


def test_resident_multi_launch(pp2):
    """A run longer than one launch (2048 steps): three launches, the epoch
    counters carried over, equal to 4100 single-step launches."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 256, 256, 8, 3)
    with a, b:
        us, zs, _ = S.synth_trajectory(grid, 4100, seed=2)
        a.loop_run(us, zs)
        b.loop_run(us, zs)
        a.synchronize()
        assert a.resident_launches()[0] == 3
        _same(a, b, "after 4100 steps")
        a.loop_run(us[:33], zs[:33])
        b.loop_run(us[:33], zs[:33])
        _same(a, b, "after a further 33 steps")


def test_resident_matches_oracle_1024(pp2, oracle):
    """The 1024^2 bench grid: 16 resident steps against the oracle's
    fp64-normalised loop (J/A bit-exact, belief rel 1e-5 above a 1e-30 floor:
    cells the FTZ build drops may keep ~1e-36-scale values here)."""
    from path_planning_2d_amd import synthetic as S
    O = oracle
    H = W = 1024
    grid = S.synth_grid(H, W, H)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 16, seed=42)
    T, L, R = O.model_pomdp(grid, goal)
    _, C = O.model_mdp(grid, goal)
    bo = S.uniform_belief(grid)
    J = np.zeros(H * W, np.float32)
    for k in range(16):
        bo = O.belief_step(H, W, T, L, bo, us[k], zs[k], mode="f64")
        J, A = O.mdp_sweep(H, W, GAMMA, T, C, J)
    with pp2.GridContext(grid, goal, gamma=float(GAMMA)) as c:
        c.model_generate()
        c.belief_set(S.uniform_belief(grid))
        c.mdp_reset()
        assert c.loop_steps_per_launch() == RESIDENT_STEPS
        c.loop_run(us, zs)
        c.synchronize()
        assert c.resident_launches()[0] == 1
        Jd, Ad = c.mdp_get()
        bd = c.belief_get()
    np.testing.assert_array_equal(Jd.reshape(-1), J.reshape(-1))
    np.testing.assert_array_equal(Ad.reshape(-1), A.reshape(-1))
    bo = np.asarray(bo, np.float32).reshape(-1)
    bd = bd.reshape(-1)
    big = np.abs(bo) > 1e-30
    np.testing.assert_allclose(bd[big], bo[big], rtol=1e-5, atol=0)


@pytest.mark.parametrize("max_sweeps", [0, 150, 300])
@pytest.mark.parametrize("H,W", [(1024, 1024), (512, 512), (700, 768)])
def test_resident_mdp_solve_equals_per_sweep(pp2, H, W, max_sweeps):
    """pp2_mdp_solve as resident sweeps (k_sweep_resident: blocks of 100,
    the convergence decision in-kernel) equals the launch-per-sweep driver:
    same sweep count, same final norm, J and A bit for bit."""
    grid, a, b = _pair(pp2, H, W, 8, H + 3 * W)
    with a, b:
        ra = a.mdp_solve(max_sweeps)
        rb = b.mdp_solve(max_sweeps)
        assert a.resident_launches()[1] >= 1 and b.resident_launches()[1] == 0
        assert ra[0] == rb[0] and ra[0] % 100 == 0, (ra, rb)
        assert np.float32(ra[1]) == np.float32(rb[1]), (ra, rb)
        Ja, Aa = a.mdp_get()
        Jb, Ab = b.mdp_get()
        np.testing.assert_array_equal(Ja.view(np.uint32), Jb.view(np.uint32))
        np.testing.assert_array_equal(Aa, Ab)
        # the loop afterwards starts from the solved values on both paths
        from path_planning_2d_amd import synthetic as S
        us, zs, _ = S.synth_trajectory(grid, 10, seed=1)
        a.loop_run(us, zs)
        b.loop_run(us, zs)
        assert a.resident_launches()[0] == 1
        _same(a, b, "loop after the solve")


@pytest.mark.parametrize("n", [2, 7, 100, 301])
def test_resident_mdp_sweeps_equal_per_sweep(pp2, n):
    """pp2_mdp_sweep(n >= 2) as one resident launch equals n sweep launches
    (J, A bit for bit), also mid-solve and followed by a solve."""
    grid, a, b = _pair(pp2, 1024, 1024, 8, 77)
    with a, b:
        for c in (a, b):
            c.mdp_sweep(n)
        assert a.resident_launches()[1] == 1 and b.resident_launches()[1] == 0
        Ja, Aa = a.mdp_get()
        Jb, Ab = b.mdp_get()
        np.testing.assert_array_equal(Ja.view(np.uint32), Jb.view(np.uint32))
        np.testing.assert_array_equal(Aa, Ab)
        ra, rb = a.mdp_solve(200), b.mdp_solve(200)
        assert ra[0] == rb[0] and np.float32(ra[1]) == np.float32(rb[1])
        np.testing.assert_array_equal(a.mdp_get()[0].view(np.uint32), b.mdp_get()[0].view(np.uint32))


def test_resident_beside_other_work(pp2):
    """Resident runs while another context keeps the GPU busy on its own
    stream (a queue of launch-per-step loop kernels and sweeps): the resident
    workgroups start as CUs free up, on XCDs no placement rule predicts, and
    each edge wave learns its neighbours' XCDs from their granules.  Results
    stay bit-equal to the single-step path."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 1024, 1024, 8, 19)
    g2 = S.synth_grid(512, 512, 512)
    other = pp2.GridContext(g2, S.synth_goal(g2), gamma=float(GAMMA))
    with a, b, other:
        other.model_generate()
        other.set_tuning(other.TUNE_RESIDENT, 0)
        other.belief_set(S.uniform_belief(g2))
        other.mdp_reset()
        us, zs, _ = S.synth_trajectory(grid, 60, seed=4)
        u2, z2, _ = S.synth_trajectory(g2, 400, seed=8)
        for lo, hi in ((0, 20), (20, 41), (41, 60)):
            other.loop_run(u2, z2)  # ~400 queued launches on its stream
            other.mdp_sweep(1)
            a.loop_run(us[lo:hi], zs[lo:hi])
            b.loop_run(us[lo:hi], zs[lo:hi])
        a.synchronize()
        other.synchronize()
        assert a.resident_launches()[0] == 3
        _same(a, b, "beside other work")


# ---------------------------------------------------------------- safety
def test_resident_not_coresident_falls_back_before_launch(pp2):
    """A plan whose tiles cannot all hold a CU at once is never launched:
    with the plans limited to 128 CUs the 1024^2 grid (256 tiles) runs on
    per-step launches -- no resident launch, no fallback, same bits."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 1024, 1024, 8, 23)
    with a, b:
        a.set_tuning(a.TUNE_RESIDENT_CUS, 128)
        assert a.loop_steps_per_launch() != RESIDENT_STEPS
        us, zs, _ = S.synth_trajectory(grid, 12, seed=6)
        a.loop_run(us, zs)
        b.loop_run(us, zs)
        a.mdp_sweep(5)
        b.mdp_sweep(5)
        assert a.resident_launches() == (0, 0)
        assert a.resident_status() == (0, True)
        _same(a, b, "co-residency check")
        a.set_tuning(a.TUNE_RESIDENT_CUS, 0)  # all CUs: resident again
        a.loop_run(us, zs)
        b.loop_run(us, zs)
        assert a.resident_launches()[0] == 1
        _same(a, b, "after lifting the limit")


@pytest.mark.parametrize("what", ["loop", "sweeps", "solve"])
def test_resident_timeout_reruns_from_intact_inputs(pp2, what):
    """A resident launch whose waits time out (one tile held back, as if
    another process kept its CU) writes only the OTHER ping-pong buffers, so
    the next call re-runs it from its intact inputs on per-step launches:
    the readback is correct, the fallback is counted and the context stays
    on per-step launches."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 1024, 1024, 8, 31)
    with a, b:
        us, zs, _ = S.synth_trajectory(grid, 30, seed=12)
        for c in (a, b):
            c.loop_run(us[:10], zs[:10])  # a pending mass and a mid-block phase
        a.synchronize()
        a.set_tuning(a.TUNE_RESIDENT_STALL, 100)
        if what == "loop":
            for c in (a, b):
                c.loop_run(us[10:30], zs[10:30])
        elif what == "sweeps":
            for c in (a, b):
                c.mdp_sweep(7)
        else:
            ra, rb = a.mdp_solve(), b.mdp_solve()
            assert ra == rb, (ra, rb)
        _same(a, b, f"after a timed-out resident {what}")
        assert a.resident_status() == (1, False)
        # still correct afterwards, and the resident kernels can be re-enabled
        a.set_tuning(a.TUNE_RESIDENT_STALL, -1)
        a.set_tuning(a.TUNE_RESIDENT, 1)
        for c in (a, b):
            c.loop_run(us[:9], zs[:9])
        _same(a, b, "after re-enabling")
        assert a.resident_status() == (1, True)


def test_resident_chain_equals_single_steps(pp2):
    """Back-to-back resident runs and sweeps queue behind each other without
    a host sync (more calls than the 16-launch chain, so the queue is verified
    and restarted mid-way) and give the per-step bits."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 512, 512, 5, 77)
    with a, b:
        us, zs, _ = S.synth_trajectory(grid, 120, seed=8)
        for k in range(40):
            for c in (a, b):
                c.loop_run(us[3 * k:3 * k + 3], zs[3 * k:3 * k + 3])
                if k % 7 == 6:
                    c.mdp_sweep(4)
        assert a.resident_launches()[0] == 40
        assert a.resident_status() == (0, True)
        _same(a, b, "after 40 chained runs")


def test_resident_chain_timeout_reruns_every_queued_launch(pp2):
    """A chain whose first launch times out: the launches queued behind it
    see the sticky error word and store nothing, so the next readback re-runs
    the failed launch and every later one from the failed launch's inputs."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 1024, 1024, 8, 57)
    with a, b:
        us, zs, _ = S.synth_trajectory(grid, 40, seed=13)
        for c in (a, b):
            c.loop_run(us[:10], zs[:10])
        a.synchronize()
        a.set_tuning(a.TUNE_RESIDENT_STALL, 100)
        for c in (a, b):
            c.loop_run(us[10:20], zs[10:20])  # times out ...
            c.mdp_sweep(6)                    # ... these queue behind it
            c.loop_run(us[20:40], zs[20:40])
        _same(a, b, "after a timed-out chain")
        assert a.resident_status() == (1, False)


def test_two_resident_contexts_on_separate_streams(pp2):
    """Two contexts whose resident launches are queued on different streams
    at the same time: launches of one process run one at a time per device
    (the runtime's gate), so neither holds part of the CUs waiting for the
    rest -- no timeout, both equal their per-step twins."""
    from path_planning_2d_amd import synthetic as S
    grid, a, b = _pair(pp2, 1024, 1024, 8, 41)
    g2 = S.synth_grid(512, 1024, 5)
    c2 = pp2.GridContext(g2, S.synth_goal(g2), gamma=float(GAMMA))
    d2 = pp2.GridContext(g2, S.synth_goal(g2), gamma=float(GAMMA))
    with a, b, c2, d2:  # (every context runs on a stream of its own)
        d2.set_tuning(d2.TUNE_RESIDENT, 0)
        d2.set_tuning(d2.TUNE_STEP_PAIRS, 0)
        for c in (c2, d2):
            c.model_generate()
            c.belief_set(S.uniform_belief(g2))
            c.mdp_reset()
        us, zs, _ = S.synth_trajectory(grid, 300, seed=3)
        u2, z2, _ = S.synth_trajectory(g2, 300, seed=4)
        for lo, hi in ((0, 100), (100, 300)):
            a.loop_run(us[lo:hi], zs[lo:hi])   # queued on a's stream ...
            c2.loop_run(u2[lo:hi], z2[lo:hi])  # ... and on c2's before a's finishes
            b.loop_run(us[lo:hi], zs[lo:hi])
            d2.loop_run(u2[lo:hi], z2[lo:hi])
        assert a.resident_status() == (0, True) and c2.resident_status() == (0, True)
        assert a.resident_launches()[0] == 2 and c2.resident_launches()[0] == 2
        _same(a, b, "context 1")
        _same(c2, d2, "context 2")
