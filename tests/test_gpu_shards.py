"""GPU: row-sharded execution (pp2_shard_group_*) equals the unsharded grid.

The shard group runs the same per-shard phases as the multi-process RCCL path
(halo rows from the neighbours, local kernels, global belief mass), with
device copies as the transport, so one GPU exercises shard geometry, halo
semantics and mass bookkeeping.  Values and actions are bit-exact (every cell
sees the same neighbour values); the normalised belief differs only by the
association of the mass sum (per-shard sums, then a sum over shards)."""
import numpy as np
import pytest

from conftest import GAMMA, assert_rel_close, golden, golden_map

FTZ_FLOOR = 1e-30  # see the module docstring

pytestmark = pytest.mark.gpu


def run_pair(P, grid, goal, bounds, steps, seed=42):
    from path_planning_2d_amd import synthetic as S
    us, zs, _ = S.synth_trajectory(grid, steps, seed=seed)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.ShardGroup(grid, goal, bounds, gamma=float(GAMMA)) as grp:
        ref.model_generate()
        grp.model_generate()
        ref.belief_set(b0)
        grp.belief_set(b0)
        ref.mdp_reset()
        grp.mdp_reset()
        for k in range(steps):
            ref.loop_step(us[k], zs[k])
            grp.loop_step(us[k], zs[k])
        Jr, Ar = ref.mdp_get()
        Jg, Ag = grp.mdp_get()
        np.testing.assert_array_equal(Jg, Jr)
        np.testing.assert_array_equal(Ag, Ar)
        assert_rel_close(grp.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                         msg="sharded belief")
        # belief-only and sweep-only drivers
        ref.belief_update(us[0], zs[0])
        grp.belief_update(us[0], zs[0])
        assert_rel_close(grp.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                         msg="sharded belief update")
        ref.mdp_sweep(3)
        grp.mdp_sweep(3)
        np.testing.assert_array_equal(grp.mdp_get()[0], ref.mdp_get()[0])


@pytest.mark.parametrize("bounds", [(0, 3, 10), (0, 1, 2, 9, 10), (0, 5, 10)])
def test_shards_small_map(bounds):
    import path_planning_2d_amd as P
    name = "map_10x10"
    m = golden("model", name)
    run_pair(P, golden_map(name), tuple(m["goal"]), bounds, steps=12)


def test_shards_sparse_map_uneven():
    import path_planning_2d_amd as P
    name = "sparse_map_100x40"
    m = golden("model", name)
    run_pair(P, golden_map(name), tuple(m["goal"]), (0, 7, 20, 21, 40), steps=10)


def test_config4_2048_eight_row_shards():
    """BASELINE configs[3] decomposition: 2048x2048 grid, 8 row shards of
    256 rows (here all on one device), belief stencil + Bellman loop."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 2048
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    run_pair(P, grid, goal, tuple(range(0, N + 1, N // 8)), steps=4)


@pytest.mark.parametrize("resident", [0, 1])
def test_config4_2048_eight_row_shards_vs_oracle(oracle, resident):
    """The same 8-shard group against the CPU oracle itself (not the
    unsharded HIP context): the reference loop -- cudaBayesBeliefUpdate +
    renormalisation (point_based_value_iteration_cuda.cu:88-133,
    search_tree_cuda.cu:225-229), then cudaOneStepValueIteration
    (mdp/path_planning_2d_cuda.cu:215-264) -- 8 steps on the 2048^2 grid.
    Values and actions bit for bit, the belief rel 1e-5 above the FTZ floor
    against the fp64-normalised oracle (the reference's own sequential fp32
    mass sum errs by ~1e-4 over 4 M cells, as a fp32 row-partitioned sum
    does: measured 1.2e-4 against orc_loop_run_mt).  resident 1: the shards
    run the resident kernel on their 384-row views (the 8-GPU job's default
    path); 0: step pairs / single steps."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    O = oracle
    N = 2048
    steps = 8
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, steps, seed=42)
    T, L, _ = O.model_pomdp(grid, goal)
    _, Cc = O.model_mdp(grid, goal)
    b = S.uniform_belief(grid)
    J = np.zeros(N * N, np.float32)
    for k in range(steps):
        b = O.belief_step(N, N, T, L, b, us[k], zs[k], mode="f64")
        J, A = O.mdp_sweep(N, N, GAMMA, T, Cc, J)
    b = np.asarray(b, np.float32).reshape(-1)
    J = np.asarray(J, np.float32).reshape(-1)
    A = np.asarray(A).reshape(-1)
    with P.ShardGroup(grid, goal, tuple(range(0, N + 1, N // 8)), gamma=float(GAMMA)) as grp:
        grp.model_generate()
        grp.set_tuning(P.GridContext.TUNE_RESIDENT, resident)
        grp.belief_set(S.uniform_belief(grid))
        grp.mdp_reset()
        grp.loop_run(us, zs)
        if resident:
            assert grp.shards[0].resident_launches()[0] >= 1
        Jg, Ag = grp.mdp_get()
        bg = grp.belief_get()
    np.testing.assert_array_equal(Jg.reshape(-1).view(np.uint32), J.view(np.uint32))
    np.testing.assert_array_equal(Ag.reshape(-1), A)
    assert_rel_close(bg.reshape(-1), b, rel=1e-5, abs_floor=FTZ_FLOOR,
                     msg="8-shard belief vs the oracle")


def test_config4_shard_group_memory():
    """The 2048^2 grid in 8 row shards allocates <= 10 % above the unsharded
    context (round-4 ADVICE): a shard's deep halo (kShardHalo rows per side,
    for the resident shard runs) lives only in the per-cell b / J planes and
    the code plane; the dense model and FIB planes keep kDenseHalo rows, and
    a shard holds only its window of the map.  Counted by the
    library (every grid-sized buffer), and the group still equals the
    unsharded grid after a few loop steps."""
    import ctypes
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    f = P._lib.load().pp2_debug_context_bytes
    f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]

    def held(ctx):
        v = ctypes.c_ulonglong()
        assert f(ctx.handle, ctypes.byref(v)) == 0
        return v.value

    N = 2048
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.ShardGroup(grid, goal, tuple(range(0, N + 1, N // 8)), gamma=float(GAMMA)) as grp:
        ref.model_generate()
        grp.model_generate()
        used_ref = held(ref)
        used_grp = sum(held(s) for s in grp.shards)
        assert used_ref > 2_000_000_000  # the dense planes are there
        print(f"unsharded {used_ref / 1e6:.1f} MB, 8 shards {used_grp / 1e6:.1f} MB")
        assert used_grp <= 1.10 * used_ref, (used_grp, used_ref)
        us, zs, _ = S.synth_trajectory(grid, 3, seed=9)
        b0 = S.uniform_belief(grid)
        for c in (ref, grp):
            c.belief_set(b0)
            c.mdp_reset()
            for k in range(3):
                c.loop_step(us[k], zs[k])
        Jr, Ar = ref.mdp_get()
        Jg, Ag = grp.mdp_get()
        np.testing.assert_array_equal(Jg, Jr)
        np.testing.assert_array_equal(Ag, Ar)


def test_shards_mdp_solve_and_fib():
    import path_planning_2d_amd as P
    name = "sparse_map_100x40"
    m = golden("model", name)
    g = golden("mdp", name)
    grid = golden_map(name)
    with P.ShardGroup(grid, tuple(m["goal"]), (0, 13, 27, 40), gamma=float(GAMMA)) as grp:
        grp.model_generate()
        sweeps, _ = grp.mdp_solve()
        J, A = grp.mdp_get()
        assert sweeps == int(g["sweeps"])
        np.testing.assert_array_equal(J, g["J"])
        np.testing.assert_array_equal(A, g["A"])
        grp.fib_reset()
        grp.fib_sweep(4)
        got = grp.fib_get()
    with P.GridContext(grid, tuple(m["goal"]), gamma=float(GAMMA)) as ref:
        ref.model_generate()
        ref.fib_sweep(4)
        np.testing.assert_array_equal(got, ref.fib_get())


@pytest.mark.parametrize("depth", [1, 3, 8])
def test_shards_halo_depths(depth):
    """Loop steps with halo rows exchanged `depth` deep every `depth` steps
    (extended-domain views in between) and the lagged belief normalisation,
    interleaved with belief-only and sweep-only steps that restart the
    pipeline, against the unsharded grid."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    name = "sparse_map_100x40"
    grid = golden_map(name)
    goal = tuple(golden("model", name)["goal"])
    us, zs, _ = S.synth_trajectory(grid, 40, seed=9)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.ShardGroup(grid, goal, (0, 13, 27, 40), gamma=float(GAMMA)) as grp:
        ref.model_generate()
        grp.model_generate()
        grp.set_halo_depth(depth)
        for c in (ref, grp):
            c.belief_set(b0)
            c.mdp_reset()
        k = 0
        for phase in (17, 5, 11):
            for _ in range(phase):
                ref.loop_step(us[k], zs[k])
                grp.loop_step(us[k], zs[k])
                k += 1
            np.testing.assert_array_equal(grp.mdp_get()[0], ref.mdp_get()[0])
            np.testing.assert_array_equal(grp.mdp_get()[1], ref.mdp_get()[1])
            assert_rel_close(grp.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                             msg=f"belief after {k} steps, depth {depth}")
            ref.belief_update(us[k], zs[k])
            grp.belief_update(us[k], zs[k])
            k += 1
            ref.mdp_sweep(2)
            grp.mdp_sweep(2)


def test_halo_depth_bounds():
    import path_planning_2d_amd as P
    grid = golden_map("map_10x10")
    with P.ShardGroup(grid, (8, 7), (0, 3, 10)) as grp:
        with pytest.raises(P.Pp2Error):
            grp.set_halo_depth(4)  # the 3-row shard cannot feed 4 halo rows
        grp.set_halo_depth(3)
    with P.GridContext(grid, (8, 7)) as ctx:
        with pytest.raises(P.Pp2Error):
            ctx.set_tuning(ctx.TUNE_HALO_DEPTH, 2)  # unsharded: depth 1 only


def test_grouped_context_rejects_per_context_stepping():
    import path_planning_2d_amd as P
    grid = golden_map("map_10x10")
    with P.ShardGroup(grid, (8, 7), (0, 5, 10)) as grp:
        grp.model_generate()
        with pytest.raises(P.Pp2Error):
            grp.shards[0].loop_step(0, 0)


def test_rccl_single_rank_pipeline():
    """The RCCL shard path on one GPU: a full-grid shard context with a
    1-rank communicator runs the sharded loop pipeline -- comm stream, events,
    asynchronous all-reduce of the mass, lagged normalisation, 8-deep
    extended-domain views (neighbour transfers aside, which need 2 GPUs)."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    name = "sparse_map_100x40"
    grid = golden_map(name)
    goal = tuple(golden("model", name)["goal"])
    H = grid.shape[0]
    us, zs, _ = S.synth_trajectory(grid, 40, seed=5)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.GridContext(grid, goal, gamma=float(GAMMA), rows=(0, H)) as sh:
        sh.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
        for c in (ref, sh):
            c.model_generate()
            c.belief_set(b0)
            c.mdp_reset()
        k = 0
        for phase in (13, 8):
            for _ in range(phase):
                ref.loop_step(us[k], zs[k])
                sh.loop_step(us[k], zs[k])
                k += 1
            np.testing.assert_array_equal(sh.mdp_get()[0], ref.mdp_get()[0])
            np.testing.assert_array_equal(sh.mdp_get()[1], ref.mdp_get()[1])
            assert_rel_close(sh.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                             msg=f"belief after {k} steps")
            ref.belief_update(us[k], zs[k])
            sh.belief_update(us[k], zs[k])
            k += 1
            ref.mdp_sweep(3)
            sh.mdp_sweep(3)
        assert ref.mdp_solve() == sh.mdp_solve()
        np.testing.assert_array_equal(sh.mdp_get()[0], ref.mdp_get()[0])


@pytest.mark.parametrize("bounds,depth", [((0, 512, 1024), 8), ((0, 300, 777, 1024), 8),
                                          ((0, 512, 1024), 3), ((0, 400, 1024), 5)])
def test_shard_group_step_pairs(bounds, depth):
    """Two loop steps of a halo block per launch on row shards
    (k_loop_pair_coded on step 2's extended view, step 1 one row deeper from
    the halo rows of the neighbour shards; pp2_shard_group_loop_run), forced
    with PP2_TUNE_STEP_PAIRS = 2 on these small shards: values and actions
    bit-exact with the unsharded grid, beliefs rel 1e-5, across block
    boundaries, odd chunks and halo depths whose blocks end on a single step."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 23, seed=9)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.ShardGroup(grid, goal, bounds, gamma=float(GAMMA)) as grp:
        ref.model_generate()
        grp.model_generate()
        grp.set_halo_depth(depth)
        grp.set_tuning(P.GridContext.TUNE_RESIDENT, 0)  # (these shards fit resident views)
        grp.set_tuning(P.GridContext.TUNE_STEP_PAIRS, 2)
        assert grp.loop_steps_per_launch() == [2] * (len(bounds) - 1)
        for c in (ref, grp):
            c.belief_set(b0)
            c.mdp_reset()
        for lo, hi in ((0, 5), (5, 6), (6, 23)):
            ref.loop_run(us[lo:hi], zs[lo:hi])
            grp.loop_run(us[lo:hi], zs[lo:hi])
            Jr, Ar = ref.mdp_get()
            Jg, Ag = grp.mdp_get()
            np.testing.assert_array_equal(Jg.view(np.uint32), Jr.view(np.uint32),
                                          err_msg=f"J after {hi} steps")
            np.testing.assert_array_equal(Ag, Ar, err_msg=f"A after {hi} steps")
            assert_rel_close(grp.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                             msg=f"belief after {hi} steps")


def test_rccl_single_rank_step_pairs():
    """The RCCL shard path with step pairs at the bench size (1024^2, a tile
    per CU): a full-grid shard with a 1-rank communicator runs pp2_loop_run in
    pair launches over its 8-deep halo blocks; equals the unsharded grid."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 21, seed=4)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.GridContext(grid, goal, gamma=float(GAMMA), rows=(0, N)) as sh:
        sh.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
        for c in (ref, sh):
            c.model_generate()
            c.belief_set(b0)
            c.mdp_reset()
        assert sh.loop_steps_per_launch() == 2
        for lo, hi in ((0, 7), (7, 21)):
            ref.loop_run(us[lo:hi], zs[lo:hi])
            sh.loop_run(us[lo:hi], zs[lo:hi])
            np.testing.assert_array_equal(sh.mdp_get()[0].view(np.uint32),
                                          ref.mdp_get()[0].view(np.uint32))
            np.testing.assert_array_equal(sh.mdp_get()[1], ref.mdp_get()[1])
            assert_rel_close(sh.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                             msg=f"belief after {hi} steps")


# ------------------------------------------------- row shards on the resident loop
def _resident_shard_run(P, grid, goal, bounds, chunks, halo=0, mixed=True, tiling=0, lag=0):
    """pp2_shard_group_loop_run on the resident kernel (one launch per halo
    block of up to e steps on the view of the owned rows plus e halo rows per
    side, power-of-two rescaling inside, rebased at each exchange) against
    the unsharded grid: values and actions bit-exact, beliefs rel 1e-5."""
    from path_planning_2d_amd import synthetic as S
    steps = chunks[-1][1]
    us, zs, _ = S.synth_trajectory(grid, steps + 1, seed=21)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.ShardGroup(grid, goal, bounds, gamma=float(GAMMA)) as grp:
        ref.model_generate()
        grp.model_generate()
        if halo:
            grp.set_tuning(P.GridContext.TUNE_RESIDENT_HALO, halo)
        if tiling:
            grp.set_tuning(P.GridContext.TUNE_RESIDENT_TILE_COLS, tiling)
        if lag:
            grp.set_tuning(P.GridContext.TUNE_SHARD_LAG, lag)
        # each shard's own depth; the group runs the smallest (every shard's
        # view must hold it)
        e_all = grp.loop_steps_per_launch()
        e = min(e_all)
        assert e >= 2, e_all
        for c in (ref, grp):
            c.belief_set(b0)
            c.mdp_reset()
        launches = 0
        for lo, hi in chunks:
            ref.loop_run(us[lo:hi], zs[lo:hi])
            grp.loop_run(us[lo:hi], zs[lo:hi])
            launches += -(-(hi - lo) // e)
            assert grp.shards[0].resident_launches()[0] == launches
            Jr, Ar = ref.mdp_get()
            Jg, Ag = grp.mdp_get()
            np.testing.assert_array_equal(Jg.view(np.uint32), Jr.view(np.uint32),
                                          err_msg=f"J after {hi} steps")
            np.testing.assert_array_equal(Ag, Ar, err_msg=f"A after {hi} steps")
            assert_rel_close(grp.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                             msg=f"belief after {hi} steps")
        if mixed:  # per-step drivers after resident runs: the state is theirs
            ref.belief_update(us[steps], zs[steps])
            grp.belief_update(us[steps], zs[steps])
            assert_rel_close(grp.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                             msg="belief update after resident runs")
            ref.mdp_sweep(2)
            grp.mdp_sweep(2)
            np.testing.assert_array_equal(grp.mdp_get()[0], ref.mdp_get()[0])
            ref.loop_run(us[:3], zs[:3])
            grp.loop_run(us[:3], zs[:3])
            np.testing.assert_array_equal(grp.mdp_get()[1], ref.mdp_get()[1])
            assert_rel_close(grp.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                             msg="loop after the per-step drivers")
        return e


@pytest.mark.parametrize("tiling,lag", [(0, 0), (3, 0), (0, 1), (3, 1)])
def test_shard_group_resident_config4(tiling, lag):
    """BASELINE configs[3]'s per-rank geometry: the 2048^2 grid in 8 row shards
    of 256 rows (one device here), each shard's run on the resident kernel
    (view 256 + 2e rows, e = 64: 256 tiles of 3 x 1024 cells -- the halved
    depth's tiles hold fewer rows than e = 128's 4 x 1024 --, or -- tiling 3
    -- e = 128 and 256 transposed tiles of 8 grid columns x the 512 view
    rows), with block starts waited for or lagged (PP2_TUNE_SHARD_LAG)."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 2048
    grid = S.synth_grid(N, N, N)
    e = _resident_shard_run(P, grid, S.synth_goal(grid), tuple(range(0, N + 1, N // 8)),
                            ((0, 30), (30, 41)), mixed=tiling == 3, tiling=tiling, lag=lag)
    assert e == (128 if tiling == 3 else 64)


@pytest.mark.parametrize("bounds,halo,lag,e_want", [((0, 256, 512), 0, 0, 128), ((0, 200, 512), 6, 0, 6),
                                                    ((0, 128, 300, 512), 9, 0, 9),
                                                    ((0, 200, 512), 0, 1, 64)])
def test_shard_group_resident_blocks(bounds, halo, lag, e_want):
    """Uneven shards, several halo blocks per call (e = 6, 9: in-kernel
    power-of-two block starts every 8 steps, rebases at every exchange),
    calls ending mid-block, then per-step drivers on the same state.  Without
    a requested halo the shards agree on the deepest e, halved while that
    gives tiles of fewer rows: 128 for the 256-row shards (2-row tiles
    either way), 64 for the 312-row one (3 -> 2 rows per tile)."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(512, 1024, 7)
    e = _resident_shard_run(P, grid, S.synth_goal(grid), bounds,
                            ((0, 2), (2, 19), (19, 40)), halo=halo, lag=lag)
    assert e == e_want


def test_shard_group_resident_weak_scaling_shards():
    """The bench's weak-scaling decomposition at N >= 2: 896-row shards of a
    1024-wide grid, whose views with e = 64 halo rows per side are 1024 rows
    (one 4-row tile per CU), resident in the shard group; J/A bit-exact and
    beliefs rel 1e-5 against the unsharded grid."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(1792, 1024, 1792)
    goal = S.synth_goal(grid)
    _resident_shard_run(P, grid, goal, [0, 896, 1792], [(0, 70), (70, 200)])


def test_rccl_single_rank_resident_896x1024():
    """The RCCL path of an 896 x 1024 shard (the weak-scaling bench's rank
    share) with a 1-rank communicator: e = 64, so 200 steps take 4 launches,
    and the shard equals the unsharded grid."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(896, 1024, 896)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 200, seed=9)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.GridContext(grid, goal, gamma=float(GAMMA), rows=(0, 896)) as sh:
        sh.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
        for c in (ref, sh):
            c.model_generate()
            c.belief_set(b0)
            c.mdp_reset()
        assert sh.loop_steps_per_launch() == 64
        ref.loop_run(us, zs)
        sh.loop_run(us, zs)
        np.testing.assert_array_equal(sh.mdp_get()[0].view(np.uint32),
                                      ref.mdp_get()[0].view(np.uint32))
        np.testing.assert_array_equal(sh.mdp_get()[1], ref.mdp_get()[1])
        assert_rel_close(sh.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                         msg="belief after 200 steps")
        assert sh.resident_launches()[0] == 4


def test_comm_round_timing_single_rank():
    """PP2_TUNE_COMM_TIMING / pp2_comm_rounds on the config-4 rank share with
    a 1-rank communicator: one timed round per resident block (its halo
    exchange, with the {mass, shift, lost} records after the first) plus the
    closing all-reduce; durations positive; the record clears on read; no
    events without the knob; results unchanged."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(256, 2048, 256)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 150, seed=8)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA), rows=(0, 256)) as sh, \
            P.GridContext(grid, goal, gamma=float(GAMMA), rows=(0, 256)) as sh2:
        for c in (sh, sh2):
            c.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
            c.model_generate()
            c.belief_set(b0)
            c.mdp_reset()
        e = sh.loop_steps_per_launch()
        sh.loop_run(us[:10], zs[:10])  # (agreement on e happens here)
        sh2.loop_run(us[:10], zs[:10])
        sh.set_tuning(sh.TUNE_COMM_TIMING, 1)
        sh.loop_run(us[10:], zs[10:])
        sh2.loop_run(us[10:], zs[10:])
        t, untimed = sh.comm_rounds()
        assert untimed == 0
        nblk = -(-140 // e)
        assert nblk + 1 <= t.size <= nblk + 2, (t, e)
        assert (t > 0).all() and (t < 1e5).all(), t
        assert sh.comm_rounds()[0].size == 0  # cleared
        sh.set_tuning(sh.TUNE_COMM_TIMING, 0)
        sh.loop_run(us[:5], zs[:5])
        sh2.loop_run(us[:5], zs[:5])
        assert sh.comm_rounds()[0].size == 0
        np.testing.assert_array_equal(sh.mdp_get()[0].view(np.uint32),
                                      sh2.mdp_get()[0].view(np.uint32))
        np.testing.assert_array_equal(sh.belief_get(), sh2.belief_get())


@pytest.mark.parametrize("tiling", [0, 3])
def test_rccl_single_rank_resident_256x2048(tiling):
    """The RCCL path of a 256 x 2048 shard -- the per-rank share of the
    2048^2 grid at 8 ranks -- with a 1-rank communicator: pp2_loop_run takes
    the resident shard path (e = 64: 384-row view; transposed tiles: e = 128,
    512-row view; exchanges with the {mass, shift, lost} records, rebase) and
    equals the unsharded grid."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    grid = S.synth_grid(256, 2048, 256)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 300, seed=8)
    b0 = S.uniform_belief(grid)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ref, \
            P.GridContext(grid, goal, gamma=float(GAMMA), rows=(0, 256)) as sh:
        sh.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
        if tiling:
            sh.set_tuning(sh.TUNE_RESIDENT_TILE_COLS, tiling)
        for c in (ref, sh):
            c.model_generate()
            c.belief_set(b0)
            c.mdp_reset()
        assert sh.loop_steps_per_launch() == (128 if tiling == 3 else 64)
        # the 384-row view runs 2-D tiles (3 x 1024, two tile columns), the
        # 512-row one transposed tiles (8 grid columns x 512 view rows)
        assert sh.resident_tiling() == ((256, 8, 3) if tiling == 3 else (256, 3, 2))
        for lo, hi in ((0, 17), (17, 300)):
            ref.loop_run(us[lo:hi], zs[lo:hi])
            sh.loop_run(us[lo:hi], zs[lo:hi])
            np.testing.assert_array_equal(sh.mdp_get()[0].view(np.uint32),
                                          ref.mdp_get()[0].view(np.uint32))
            np.testing.assert_array_equal(sh.mdp_get()[1], ref.mdp_get()[1])
            assert_rel_close(sh.belief_get(), ref.belief_get(), rel=1e-5, abs_floor=FTZ_FLOOR,
                             msg=f"belief after {hi} steps")
        e = sh.loop_steps_per_launch()
        assert sh.resident_launches()[0] == -(-17 // e) + -(-283 // e)  # 1 + 3, or 1 + 5 at e = 64
        assert abs(float(sh.belief_get().astype(np.float64).sum()) - 1.0) < 1e-4
