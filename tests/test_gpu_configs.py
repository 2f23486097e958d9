"""GPU: BASELINE.json's configurations at their full sizes.

configs[2] -- "1024x1024 grid, MDP Bellman backup to convergence": value
iteration with valueIteration's stopping rule (src/mdp/path_planning_2d.cu:
219-263: blocks of 100 sweeps until max|J - J_prev| <= 1e-3 * 5 / (1 - gamma))
on the bench's synthetic 1024^2 grid, coded and dense kernels, against the
oracle's orc_mdp_solve: the same sweep count and final norm, J and A bit for
bit (J compared as bit patterns).
"""
import numpy as np
import pytest

from conftest import GAMMA

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pp2():
    import path_planning_2d_amd as P
    assert P.device_count() >= 1, "no GPU visible"
    return P


@pytest.fixture(scope="module")
def config3(oracle):
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    T, _, _ = oracle.model_pomdp(grid, goal)
    _, Cc = oracle.model_mdp(grid, goal)
    Jo, Ao, n, nrm = oracle.mdp_solve(N, N, GAMMA, T, Cc)
    return grid, goal, Jo, Ao, n, nrm


@pytest.mark.parametrize("coded", [1, 0], ids=["coded", "dense"])
def test_config3_mdp_solve_1024_to_convergence(pp2, config3, coded):
    grid, goal, Jo, Ao, n_o, nrm_o = config3
    assert n_o == 300  # the rule stops after the third block of 100 on this grid
    with pp2.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        ctx.set_tuning(ctx.TUNE_CODED_MODEL, coded)
        assert ctx.model_dict_info()[1] == bool(coded)
        n, nrm = ctx.mdp_solve()
        J, A = ctx.mdp_get()
    assert n == n_o
    assert nrm == nrm_o
    np.testing.assert_array_equal(J.view(np.uint32), Jo.view(np.uint32))
    np.testing.assert_array_equal(A, Ao)
