"""GPU: the ROS node adapters RUN -- the catkin drop-in's logic, driven as the
reference's node mains and dummy simulator drive the nodes.

ros/src/pomdp/path_planning_2d_pp2.cpp and ros/src/mdp/path_planning_2d_pp2.cpp
(replacing src/pomdp/path_planning_2d.cu:80-282 and src/mdp/path_planning_2d.cu:
72-189) are built against the stand-in roscpp / OpenCV headers of
tests/ros_stubs/ (an in-process transport: parameters, a capturing ~control
publisher, a callable ~belief subscriber and services) plus the real
include/pp2.h, linked to libpp2_hip.so, and run by tests/ros_stubs/run_node.cpp:
construct with the private NodeHandle, initialize(), one beliefCallback per
message.

POMDP node, launch defaults (pomdp_path_planning_2d.launch: sparse_map_100x40,
goal (95, 34), gamma 0.95, max_search_tree_depth 50, max_online_iteration 15):
initialize() solves the model, FIB and PBVI (S = 500) on the GPU; the tree's
leaf lower bounds are the PBVI alphas and its rand() stream continues after
PBVI's draws.  The published actions must equal, bit for bit, those of the
oracle's reference-arithmetic QV-tree (oracle/pp2_oracle_tree.c, sequential
fp32 sums) over the same alphas and messages.  Then ~save_data writes the
reference's text files and a second node started with read_data_from_file
loads them; its actions must equal the oracle tree's over the RELOADED data
with a fresh rand() stream (the reference's own behaviour: the text format
keeps 8 decimals and no belief set is generated, so the first run's actions
are not the criterion).

MDP node (mdp_path_planning_2d.launch): the action published for a one-hot
belief at every cell must equal orc_mdp_solve's action table there, and the
two latched markers carry one point per cell.
"""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from conftest import GAMMA, ROOT, golden, golden_map

pytestmark = pytest.mark.gpu

STUBS = os.path.join(ROOT, "tests", "ros_stubs")
PKG = os.path.join(ROOT, "path_planning_2d_amd")


def build_node(node, out_dir):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = os.path.join(out_dir, f"run_{node}")
    cmd = [cxx, "-std=c++14", "-O1", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
           "-DPP2_NODE_POMDP" if node == "pomdp" else "-DPP2_NODE_MDP",
           "-I", os.path.join(ROOT, "ros", "include"), "-I", STUBS,
           "-I", os.path.join(STUBS, "path_planning_2d"), "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "ros", "src", node, "path_planning_2d_pp2.cpp"),
           os.path.join(STUBS, "run_node.cpp"), "-L", PKG, "-lpp2_hip",
           f"-Wl,-rpath,{PKG}", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def write_pgm(path, grid):
    """The map image: occupied cells black (0), free cells white (255)."""
    H, W = grid.shape
    img = np.where(grid > 0, 0, 255).astype(np.uint8)
    with open(path, "wb") as f:
        f.write(f"P5 {W} {H} 255\n".encode())
        f.write(img.tobytes())


def write_params(path, params):
    with open(path, "w") as f:
        for k, v in params.items():
            f.write(f"{k} {v}\n")


def measurement_bits(z):
    return [(z >> k) & 1 for k in range(4)]  # z = m3 << 3 | m2 << 2 | m1 << 1 | m0


def write_messages(path, msgs, n, kind):
    with open(path, "wb") as f:
        f.write(struct.pack("<iii", len(msgs), kind, n))
        for action, z, payload in msgs:
            f.write(struct.pack("<B4B", action, *measurement_bits(z)))
            if kind == 0:
                f.write(np.ascontiguousarray(payload, np.float32).tobytes())
            else:
                f.write(struct.pack("<i", int(payload)))


def run_node(exe, cwd, params, msgs, n, kind, save=False):
    pf, mf, of = (os.path.join(cwd, x) for x in ("params.txt", "messages.bin", "out.txt"))
    write_params(pf, params)
    write_messages(mf, msgs, n, kind)
    cmd = [exe, pf, mf, of] + (["save"] if save else [])
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}"
    lines = open(of).read().split("\n")
    actions = [int(x) for x in lines if x and x[0].isdigit()]
    extra = {ln.split()[0]: [int(t) for t in ln.split()[1:]] for ln in lines
             if ln and not ln[0].isdigit()}
    return actions, extra


def oracle_actions(oracle, grid, T, L, R, alphas, pal, pact, skip, b0, zs, depth, iters):
    """The reference-arithmetic tree over the messages the node receives:
    message 0 = (0, 0, b0), message k = (its previous action, zs[k-1])."""
    rpl = oracle.Planner(grid, T, L, R, alphas, max_depth=depth, max_iter=iters)
    rpl.set_pbvi(pal, pact)
    rpl.skip_rand(skip)
    acts = []
    msgs = [(0, 0, b0)]
    a, _ = rpl.step(0, 0, b0)
    acts.append(a)
    for z in zs:
        msgs.append((a, int(z), b0))  # the simulator's belief: used only by the first step
        a, _ = rpl.step(a, int(z))
        acts.append(a)
    rpl.close()
    return acts, msgs


def test_pomdp_node_publishes_reference_actions_and_reloads(oracle, tmp_path):
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    name, goal, depth, iters, steps = "sparse_map_100x40", (95, 34), 50, 15, 6
    grid = golden_map(name)
    H, W = grid.shape
    exe = build_node("pomdp", str(tmp_path))
    write_pgm(str(tmp_path / "map.pgm"), grid)
    params = {"map_path": str(tmp_path / "map.pgm"), "goal_x": goal[0], "goal_y": goal[1],
              "discount_factor": 0.95, "map_resolution": 0.2, "read_data_from_file": "false",
              "max_search_tree_depth": depth, "max_online_iteration": iters}
    b0 = S.uniform_belief(grid)
    _, zs, _ = S.synth_trajectory(grid, steps, seed=5)
    # the node's offline solution, formed the same way (bit-exact with the
    # oracle's: tests/test_gpu_pbvi.py, test_gpu_parity.py)
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_generate()
        T, L, R, _ = ctx.model_download()
        ctx.fib_solve()
        alphas = ctx.fib_get()
        draws = ctx.pbvi_solve(b0, 500)
        pal, pact = ctx.pbvi_get()
    m = golden("model", name)
    assert np.array_equal(T, m["T"]) and np.array_equal(L, m["L"]) and np.array_equal(R, m["R"])
    want, msgs = oracle_actions(oracle, grid, T, L, R, alphas, pal, pact, draws, b0, zs, depth,
                                iters)
    got, extra = run_node(exe, str(tmp_path), params, msgs, H * W, 0, save=True)
    assert got == want, f"published {got}, reference tree {want}"
    assert extra["save_data"] == [1]
    for f in ("model_data_trans_prob", "model_data_meas_prob", "model_data_stage_reward",
              "fib_alphas", "fib_actions", "pbvi_alphas", "pbvi_actions"):
        assert (tmp_path / f).exists(), f
    # restart from the saved files: the reloaded (8-decimal) data, no belief-set draws
    with P.GridContext(grid, goal, gamma=float(GAMMA)) as ctx:
        ctx.model_load(str(tmp_path))
        T2, L2, R2, _ = ctx.model_download()
        ctx.fib_load(str(tmp_path))
        alphas2 = ctx.fib_get()
        ctx.pbvi_load(str(tmp_path), 500)
        pal2, pact2 = ctx.pbvi_get()
    want2, msgs2 = oracle_actions(oracle, grid, T2, L2, R2, alphas2, pal2, pact2, 0, b0, zs,
                                  depth, iters)
    params["read_data_from_file"] = "true"
    got2, _ = run_node(exe, str(tmp_path), params, msgs2, H * W, 0)
    assert got2 == want2, f"reloaded node published {got2}, reference tree {want2}"


def test_mdp_node_publishes_the_value_iteration_policy(oracle, tmp_path):
    name, goal = "sparse_map_100x40", (95, 34)
    grid = golden_map(name)
    H, W = grid.shape
    exe = build_node("mdp", str(tmp_path))
    write_pgm(str(tmp_path / "map.pgm"), grid)
    params = {"map_path": str(tmp_path / "map.pgm"), "goal_x": goal[0], "goal_y": goal[1],
              "discount_factor": 0.95, "map_resolution": 0.2}
    msgs = [(4, 0, cell) for cell in range(H * W)]
    got, extra = run_node(exe, str(tmp_path), params, msgs, H * W, 1)
    T, Cc = oracle.model_mdp(grid, goal)
    _, A, _, _ = oracle.mdp_solve(H, W, GAMMA, T, Cc)
    assert np.array_equal(np.array(got, np.uint8), A), \
        f"{int((np.array(got) != A).sum())} cells publish another action"
    assert extra["markers"] == [1, 1, H * W]
