#!/usr/bin/env python3
"""Benchmark of the north-star loop: belief update + MDP Bellman sweep.

One *step* = one Bayesian belief update (9-neighbour transition stencil,
observation likelihood, renormalisation) with the next (u, z) of a seeded
trajectory, plus one MDP Bellman sweep (per-cell min over 9 action values),
on a 1024 x 1024 synthetic grid per GPU (BASELINE.json configs[2]; the metric
"grid cells/sec for belief-update+Bellman loop, 1024x1024").  Inputs are
resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 1024] [--grid G]

For N > 1 launch with torch.distributed.run, or run it directly: without a
launcher environment `bench.py --gpus N` starts `torch.distributed.run
--nproc-per-node N bench.py ...` as a child process (the parent imports no
torch and touches no GPU) and exits with its code.  Default (weak scaling): rank r
owns rows [r*R, (r+1)*R) of an (N*R) x S grid, S = --size = 1024 and R =
--shard-rows = 896: a rank's view (its rows plus e = 64 halo rows per side)
is then 1024 x 1024, one 4-row tile per CU, so every rank runs the
tile-resident loop; per-GPU work is fixed for N >= 2 (7/8 of
N = 1's grid).  Each resident launch of up to e steps follows one RCCL
exchange of e halo rows of belief and values and a {mass, shift} all-reduce
(768 / 896 / 960 rows measured 0.61-0.67 / 0.63-0.74 / 0.56-0.71 projected
efficiency, tools/weak_shard_rows.py).  --grid G
(strong scaling): one fixed G x G grid, rows split as evenly as possible over
the N ranks.

Every run also reports `config4` (BASELINE.json configs[3]): the 2048 x 2048
grid row-sharded over all N ranks (strong scaling), its cells/s, the same
grid unsharded on rank 0's GPU in the same job (speedup), and a parity gate:
the sharded J / A gathered to rank 0 equal the unsharded run bit for bit and
the belief agrees to rel 1e-5.

Rank 0 prints ONE JSON line.  `roofline` is for the dominant (and only)
kernel, timed live with HIP events on the stream it runs on: at 1024^2 the
tile-resident k_loop_resident (the whole timed trajectory in one launch,
DESIGN.md §3.2) on the dictionary-coded model; with
PP2_TUNE_RESIDENT 0 the launch-per-pair k_loop_pair_coded.  Its algorithmic bytes are the ones the kernel must move
per cell and launch: code 2 + b 4 + b' 4 + J 4 + J' 4 + A 1 = 19 B (the
intermediate step of a pair stays in LDS); `traffic` is the PMC-measured HBM
bytes per launch from profiles/pmc_*.json.  `contract_equivalent` states the
same throughput on SURVEY.md §8(d)'s 417 B/cell fp32 tensor contract of the
reference (T 324 + C 36 + T_u 36 + L_z 4 + b/b'/J/J' 16 + A 1), which the coded
kernel does not move; the `dense_path` leg runs the dense-plane kernel that
does (k_loop_step, or --dense).  Both give bit-identical beliefs, values and
actions (tests/test_gpu_coded.py).  `cpu_baseline` is the C restatement of
the reference (oracle/) timed on this host on a bounded sample of the same
workload.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0            # measured float4 copy rate, the achievable ceiling (same table)
MFMA_F32_PEAK_TFLOPS = 157.3     # dense f32-input MFMA peak (MI355X_MICROARCH.md, Matrix cores)
BYTES_SWEEP = 369                # per cell: T 324 + C 36 + J 4 + J' 4 + A 1
BYTES_BELIEF = 48                # per cell: T_u 36 + L_z 4 + b 4 + b' 4
BYTES_BELIEF_CODED = 10          # per cell: code 2 + b 4 + b' 4 (pp2_belief_update on the coded model)
BYTES_LOOP = BYTES_SWEEP + BYTES_BELIEF   # SURVEY.md §8(d) contract (T counted twice)
FIB_FLOP_CELL = 25920           # reference full-sum flops per cell and FIB sweep (~25.9 k)
F32_VALU_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: f32 vector (v_pk_fma_f32) peak
BYTES_LOOP_DENSE = 381           # k_loop_step: T 324 read ONCE for gather and sweep + C 36 + L_z 4 + b 4 + b' 4 + J 4 + J' 4 + A 1
BYTES_LOOP_CODED = 19            # per cell: code 2 + b 4 + b' 4 + J 4 + J' 4 + A 1
BYTES_SWEEP_CODED = 11           # per cell: code 2 + J 4 + J' 4 + A 1
LDS_BYTES_LOOP_CODED = 204       # per cell-step (factored rows): T_u gather 4*4 + L_z 4 + backup record 16 + quads 8*16 + stay 4 + costs 9*4
LDS_BYTES_LOOP_RESIDENT = 235    # - the backup record (registers) + class-plane rows (<= 3 dwords per quad = 3) + the b / J window rows (2 planes x 3 rows x 24 B per quad = 36) + b', J' stored (8)
RESIDENT_STEPS = 2048            # pp2_loop_steps_per_launch of the tile-resident loop
LDS_PEAK_GBS = 150000.0          # ds_read_b64/b128 chip aggregate (MI355X_MICROARCH.md LDS)
GAMMA = 0.95
RCCL_ROUND_US = (10.0, 30.0)     # assumed RCCL small-message round trip over xGMI (not measurable on 1 GPU)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, default=1024, help="grid side per GPU (weak scaling)")
    ap.add_argument("--shard-rows", type=int, default=896,
                    help="owned rows per GPU at N > 1 (weak scaling; the view adds 2 x e "
                         "halo rows, e = (1024 - rows) / 2)")
    ap.add_argument("--grid", type=int, default=0,
                    help="strong scaling: one G x G grid row-sharded over the ranks")
    ap.add_argument("--c4-size", type=int, default=2048,
                    help="config4 leg: grid side (0 disables)")
    ap.add_argument("--c4-steps", type=int, default=200)
    ap.add_argument("--c4-warmup", type=int, default=16)
    ap.add_argument("--cpt", type=int, default=4, help="cells per lane")
    ap.add_argument("--kernel-reps", type=int, default=100,
                    help="launches per kernel in the per-kernel timing segment")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU-baseline sample budget (rank 0, N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--plan-steps", type=int, default=200,
                    help="QV-tree plan steps for the p50 (0 disables)")
    ap.add_argument("--plan-size", type=int, default=256)
    ap.add_argument("--plan-depth", type=int, default=3)
    ap.add_argument("--cpu-plan-seconds", type=float, default=15.0)
    ap.add_argument("--rollout-copies", type=int, default=4096,
                    help="batched fp16 rollout copies (0 disables)")
    ap.add_argument("--rollout-depth", type=int, default=5)
    ap.add_argument("--rollout-size", type=int, default=512)
    ap.add_argument("--pbvi-S", type=int, default=500, help="PBVI belief set size")
    ap.add_argument("--no-pbvi", action="store_true", help="skip the PBVI leg")
    ap.add_argument("--dense", action="store_true",
                    help="time the dense-plane kernels as the main loop")
    ap.add_argument("--profile", action="store_true",
                    help="only run warmup+timed steps (for rocprofv3)")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="ranks join a gloo group, all-reduce one value and rank 0 prints "
                         "one JSON line; nothing touches a GPU (tests the N > 1 launch)")
    return ap.parse_args(argv)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, n, port):
    """The torch.distributed.run command that starts this script's n ranks
    (one process per GPU, rendezvous on 127.0.0.1) with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def launch_ranks(argv, n):
    """`bench.py --gpus N` (N > 1) started without a launcher: start the
    N-rank job as a CHILD process and return its exit code.  This process
    never imports torch and never touches a GPU, and it does not exec: the
    child's stdout is this process's stdout, so rank 0's JSON line is relayed
    as is."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = launcher_cmd(argv, n, free_port())
    print(f"bench.py: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def launcher_selftest(ws, rank):
    """--launcher-selftest: the ranks of this job join a gloo process group
    and all-reduce their rank + 1; rank 0 prints one JSON line."""
    if os.environ.get("PP2_BENCH_FORCE_FAIL"):  # (tests: the exit code is relayed)
        raise SystemExit(3)
    import torch
    import torch.distributed as dist
    if ws > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)])
    if ws > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launcher_selftest": True, "world_size": ws,
                          "rank_sum": float(t.item()),
                          "launched_by": "torch.distributed.run"
                          if "TORCHELASTIC_RUN_ID" in os.environ else "direct"}), flush=True)
    if ws > 1:
        dist.destroy_process_group()


def pmc_traffic(kernel_substr: str, cells: int, exclude: str | None = None,
                steps: int | None = None):
    """HBM bytes per launch of the dominant kernel from the newest committed
    rocprofv3 PMC summary (profiles/pmc_*.json, written by
    profiles/collect_pmc.py), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        k = d.get("kernels", {})
        for name, v in k.items():
            if (kernel_substr in name and v.get("cells") == cells
                    and not (exclude and exclude in name)
                    and v.get("steps_per_launch") == steps):
                return v.get("hbm_bytes_per_launch"), os.path.basename(f)
    return None, None


def pmc_kernel(kernel_name: str):
    """The newest committed PMC summary entry of a kernel (by short name)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        v = d.get("kernels", {}).get(kernel_name)
        if v and v.get("hbm_bytes_per_launch"):
            return v, os.path.basename(f)
    return None, None


def sweep_resident_traffic(cells):
    """k_sweep_resident's PMC memory-side bytes per solve launch against the
    bytes it must move (code 2 + J 4 + J' 4 + A 1 per cell, + the convergence
    snapshot 4 + 4), from the newest committed PMC summary."""
    v, src = pmc_kernel("k_sweep_resident")
    if not v:
        return None
    algo = (11 + 8) * cells
    return {"traffic_per_launch": v["hbm_bytes_per_launch"], "avg_launch_us": v.get("avg_us"),
            "algorithmic_bytes_per_launch": algo,
            "traffic_over_algorithmic": v["hbm_bytes_per_launch"] / algo, "source": src,
            "cause": "edge-row hand-off granules: plain stores where the neighbouring tile "
                     "sits on the same XCD (they stay in its L2), sc1 stores / loads only at "
                     "the XCD boundaries, which go past L2 to the memory side (DESIGN.md §5)"}


def cgroup_cpu_quota():
    """The CPU bandwidth this process's cgroup grants, in cores (quota /
    period; cgroup v2 cpu.max or v1 cpu.cfs_quota_us), or None when unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) // int(p)))
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return max(1, q // p) if q > 0 and p > 0 else None
    except (OSError, ValueError):
        return None


def cpu_affinity():
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return max(1, os.cpu_count() or 1)


def cpu_threads():
    """Host threads for the CPU baseline: every core this process may use --
    its affinity mask (os.sched_getaffinity), capped by its cgroup's CPU
    quota (on the GPU box the mask lists the whole machine while the quota
    grants a share; threads beyond the quota only time-slice).  Reported as
    cpu_baseline.cores, with both inputs beside it."""
    q = cgroup_cpu_quota()
    a = cpu_affinity()
    return min(a, q) if q else a


def cpu_baseline(grid, goal, us, zs, budget_s):
    """The oracle's reference-order loop step (belief kernel + renormalisation
    + Bellman sweep) on the same grid, in the two CPU modes of SURVEY.md §8(d):
    single thread (the reference's serial host loops), and rows split over
    the host threads (orc_loop_run_mt).  The threaded run is the headline."""
    from oracle import oracle as O
    H, W = grid.shape
    T, L, _ = O.model_pomdp(grid, goal)
    _, Cc = O.model_mdp(grid, goal)
    from path_planning_2d_amd import synthetic as S
    lib = O.lib()
    b0 = S.uniform_belief(grid)
    # single thread
    b = b0.copy()
    J = np.zeros(H * W, np.float32)
    bo = np.empty_like(b)
    Jo = np.empty_like(J)
    A = np.empty(H * W, np.uint8)
    steps = 0
    t0 = time.perf_counter()
    while True:
        u, z = int(us[steps % len(us)]), int(zs[steps % len(zs)])
        lib.orc_belief_update(H, W, T, L, b, u, z, bo, 1)
        lib.orc_normalize_seq(bo.size, bo)
        b, bo = bo, b
        lib.orc_mdp_sweep(H, W, np.float32(GAMMA), T, Cc, J, Jo, A)
        J, Jo = Jo, J
        steps += 1
        el = time.perf_counter() - t0
        if el >= budget_s / 2 or steps >= 10000:
            break
    single = {"value": H * W * steps / el, "cores": 1,
              "sample": f"{steps} loop steps, {el:.1f} s"}
    # rows split over threads, in chunks of steps until half the budget
    nt = cpu_threads()
    b = b0.copy()
    J = np.zeros(H * W, np.float32)
    u8 = np.ascontiguousarray(np.resize(us, 4096), np.uint8)
    z8 = np.ascontiguousarray(np.resize(zs, 4096), np.uint8)
    msteps = 0
    t0 = time.perf_counter()
    while True:
        chunk = 8
        lib.orc_loop_run_mt(H, W, np.float32(GAMMA), T, L, Cc, b, bo, J, Jo, A, chunk,
                            u8[msteps % 4000:], z8[msteps % 4000:], nt)
        msteps += chunk
        el = time.perf_counter() - t0
        if el >= budget_s / 2 or msteps >= 100000:
            break
    # the simulator's scatter-form CPU filter (dummy_simulator.cpp:671-773),
    # belief steps only, single thread: the other CPU formulation of the step
    gu8 = np.ascontiguousarray(grid, np.uint8)
    b = b0.copy()
    p = np.empty_like(b)
    ssteps = 0
    t0 = time.perf_counter()
    while True:
        lib.orc_sim_predict(H, W, gu8, b, int(us[ssteps % len(us)]), p)
        lib.orc_sim_correct(H, W, gu8, p, int(zs[ssteps % len(zs)]), b)
        ssteps += 1
        el_s = time.perf_counter() - t0
        if el_s >= min(3.0, budget_s / 4) or ssteps >= 10000:
            break
    scatter = {"value": H * W * ssteps / el_s, "unit": "cells/s (belief step only)", "cores": 1,
               "sample": f"{ssteps} predict+correct steps, {el_s:.1f} s (orc_sim_predict/"
                         f"orc_sim_correct, dummy_simulator.cpp:671-773)"}
    return {"value": H * W * msteps / el, "unit": "cells/s", "cores": nt,
            "kind": "port",
            "scatter_filter": scatter,
            "sample": f"{msteps} loop steps on the same {H}x{W} grid ({el:.1f} s), rows split "
                      f"over {nt} threads (oracle/pp2_oracle.c orc_loop_run_mt, -O3 "
                      f"-march=native); single thread: {single['value']:.3g} cells/s "
                      f"({single['sample']})",
            "single_thread": single,
            "cpu": cpu_model(), "host_cpus": os.cpu_count(),
            "cores_source": "min(len(os.sched_getaffinity(0)), cgroup CPU quota): every core "
                            "this process may run on, capped by the cores its cgroup grants",
            "affinity_cores": cpu_affinity(), "cgroup_quota_cores": cgroup_cpu_quota(),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def closed_loop(grid, b0, step_fn, max_steps, budget_s=1e9, min_steps=0):
    """Closed-loop plan steps (synthetic.closed_loop): (ms, actions, values)."""
    from path_planning_2d_amd import synthetic as S
    return S.closed_loop(grid, b0, step_fn, max_steps, budget_s, min_steps=min_steps)


def step_stats(ms):
    return {"steps": int(ms.size), "p50_ms": float(np.percentile(ms, 50)),
            "p90_ms": float(np.percentile(ms, 90)), "mean_ms": float(ms.mean())}


def gpu_plan_run(grid, b0, make_planner, steps):
    """A warm-up of 3 closed-loop steps (code objects, allocations) on one
    planner, then `steps` timed steps on a fresh one (the warm-up advanced
    the first planner's rand() stream, which a reset keeps): (ms, actions,
    values, tree info after the last step)."""
    with make_planner() as pl:
        closed_loop(grid, b0, pl.step, 3)
    with make_planner() as pl:
        ms, acts, vals = closed_loop(grid, b0, pl.step, steps)
        return ms, acts, vals, pl.info()


def oracle_plan_run(grid, b0, opl, steps, budget_s, min_steps, gpu_acts, gpu_vals, what):
    """The oracle's reference-arithmetic QV-tree (oracle/pp2_oracle_tree.c,
    every node holding its own host belief, sequential fp32 sums) on the same
    closed loop: its plan-step times beside the GPU's, and the parity gate
    -- the GPU's actions and values equal the oracle's at every step the
    CPU leg ran (synthetic.action_parity)."""
    from path_planning_2d_amd import synthetic as S
    cms, ca, cv = closed_loop(grid, b0, opl.step, steps, budget_s, min_steps=min_steps)
    cpu = {"p50_ms": float(np.percentile(cms, 50)), "p90_ms": float(np.percentile(cms, 90)),
           "steps": int(cms.size), "cores": 1, "kind": "port",
           "sample": f"{cms.size} closed-loop plan steps of the oracle's reference-semantics "
                     f"QV-tree (oracle/pp2_oracle_tree.c, every node holds a host belief), "
                     f"{what}"}
    parity = S.action_parity(gpu_acts, gpu_vals, ca, cv)
    parity["reference"] = ("oracle/pp2_oracle_tree.c in reference arithmetic on the same "
                           "seeded closed loop: actions equal and values equal as fp32 bits "
                           "at every compared step")
    return cpu, parity


def plan_step_bench(args, device, stream_handle, with_cpu):
    """BASELINE configs[1]: 256x256 synthetic grid, POMDP belief update +
    QV-tree with max_search_tree_depth 3 (FIB upper bound, constant lower
    bound -5/(1-gamma)).  Closed loop: the planner's action moves a simulated
    robot (T), whose observation (L) is the next message.  Wall time of each
    plan step (tree update + expansions + argmax), as beliefCallback measures
    it (src/pomdp/path_planning_2d.cu:210-231).  With the CPU leg, the parity
    gate: the GPU's actions and values equal the reference-arithmetic oracle's
    at every step the oracle ran (>= 100)."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = args.plan_size
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    ctx = P.GridContext(grid, goal, gamma=GAMMA, device=device)
    ctx.set_stream(stream_handle)
    ctx.model_generate()
    t0 = time.perf_counter()
    fib_sweeps, _ = ctx.fib_solve()
    fib_s = time.perf_counter() - t0
    alphas = ctx.fib_get()
    b0 = S.uniform_belief(grid)

    # the drop-in's mode (pp2_planner_default_params: reference_order = 1):
    # bit-exact with the reference's fp32 host arithmetic -- the headline p50
    ms, acts, vals, info = gpu_plan_run(
        grid, b0, lambda: P.QVTreePlanner(ctx, max_search_tree_depth=args.plan_depth,
                                          max_online_iteration=15, reference_order=1),
        args.plan_steps)
    # opt-in fast variant (reference_order = 0): parallel tree / fp64 sums,
    # within rel 1e-4 of the reference arithmetic, NOT bit-exact
    ms_ts, _, _, _ = gpu_plan_run(
        grid, b0, lambda: P.QVTreePlanner(ctx, max_search_tree_depth=args.plan_depth,
                                          max_online_iteration=15, reference_order=0),
        args.plan_steps)
    ctx.close()
    out = {"config": f"{N}x{N} synthetic grid, max_search_tree_depth {args.plan_depth}, "
                     f"max_online_iteration 15, FIB upper bound ({fib_sweeps} sweeps, "
                     f"{fib_s * 1e3:.1f} ms on GPU), lower bound -5/(1-gamma)",
           "mode": "reference_order=1 (default; bit-exact with the reference's host "
                   "fp32 arithmetic)",
           **step_stats(ms),
           "first_ms": float(ms[0]), "final_tree_vnodes": int(info["total_vnodes"]),
           "tree_sum_variant": {**step_stats(ms_ts),
                                "note": "opt-in reference_order=0: grid-wide sums as "
                                        "parallel trees, within rel 1e-4 of the reference "
                                        "arithmetic, NOT bit-exact"}}
    if with_cpu:
        from oracle import oracle as O
        T, L, R = O.model_pomdp(grid, goal)
        opl = O.Planner(grid, T, L, R, alphas, max_depth=args.plan_depth, max_iter=15)
        out["cpu_baseline"], out["parity"] = oracle_plan_run(
            grid, b0, opl, args.plan_steps, args.cpu_plan_seconds, 100, acts, vals,
            "same grid/alphas")
        opl.close()
    return out


def pbvi_plan_leg(args, ctx, grid, b0, calls, depth, with_cpu, cpu_budget, min_cpu_steps, what):
    """Closed-loop plan steps with PBVI leaf lower bounds (lower_bound_mode 1,
    evaluatePbviCpu per VNode, search_tree_cuda.cu:379) on a context that
    holds the PBVI alphas, the tree's rand() stream continuing after
    generateBeliefSet's `calls` draws (PomdpPathPlanning2d::initialize runs
    PBVI before the first plan step).  Reference order (the drop-in's mode)
    timed and parity-gated against the oracle; the tree-sum variant timed."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    def planner(ref):
        return lambda: P.QVTreePlanner(ctx, max_search_tree_depth=depth,
                                       max_online_iteration=15, lower_bound_mode=1,
                                       rand_skip=calls, reference_order=ref)
    ms, acts, vals, _ = gpu_plan_run(grid, b0, planner(1), args.plan_steps)
    ms_ts, _, _, _ = gpu_plan_run(grid, b0, planner(0), args.plan_steps)
    out = {"mode": "reference_order=1 (default; bit-exact)", "config": what, **step_stats(ms),
           "tree_sum_variant": {
               **step_stats(ms_ts),
               "note": "opt-in reference_order=0 (PBVI dots by the split-x MFMA GEMM, not the "
                       "reference's x-ordered chains): NOT bit-exact"}}
    if with_cpu:
        from oracle import oracle as O
        H, W = grid.shape
        goal = ctx.goal
        T, L, R = O.model_pomdp(grid, goal)
        pal, pact = ctx.pbvi_get()
        opl = O.Planner(grid, T, L, R, ctx.fib_get(), max_depth=depth, max_iter=15)
        opl.set_pbvi(pal, pact)
        opl.skip_rand(calls)
        out["cpu_baseline"], out["parity"] = oracle_plan_run(
            grid, b0, opl, args.plan_steps, cpu_budget, min_cpu_steps, acts, vals,
            "same grid, FIB and PBVI alphas, rand() stream")
        opl.close()
    return out


def pbvi_bench(args, device, stream_handle, with_cpu):
    """PBVI lower bound (point_based_value_iteration_cuda.cu): the reference
    node's configuration -- S = 500 beliefs on the 100x40 map, 167 backups
    (gamma 0.95) -- end to end, and the same at 256x256 (BASELINE configs[1]'s
    grid, which the reference cannot run).  Each is followed
    by closed-loop plan steps with PBVI leaf lower bounds: on the 100x40 map
    the reference node's own launch configuration (`node_plan_step`: goal
    (95, 34), max_search_tree_depth 50, max_online_iteration 15,
    launch/pomdp_path_planning_2d.launch:7-14), at 256x256 depth 3.
    `gemm_equiv_tflops` = the iteration's Sgemm flops (2 * 144 * Sp^2 * ld) /
    the whole iteration's time: a lower bound on the MFMA GEMM kernel's own
    rate (its rocprof time is in profiles/)."""
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden")
    out = {}
    cases = [("sparse_map_100x40 (reference node: S=500, 167 backups)",
              np.load(os.path.join(gold, "maps", "sparse_map_100x40.npy"), allow_pickle=False),
              (95, 34), 0)]
    g256 = S.synth_grid(256, 256, seed=256)
    cases.append((f"256x256 synthetic, S={args.pbvi_S}", g256, S.synth_goal(g256), 0))
    for label, grid, goal, iters in cases:
        with P.GridContext(grid, goal, gamma=GAMMA, device=device) as ctx:
            ctx.set_stream(stream_handle)
            ctx.model_generate()
            b0 = S.uniform_belief(grid)
            ctx.pbvi_belief_set(b0, 8)  # warm-up: code objects, allocations
            ctx.pbvi_backup(1)
            ctx.synchronize()
            t0 = time.perf_counter()
            calls = ctx.pbvi_belief_set(b0, args.pbvi_S)
            ctx.synchronize()
            t_set = time.perf_counter() - t0
            t0 = time.perf_counter()
            ctx.pbvi_backup(iters)
            ctx.synchronize()
            t_bk = time.perf_counter() - t0
            plan = node = None
            if iters == 0 and args.plan_steps > 0:
                ctx.fib_solve()
                if grid.shape == (256, 256):
                    # BASELINE configs[1] with the reference node's PBVI leaf
                    # bounds (the reference itself falls back to -5/(1-gamma))
                    plan = pbvi_plan_leg(
                        args, ctx, grid, b0, calls, args.plan_depth, with_cpu,
                        args.cpu_plan_seconds, 3,
                        f"256x256 synthetic grid, max_search_tree_depth {args.plan_depth}, "
                        f"max_online_iteration 15, FIB upper bound, PBVI lower bound "
                        f"(S={args.pbvi_S}, 167 backups)")
                elif grid.shape == (40, 100):
                    node = pbvi_plan_leg(
                        args, ctx, grid, b0, calls, 50, with_cpu, args.cpu_plan_seconds, 10,
                        f"the reference node's launch configuration: sparse_map_100x40, goal "
                        f"(95, 34), max_search_tree_depth 50, max_online_iteration 15, FIB "
                        f"upper bound, PBVI lower bound (S={args.pbvi_S}, 167 backups), "
                        f"rand() continuing after generateBeliefSet "
                        f"(launch/pomdp_path_planning_2d.launch:7-14)")
            n_it = iters if iters > 0 else int(np.ceil(np.log(np.float32(1e-3) / np.float32(5))
                                                       / np.log(np.float32(GAMMA))))
            Sp = (args.pbvi_S + 127) // 128 * 128
            ld = (grid.size + 63) // 64 * 64
            flop = 2.0 * 144 * Sp * Sp * ld
            v, _ = ctx.pbvi_evaluate(b0[None, :])
        key = "ref_100x40" if grid.shape == (40, 100) else "synth_256"
        out[key] = {"config": label, "S": args.pbvi_S, "iterations": n_it,
                    "belief_set_s": t_set, "backup_s": t_bk,
                    "backup_iter_ms": 1e3 * t_bk / n_it,
                    "gemm_equiv_tflops": flop * n_it / t_bk / 1e12,
                    "mfma_f32_peak_tflops": MFMA_F32_PEAK_TFLOPS,
                    "root_lower_bound": float(v[0])}
        if plan is not None:
            out[key]["plan_step_pbvi_lb"] = plan
        if node is not None:
            out[key]["node_plan_step"] = node
    if with_cpu:
        from oracle import oracle as O
        grid = cases[0][1]
        H, W = grid.shape
        T, L, R = O.model_pomdp(grid, (95, 34))
        b0 = S.uniform_belief(grid)
        t0 = time.perf_counter()
        B, _ = O.pbvi_belief_set(H, W, T, L, b0, args.pbvi_S)
        cs = time.perf_counter() - t0
        s_small = 64
        t0 = time.perf_counter()
        O.pbvi_backup(H, W, GAMMA, T, L, R, B[:s_small], iterations=1)
        cb = time.perf_counter() - t0
        it_cpu = cb * (args.pbvi_S / s_small) ** 2
        n_it = out["ref_100x40"]["iterations"]
        out["cpu_baseline"] = {
            "belief_set_s": cs, "backup_iter_s_extrapolated": it_cpu,
            "total_s_extrapolated": cs + it_cpu * n_it, "cores": 1, "kind": "port",
            "sample": f"oracle/pp2_oracle_pbvi.c on 100x40: generateBeliefSet at S={args.pbvi_S} "
                      f"timed in full; one backup at S={s_small} timed and scaled by "
                      f"(S/{s_small})^2 (the per-(a,o) Sgemm dominates)"}
        out["speedup_vs_cpu"] = out["cpu_baseline"]["total_s_extrapolated"] / (
            out["ref_100x40"]["belief_set_s"] + out["ref_100x40"]["backup_s"])
    return out


def rollout_bench(args, device, stream):
    """BASELINE configs[4]: 512x512 grid, 4096 belief copies x depth 5, fp16
    beliefs.  Algorithmic bytes per cell-copy-step: fp16 belief read 2 +
    write 2 (T_u / L_z / R_u amortised over the copies sharing the action),
    plus 2 per cell-copy for the FIB leaf pass."""
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N, C, D = args.rollout_size, args.rollout_copies, args.rollout_depth
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    b0 = S.uniform_belief(grid)
    us, zs = S.rollout_trajectories(grid, b0, C, D, seed=13)
    ctx = P.GridContext(grid, goal, gamma=GAMMA, device=device)
    ctx.set_stream(stream.cuda_stream)
    ctx.model_generate()
    ctx.fib_solve(max_sweeps=40)
    with P.BatchedRollout(ctx, C, D) as r:
        r.set_root(b0)
        r.run(us, zs)  # warm-up
        torch.cuda.synchronize()
        times = []
        for _ in range(5):
            r.set_root(b0)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            r.run(us, zs)
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        res = r.results()
    ctx.close()
    ms = float(np.median(times))
    cell_copy_steps = N * N * C * D
    algo_bytes = cell_copy_steps * 4 + N * N * C * 2
    return {"config": f"{N}x{N} grid, {C} belief copies x depth {D}, fp16 beliefs "
                      f"(fp32 math), copies grouped by action",
            "ms_per_rollout": ms,
            "cell_copy_steps_per_s": cell_copy_steps / (ms * 1e-3),
            "algorithmic_GBps": algo_bytes / (ms * 1e-3) / 1e9,
            "hbm_frac": algo_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "mean_value": float(res["value"].mean())}


def _gather_rows(arr, r0, r1, G, W, ws, torch, dist):
    """Rows [r0, r1) (flat, row-major) of a G x W array from every rank,
    assembled in row order on every rank (all_gather over RCCL)."""
    maxr = -(-G // ws)
    t = torch.zeros((maxr * W,), dtype=torch.from_numpy(arr[:1]).dtype, device="cuda")
    t[: (r1 - r0) * W] = torch.from_numpy(np.ascontiguousarray(arr)).cuda()
    parts = [torch.empty_like(t) for _ in range(ws)]
    dist.all_gather(parts, t)
    out = []
    for r in range(ws):
        a, b = r * G // ws, (r + 1) * G // ws
        out.append(parts[r][: (b - a) * W].cpu().numpy())
    return np.concatenate(out)


def config4_leg(args, ws, rank, local, stream):
    """BASELINE.json configs[3]: the G x G (2048^2) grid, belief stencil +
    Bellman sweep row-sharded over the ws ranks (strong scaling, RCCL halo
    every 8 steps), and the same grid unsharded on rank 0's GPU in the same
    job: cells/s of both, the speedup, and the parity gate (sharded J / A ==
    unsharded bit for bit, belief rel 1e-5 above a 1e-30 floor; the reference
    loop is single-GPU, src/mdp/path_planning_2d.cu:226-237)."""
    import torch
    import torch.distributed as dist
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    G = args.c4_size
    grid = S.synth_grid(G, G, seed=G)
    goal = S.synth_goal(grid)
    w, k = args.c4_warmup, args.c4_steps
    us, zs, _ = S.synth_trajectory(grid, w + k, seed=42)
    b0 = S.uniform_belief(grid)
    r0, r1 = rank * G // ws, (rank + 1) * G // ws

    def run(ctx, sharded):
        ctx.loop_run(us[:w], zs[:w])
        torch.cuda.synchronize()
        if sharded:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.loop_run(us[w:], zs[w:])
        torch.cuda.synchronize()
        if sharded:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if sharded:
            t = torch.tensor([el], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    out = None
    rank_share = None
    if ws == 1:
        rank_share = config4_rank_share(args, grid, goal, us, zs, b0, local, stream, run)
    if ws > 1:
        ctx = P.GridContext(grid, goal, gamma=GAMMA, device=local, rows=(r0, r1))
        ctx.set_stream(stream.cuda_stream)
        uid = torch.zeros(P._lib.RCCL_ID_BYTES, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(P.GridContext.rccl_unique_id()),
                                       dtype=torch.uint8))
        dist.broadcast(uid, src=0)
        ctx.shard_comm_init(bytes(uid.cpu().numpy().tobytes()), ws, rank)
        ctx.model_generate()
        ctx.belief_set(b0[r0 * G:r1 * G])
        ctx.mdp_reset()
        ctx.synchronize()
        el = run(ctx, True)
        b = ctx.belief_get()  # collective: global mass all-reduce
        J, A = ctx.mdp_get()
        # the RCCL rounds of the same call, event-timed on the stream they run
        # on, in a second (untimed) run continuing from the gathered state
        rounds = comm_round_stats(ctx, lambda: ctx.loop_run(us[w:], zs[w:]), torch, dist)
        ctx.close()
        bg = _gather_rows(b, r0, r1, G, G, ws, torch, dist)
        Jg = _gather_rows(J, r0, r1, G, G, ws, torch, dist)
        Ag = _gather_rows(A, r0, r1, G, G, ws, torch, dist)
    if rank == 0:
        with P.GridContext(grid, goal, gamma=GAMMA, device=local) as c1:
            c1.set_stream(stream.cuda_stream)
            c1.model_generate()
            c1.belief_set(b0)
            c1.mdp_reset()
            c1.synchronize()
            el1 = run(c1, False)
            b1 = c1.belief_get()
            J1, A1 = c1.mdp_get()
        v1 = G * G * k / el1
        out = {"workload": f"{G}x{G} grid (BASELINE.json configs[3]), {k} timed loop steps "
                           f"after {w} warm-up, rows split over {ws} rank(s)",
               "n_gpus": ws, "scaling": "strong",
               "unsharded_1gpu": {"cells_per_s": v1, "ms_per_step": 1e3 * el1 / k}}
        if ws > 1:
            v = G * G * k / el
            j_ok = bool(np.array_equal(Jg.view(np.uint32), J1.view(np.uint32)))
            a_ok = bool(np.array_equal(Ag, A1))
            err = np.abs(bg.astype(np.float64) - b1) / np.maximum(np.abs(b1.astype(np.float64)),
                                                                   1e-300)
            bmask = np.abs(b1) > 1e-30
            b_rel = float(err[bmask].max()) if bmask.any() else 0.0
            b_ok = b_rel <= 1e-5 and bool(np.all(np.abs(bg[~bmask]) <= 1e-30))
            out.update({"cells_per_s": v, "ms_per_step": 1e3 * el / k,
                        "speedup_vs_unsharded_1gpu": v / v1,
                        "rccl_round_us": rounds,
                        "parity": {"J_bit_exact": j_ok, "A_bit_exact": a_ok,
                                   "belief_max_rel_err": b_rel, "belief_ok": b_ok,
                                   "pass": j_ok and a_ok and b_ok}})
        else:
            out.update({"cells_per_s": v1, "ms_per_step": 1e3 * el1 / k,
                        "speedup_vs_unsharded_1gpu": 1.0,
                        "parity": "single rank: nothing to gather"})
            if rank_share is not None:
                t1 = 1e6 * el1 / k
                proj = rank_share["projection_8_ranks"]
                proj["unsharded_1gpu_us_per_step"] = t1
                proj["speedup_vs_unsharded_1gpu"] = [t1 / proj["us_per_step"][1],
                                                     t1 / proj["us_per_step"][0]]
                # the share's SQ counters (its 2-D resident instance), newest round
                rank_share["sq_counters"] = sq_counters("c4_share_sq.json")
                out["rank_share_8"] = rank_share
    if ws > 1:
        dist.barrier()
    return out


def comm_round_stats(ctx, call, torch, dist=None):
    """Run `call` once with PP2_TUNE_COMM_TIMING on: every RCCL round of the
    context (halo exchange + {mass, shift, lost} records, closing all-reduce)
    between HIP events on the stream it is issued on.  Per rank: rounds,
    mean / median / max us; with `dist`, the max over ranks of each figure
    beside rank 0's own."""
    ctx.synchronize()
    ctx.set_tuning(ctx.TUNE_COMM_TIMING, 1)
    call()
    us_r, untimed = ctx.comm_rounds()
    ctx.set_tuning(ctx.TUNE_COMM_TIMING, 0)
    n = int(us_r.size)
    mine = [float(n), float(us_r.mean()) if n else 0.0,
            float(np.median(us_r)) if n else 0.0, float(us_r.max()) if n else 0.0,
            float(us_r.sum())]
    out = {"rounds": n, "untimed_rounds": int(untimed), "mean_us": mine[1],
           "median_us": mine[2], "max_us": mine[3], "total_us": mine[4],
           "first_us": float(us_r[0]) if n else None,
           "method": "hipEventRecord before / after each RCCL group on the issuing stream "
                     "(PP2_TUNE_COMM_TIMING): the group's own time plus any wait for the "
                     "peers; a second run of the timed call, not inside the timed region"}
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor(mine, dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        m = t.cpu().tolist()
        out["max_over_ranks"] = {"mean_us": m[1], "median_us": m[2], "max_us": m[3],
                                 "total_us": m[4]}
    return out


def config4_rank_share(args, grid, goal, us, zs, b0, local, stream, run):
    """config4's per-rank work at 8 ranks, measured on this GPU: rank 3's
    256 x 2048 shard of the 2048^2 grid as an RCCL shard with a 1-rank
    communicator, so pp2_loop_run takes the resident shard path exactly as
    a rank of the 8-GPU job does (views of 256 + 2e rows, one launch per e
    steps, the {mass, shift} all-reduce, halo exchanges and rebases) -- with
    every RCCL call a 1-rank no-op.  The 8-GPU time is then projected as this
    measured step plus the RCCL rounds the real job adds per call (one per
    block: the first block's halo exchange, every later block's {mass, shift,
    lost} records and halo rows in ONE RCCL group; plus the closing
    all-reduce; the ranks' agreement on e is made once per model / tuning /
    reset, not per call) at an ASSUMED
    xGMI round trip
    (RCCL_ROUND_US; multi-GPU RCCL cannot run on one GPU)."""
    import torch
    import path_planning_2d_amd as P
    G = args.c4_size
    R = 8
    r0, r1 = 3 * G // R, 4 * G // R
    w, k = args.c4_warmup, args.c4_steps
    ctx = P.GridContext(grid, goal, gamma=GAMMA, device=local, rows=(r0, r1))
    ctx.set_stream(stream.cuda_stream)
    ctx.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
    ctx.model_generate()
    ctx.belief_set(b0[r0 * G:r1 * G])
    ctx.mdp_reset()
    ctx.synchronize()
    e = ctx.loop_steps_per_launch()
    tiling = ctx.resident_tiling()
    l0 = ctx.resident_launches()[0]
    el = run(ctx, False)
    launches = ctx.resident_launches()[0] - l0
    rounds1 = comm_round_stats(ctx, lambda: ctx.loop_run(us[w:], zs[w:]), torch)
    rounds1["note"] = ("1-rank communicator: every round is an RCCL no-op group / all-reduce, so "
                       "this is the issue floor of a round on this GPU, not an xGMI transfer")
    ctx.close()
    t = 1e6 * el / k
    nblk = -(-k // e)
    rounds = nblk + 1
    lo, hi = (t + rounds * r / k for r in RCCL_ROUND_US)
    return {"shard": f"rows [{r0}, {r1}) x {G} of the {G}^2 grid (rank 3 of 8), 1-rank RCCL "
                     f"communicator",
            "steps_per_launch": e, "resident_launches_in_run": launches,
            "resident_tiling": {"tiles": tiling[0], "rows_per_tile": tiling[1],
                                "tile_cols": tiling[2]},
            "measured_us_per_step": t,
            "rccl_round_us_1rank": rounds1,
            "projection_8_ranks": {
                "assumed_rccl_round_us": list(RCCL_ROUND_US),
                "rccl_rounds_per_call": rounds,
                "us_per_step": [lo, hi],
                "note": "measured per-rank step + rounds x assumed RCCL round trip / steps; "
                        "a projection, not a measurement (one GPU)",
                "assumption": "every round costs the assumed neighbour round trip, including "
                              "the later blocks' rounds in which the {mass, shift, lost} "
                              "records go point to point to all nranks - 1 peers of the halo "
                              "group (exchange_halos_k, records=true): an 8-peer grouped "
                              "send/recv is priced like a 2-neighbour exchange; not measured "
                              "(the 1-rank communicator skips the records loop)"}}


def weak_rank_share(args, local, stream, n1_cells_per_s):
    """The weak-scaling line's per-rank work at N >= 2, measured on this GPU:
    rank 1's shard (rows [R, 2R) of a 2R x S grid, R = --shard-rows) as an
    RCCL shard with a 1-rank communicator, so pp2_loop_run takes the resident
    shard path exactly as a rank of the N-GPU job does, with every RCCL call
    a 1-rank no-op.  Projection as in config4: + the call's RCCL rounds at an
    ASSUMED xGMI round trip; the implied weak-scaling efficiency is the
    projected per-rank cells/s over N = 1's."""
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    W, R = args.size, args.shard_rows
    grid = S.synth_grid(2 * R, W, seed=2 * R)
    goal = S.synth_goal(grid)
    w, k = args.warmup, args.steps
    us, zs, _ = S.synth_trajectory(grid, w + k, seed=42)
    b0 = S.uniform_belief(grid)
    ctx = P.GridContext(grid, goal, gamma=GAMMA, device=local, rows=(R, 2 * R))
    ctx.set_stream(stream.cuda_stream)
    ctx.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
    ctx.model_generate()
    ctx.belief_set(b0[R * W:2 * R * W])
    ctx.mdp_reset()
    ctx.synchronize()
    e = ctx.loop_steps_per_launch()
    ctx.loop_run(us[:w], zs[:w])
    torch.cuda.synchronize()
    l0 = ctx.resident_launches()[0]
    t0 = time.perf_counter()
    ctx.loop_run(us[w:], zs[w:])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    launches = ctx.resident_launches()[0] - l0
    ctx.close()
    t = 1e6 * el / k
    rounds = -(-k // e) + 1
    proj = [t + rounds * r / k for r in RCCL_ROUND_US]
    return {"shard": f"rows [{R}, {2 * R}) x {W} of a {2 * R}x{W} grid (rank 1 of 2), 1-rank "
                     f"RCCL communicator",
            "steps_per_launch": e, "resident_launches_in_run": launches,
            "measured_us_per_step": t,
            "measured_cells_per_s_per_rank": R * W / (t * 1e-6),
            "projection": {
                "assumed_rccl_round_us": list(RCCL_ROUND_US),
                "rccl_rounds_per_call": rounds,
                "us_per_step": proj,
                "weak_efficiency_vs_n1": [R * W / (p * 1e-6) / n1_cells_per_s for p in proj[::-1]],
                "note": "measured per-rank step + rounds x assumed RCCL round trip / steps; "
                        "a projection, not a measurement (one GPU)"}}


def sq_counters(name="resident_sq.json"):
    """LDS / VALU busy fractions of k_loop_resident from the newest committed
    SQ-counter summary (profiles/r*/<name>, tools/collect_lds_pmc.sh +
    tools/sq_summary.py; c4_share_sq.json: config 4's rank share), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        d["source"] = os.path.relpath(f, ROOT)
        return d
    return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def main():
    args = parse()
    ws, rank, local = dist_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher environment: start the N-rank job as a child process
        return launch_ranks(sys.argv[1:], args.gpus)
    if ws != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {ws}")
    if args.launcher_selftest:
        launcher_selftest(ws, rank)
        return 0
    import torch
    import torch.distributed as dist
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S

    torch.cuda.set_device(local)
    if ws > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    strong = args.grid > 0
    if strong:
        gh = gw = args.grid
        r0, r1 = rank * gh // ws, (rank + 1) * gh // ws
    else:
        N = args.size
        R = N if ws == 1 else args.shard_rows
        gh, gw = R * ws, N
        r0, r1 = rank * R, (rank + 1) * R
    grid = S.synth_grid(gh, gw, seed=gh)
    goal = S.synth_goal(grid)
    total = args.warmup + args.steps
    # long enough for the timed steps and for the per-kernel timing segment
    ntraj = max(total, args.kernel_reps)
    us, zs, _ = S.synth_trajectory(grid, min(ntraj, 4096), seed=42)
    us = np.resize(us, ntraj)
    zs = np.resize(zs, ntraj)
    b0 = S.uniform_belief(grid)

    ctx = P.GridContext(grid, goal, gamma=GAMMA, device=local,
                        rows=(r0, r1) if ws > 1 else None)
    ctx.set_cells_per_lane(args.cpt)
    # a dedicated stream: torch's default stream has handle 0, which the C ABI
    # reads as "use the context's own stream"
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    if ws > 1:
        uid = torch.zeros(P._lib.RCCL_ID_BYTES, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(P.GridContext.rccl_unique_id()),
                                       dtype=torch.uint8))
        dist.broadcast(uid, src=0)
        ctx.shard_comm_init(bytes(uid.cpu().numpy().tobytes()), ws, rank)
    ctx.model_generate()
    if args.dense:
        ctx.set_tuning(ctx.TUNE_CODED_MODEL, 0)
    dict_entries, coded = ctx.model_dict_info()
    steps_per_launch = ctx.loop_steps_per_launch()
    cells_per_gpu = (r1 - r0) * gw  # this rank's cells
    ctx.belief_set(b0[r0 * gw:r1 * gw])
    ctx.mdp_reset()
    ctx.synchronize()

    # ------------------------------------------- per-kernel timing (HIP events)
    # These secondary legs run BEFORE the headline's warmup and timed steps:
    # they keep the GPU busy for tens of ms, so the timed steps run at the
    # working clock (a GPU fresh out of idle runs the same 20-step launch
    # ~8 % slower, tools/micro/clock_warmup.py).  The state is reset after.
    legs_t0 = time.perf_counter()
    reps = args.kernel_reps
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)

    def timed(fn):
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    def loop_reps():
        ctx.loop_run(us[:reps], zs[:reps])

    sweep_ms = timed(lambda: ctx.mdp_sweep(reps))  # coded when active
    pairs_ms = None
    if coded and steps_per_launch >= RESIDENT_STEPS:
        # the launch-per-pair path beside the resident loop (same steps)
        ctx.set_tuning(ctx.TUNE_RESIDENT, 0)
        pairs_ms = timed(loop_reps)
        ctx.set_tuning(ctx.TUNE_RESIDENT, 1)
    belief_ms = timed(lambda: [ctx.belief_update(int(us[k]), int(zs[k])) for k in range(reps)])
    # row a5: the FIB sweep on the same grid (VALU-bound: SURVEY.md §8(d)
    # prices it on the reference's full-sum flops against the f32 VALU peak)
    fib = None
    if rank == 0 and ws == 1:
        ctx.fib_reset()
        ctx.fib_sweep(3)
        fib_ms = timed(lambda: ctx.fib_sweep(reps))
        fib = {"kernel": ("k_fib_sweep_lds" if coded and cells_per_gpu >= 512 * 1024
                          else "k_fib_sweep_sparse" if coded else "k_fib_sweep"),
               "us_per_sweep": fib_ms * 1e3,
               "full_sum_tflops": FIB_FLOP_CELL * cells_per_gpu / (fib_ms * 1e-3) / 1e12,
               "frac_of_f32_valu_peak": FIB_FLOP_CELL * cells_per_gpu / (fib_ms * 1e-3) / 1e12
               / F32_VALU_PEAK_TFLOPS,
               "note": "flops of the reference's full 9-term sums (SURVEY.md §8(d), ~25.9 "
                       "kflop/cell); the kernel executes the support terms only (~11.5 k), "
                       "bit-identical"}
    dense = None
    if coded:
        ctx.set_tuning(ctx.TUNE_CODED_MODEL, 0)
        dloop_ms = timed(loop_reps)
        dsweep_ms = timed(lambda: ctx.mdp_sweep(reps))
        ctx.set_tuning(ctx.TUNE_CODED_MODEL, 1)
        dloop_gbs = BYTES_LOOP_DENSE * cells_per_gpu / (dloop_ms * 1e-3) / 1e9
        dtraffic, dsrc = pmc_traffic("k_loop_step", cells_per_gpu, exclude="coded")
        dense = {"kernel": "k_loop_step (dense model planes)",
                 "loop_step_us": dloop_ms * 1e3,
                 "cells_per_s": cells_per_gpu / (dloop_ms * 1e-3),
                 "loop_gbs": dloop_gbs, "loop_frac": dloop_gbs / HBM_PEAK_GBS,
                 "loop_frac_of_measured_copy_rate": dloop_gbs / HBM_COPY_GBS,
                 "algorithmic_bytes_per_cell": BYTES_LOOP_DENSE,
                 "traffic_per_launch": dtraffic, "traffic_source": dsrc,
                 "mdp_sweep_us": dsweep_ms * 1e3,
                 "mdp_sweep_frac": BYTES_SWEEP * cells_per_gpu / (dsweep_ms * 1e-3) / 1e9
                 / HBM_PEAK_GBS}
    mdp_solve = None
    if rank == 0 and ws == 1:
        # BASELINE configs[2]: MDP value iteration to convergence on this grid
        # (valueIteration, src/mdp/path_planning_2d.cu:207-269, no GUI)
        # the first solve on a context also pays its one-time setup (the
        # resident solve's plan); the steady-state solve is timed after it
        solve_ms = []
        for _ in range(2):
            ctx.mdp_reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n_sw, nrm = ctx.mdp_solve()
            torch.cuda.synchronize()
            solve_ms.append((time.perf_counter() - t0) * 1e3)
        mdp_solve = {"config": f"{gh}x{gw} MDP value iteration to convergence "
                               f"(blocks of 100 sweeps, stop at inf-norm <= 1e-3*5/(1-gamma))",
                     "sweeps": n_sw, "final_norm": nrm, "ms": solve_ms[1],
                     "first_call_ms": solve_ms[0],
                     "us_per_sweep": solve_ms[1] * 1e3 / max(1, n_sw),
                     "kernel": ("k_sweep_resident" if coded and steps_per_launch >= RESIDENT_STEPS
                                else "k_mdp_sweep_coded" if coded else "k_mdp_sweep")}
    ctx.belief_set(b0[r0 * gw:r1 * gw])
    ctx.mdp_reset()
    ctx.synchronize()
    legs_ms = (time.perf_counter() - legs_t0) * 1e3

    # ---------------------------------------------------------------- warmup
    ctx.loop_run(us[:args.warmup], zs[:args.warmup])
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # ---------------------------------------------------------------- timed
    # The trajectory's arguments are converted before the region (a compiled
    # client's call: pp2_loop_run and nothing else); the HIP events of the
    # same launch are taken in a second, untimed run of the same steps.
    run_timed = ctx.loop_launcher(us[args.warmup:total], zs[args.warmup:total])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_timed()
    enqueue_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    if ws > 1:  # (one rank: the synchronize above already closes the region)
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    value = gh * gw * args.steps / elapsed
    # sanity: the belief is still a distribution (checks the timed work ran)
    mass_ok = None
    if rank == 0 and ws == 1:
        bsum = float(ctx.belief_get().astype(np.float64).sum())
        mass_ok = abs(bsum - 1.0) < 1e-4

    if args.profile:
        if rank == 0:
            print(json.dumps({"profile_run": True, "steps": args.steps,
                              "ms_per_step": 1e3 * elapsed / args.steps}))
        ctx.close()
        if ws > 1:
            dist.destroy_process_group()
        return

    # the same launch between HIP events (untimed; b and J continue from the
    # timed steps, which changes neither the work nor its bytes; skipped with
    # --profile, so a profile holds the timed region's launches only)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    ev0.record(stream)
    run_timed()
    ev1.record(stream)
    torch.cuda.synchronize()
    loop_ms_events = ev0.elapsed_time(ev1) / args.steps
    # N > 1: the timed call's RCCL rounds, event-timed in one more run
    head_rounds = comm_round_stats(ctx, run_timed, torch, dist) if ws > 1 else None

    # the resident kernel's duration per launch for the roofline: launches of
    # the timed region's length back to back, so the host enqueue of one
    # overlaps the previous (the timed region's events also hold its single
    # enqueue; rocprof's per-dispatch average is the comparable figure)
    res_launch_us = None
    if coded and steps_per_launch >= RESIDENT_STEPS:
        n_l = -(-args.steps // -(-args.steps // RESIDENT_STEPS))
        n_rep = 10
        e0.record(stream)
        for _ in range(n_rep):
            ctx.loop_run(us[:n_l], zs[:n_l])
        e1.record(stream)
        torch.cuda.synchronize()
        res_launch_us = e0.elapsed_time(e1) / n_rep * 1e3
    # a row shard (N >= 2) runs resident launches of up to e steps on its view
    shard_res = ws > 1 and coded and ctx.resident_tiling()[0] > 0
    ctx.close()

    bytes_loop = BYTES_LOOP_CODED if coded else BYTES_LOOP
    bytes_sweep = BYTES_SWEEP_CODED if coded else BYTES_SWEEP
    resident = steps_per_launch >= RESIDENT_STEPS
    loop_kernel = ("k_loop_resident" if resident or shard_res else
                   "k_loop_pair_coded" if steps_per_launch == 2 else "k_loop_step_coded") \
        if coded else "k_loop_step"
    # the resident loop runs the whole timed trajectory in ceil(steps / 2048) launches
    spl = (args.steps / -(-args.steps // RESIDENT_STEPS)) if resident else steps_per_launch
    lds_bytes = LDS_BYTES_LOOP_RESIDENT if resident else LDS_BYTES_LOOP_CODED
    # a resident sweep launch moves its 11 B/cell once for all `reps` sweeps
    sweep_res = coded and resident
    sweep_gbs = bytes_sweep * cells_per_gpu / ((sweep_ms * (reps if sweep_res else 1)) * 1e-3) / 1e9
    bytes_belief = BYTES_BELIEF_CODED if coded else BYTES_BELIEF
    belief_gbs = bytes_belief * cells_per_gpu / (belief_ms * 1e-3) / 1e9
    # one launch = spl steps; its average duration: back-to-back resident
    # launches (above), else the timed region's events
    launch_s = res_launch_us * 1e-6 if res_launch_us else loop_ms_events * 1e-3 * spl
    algo_launch = bytes_loop * cells_per_gpu  # bytes the kernel must move per launch
    loop_gbs = algo_launch / launch_s / 1e9
    contract_gbs = BYTES_LOOP * cells_per_gpu / (loop_ms_events * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(loop_kernel, cells_per_gpu,
                                       exclude=None if coded else "coded",
                                       steps=round(spl) if resident else None) \
        if not shard_res else (None, "not collected for row-shard views")

    c4 = None
    if args.c4_size > 0:
        c4 = config4_leg(args, ws, rank, local, stream)

    result = None
    plan = None
    if rank == 0 and ws == 1 and args.plan_steps > 0:
        plan = plan_step_bench(args, local, stream.cuda_stream,
                               with_cpu=not args.no_cpu_baseline)
    pbvi = None
    if rank == 0 and ws == 1 and not args.no_pbvi:
        pbvi = pbvi_bench(args, local, stream.cuda_stream, with_cpu=not args.no_cpu_baseline)
    weak = None
    if rank == 0 and ws == 1 and not strong and args.shard_rows > 0:
        weak = weak_rank_share(args, local, stream, value)
    rollout = None
    if rank == 0 and ws == 1 and args.rollout_copies > 0:
        rollout = rollout_bench(args, local, stream)
    if rank == 0:
        cpu = None
        if ws == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(grid, goal, us, zs, args.cpu_seconds)
        result = {
            "metric": "grid cells/sec for belief-update+Bellman loop, 1024x1024; plan step p50 ms",
            "value": value,
            "unit": "cells/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic: splitmix64 occupancy grid (p_occ=0.2, seed=H), "
                    "uniform initial belief, seeded simulated (u,z) trajectory",
            "config": {
                "workload": (f"{gh}x{gw} grid row-sharded over {ws} GPU(s): 1 belief update + "
                             f"1 MDP Bellman sweep per step" if strong else
                             f"{r1 - r0}x{args.size} cells per GPU: 1 belief update + 1 MDP "
                             f"Bellman sweep per step (BASELINE.json configs[2] grid"
                             + (")" if ws == 1 else f"; {r1 - r0}-row shards so that each "
                                f"rank's view with its halo rows is one tile per CU)")),
                "grid": [gh, gw],
                "rows_per_gpu": r1 - r0,
                "parallelism": (f"row-shard x{ws}: tile-resident launches of up to e steps, "
                                f"each after one RCCL exchange of e halo rows and a "
                                f"{{mass, shift}} all-reduce (e = {(args.size - (r1 - r0)) // 2})"
                                if ws > 1 else "single GPU"),
                "cells_per_lane": args.cpt,
                "model": (f"dictionary-coded ({dict_entries} entries, uint16 code per cell)"
                          if coded else "dense fp32 planes"),
            },
            "roofline": {
                "kernel": (f"{loop_kernel} (the whole timed trajectory, {args.steps} fused loop "
                           f"steps, in one launch: one tile of rows per CU resident in LDS)"
                           if resident else
                           f"{loop_kernel} (row-shard view of the owned rows + e halo rows: "
                           f"launches of up to e = {steps_per_launch} steps, each after one RCCL "
                           f"halo exchange and {{mass, shift}} all-reduce)" if shard_res else
                           f"{loop_kernel} (two fused loop steps per launch: belief update + "
                           f"MDP Bellman sweep, twice)" if spl == 2 else
                           f"{loop_kernel} (fused belief update + MDP Bellman sweep)"),
                # the resident kernel moves its bytes once per launch: its
                # period is the per-step hand-off latency chain, with HBM, LDS
                # and VALU all below saturation (sq_counters); the others are
                # HBM-priced
                "bound": "latency" if (resident or shard_res) and coded else "hbm",
                "sq_counters": sq_counters() if resident and coded else None,
                "achieved": loop_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": loop_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_over_algorithmic": (traffic / algo_launch if traffic else None),
                "steps_per_launch": spl,
                "algorithmic_bytes_per_cell_per_launch": bytes_loop,
                "algorithmic_bytes_per_launch": algo_launch,
                "avg_launch_us": launch_s * 1e6,
                "note": ("bytes the resident kernel must move per launch: code 2, b 4, J 4 in, "
                         "b' 4, J' 4, A 1 out per cell; every intermediate step stays in LDS, so "
                         "HBM is not the binding resource: the per-step edge-row hand-off chain "
                         "is, with VALU and LDS about half busy (sq_counters, roofline_lds; "
                         "DESIGN.md §3.2). `traffic` is the memory-side bytes (2*FETCH_SIZE + "
                         "WRITE_SIZE) per launch; above the algorithmic bytes are the edge-row "
                         "hand-off granules that cross an XCD boundary (sc1 stores and loads, "
                         "past L2 to the memory side; same-XCD hand-offs are plain stores that "
                         "stay in L2), not cell data"
                         if (resident or shard_res) and coded else
                         "bytes the coded kernel must move per launch: code 2, b 4, b' 4, J 4, "
                         "J' 4, A 1 per cell (a pair launch keeps its intermediate step in "
                         "LDS); launch-latency and LDS bound, see roofline_lds"
                         if coded else "dense planes: SURVEY.md §8(d) fp32 tensor contract"),
            },
            "contract_equivalent": {
                "bytes_per_cell_step": BYTES_LOOP,
                "GBps": contract_gbs,
                "frac_of_hbm_peak": contract_gbs / HBM_PEAK_GBS,
                "note": ("the loop's throughput priced on the reference's fp32 tensor contract "
                         "(SURVEY.md §8(d): T, C, T_u, L_z read per cell, 417 B/cell-step); the "
                         "coded kernel does not move these bytes, so this can exceed 1 and is "
                         "not a roofline fraction -- the 11.5 G cells/s target of BASELINE.md "
                         "is 60 % of 8 TB/s / 417 B"),
            },
            "roofline_lds": ({
                "achieved": lds_bytes * cells_per_gpu / (loop_ms_events * 1e-3) / 1e9,
                "peak": LDS_PEAK_GBS, "unit": "GB/s",
                "frac": lds_bytes * cells_per_gpu / (loop_ms_events * 1e-3) / 1e9
                / LDS_PEAK_GBS,
                "bytes_per_cell": lds_bytes} if coded else None),
            "sweep_resident_traffic": sweep_resident_traffic(cells_per_gpu),
            "dense_path": dense,
            "rccl_round_us": head_rounds,
            "config4": c4,
            "weak_rank_share": weak,
            "kernels": {
                "mdp_sweep_kernel": (("k_sweep_resident (all the timed sweeps in one launch; "
                                      "gbs/frac count its 11 B/cell once per launch)")
                                     if coded and resident else
                                     "k_mdp_sweep_coded" if coded else "k_mdp_sweep"),
                "mdp_sweep_us": sweep_ms * 1e3,
                "mdp_sweep_gbs": sweep_gbs,
                "mdp_sweep_frac": sweep_gbs / HBM_PEAK_GBS,
                "belief_update_kernel": ("k_loop_step_coded without its sweep + k_sum_finalize "
                                         "(10 B/cell: code, b, b')" if coded else
                                         "k_belief_update + k_sum_finalize (48 B/cell)"),
                "belief_update_us": belief_ms * 1e3,
                "belief_update_gbs": belief_gbs,
                "belief_update_frac": belief_gbs / HBM_PEAK_GBS,
                "loop_step_us_events": loop_ms_events * 1e3,
                "loop_step_us_step_pairs": (pairs_ms * 1e3 if pairs_ms else None),
                "loop_enqueue_us_per_step": 1e6 * enqueue_s / args.steps,
                "loop_gbs": loop_gbs,
                "loop_frac": loop_gbs / HBM_PEAK_GBS,
            },
            "fib_sweep": fib,
            "headline_after": {
                "secondary_legs_ms": legs_ms,
                "note": "the per-kernel timings, FIB sweeps, dense path and MDP solve run before "
                        "the warmup + timed steps (then belief and values are reset), so the "
                        "timed steps run at the GPU's working clock; a GPU fresh out of idle "
                        "runs the same 20-step launch ~8 % slower (tools/micro/clock_warmup.py, "
                        "profiles/r03/clock_warmup.txt)"},
            "belief_mass_ok": mass_ok,
            "mdp_solve": mdp_solve,
            "plan_step": plan,
            "rollout": rollout,
            "pbvi": pbvi,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result))
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
