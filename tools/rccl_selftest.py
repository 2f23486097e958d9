"""RCCL shard-path self test: N ranks (torch.distributed.run) on the GPUs
given by PP2_DEVICES (comma list, default = local rank), row-sharded loop
steps over RCCL, compared on rank 0 with an unsharded context.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_selftest.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    ws = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    devs = os.environ.get("PP2_DEVICES")
    dev = int(devs.split(",")[local]) if devs else local
    dist.init_process_group("gloo")
    N = int(os.environ.get("PP2_N", "256"))
    steps = 6
    grid = S.synth_grid(N, N, N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, steps, seed=42)
    b0 = S.uniform_belief(grid)
    bounds = np.linspace(0, N, ws + 1).astype(int)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    ctx = P.GridContext(grid, goal, device=dev, rows=(r0, r1))
    uid = [P.GridContext.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    ctx.shard_comm_init(uid[0], ws, rank)
    ctx.model_generate()
    ctx.belief_set(b0[r0 * N:r1 * N])
    ctx.mdp_reset()
    for k in range(steps):
        ctx.loop_step(us[k], zs[k])
    ctx.mdp_sweep(2)
    b = ctx.belief_get()
    J, A = ctx.mdp_get()
    sweeps, norm = ctx.mdp_solve(max_sweeps=200)
    J2, _ = ctx.mdp_get()
    parts = [None] * ws
    dist.all_gather_object(parts, (b, J, A, J2, sweeps, norm))
    if rank == 0:
        bs = np.concatenate([p[0] for p in parts])
        Js = np.concatenate([p[1] for p in parts])
        As = np.concatenate([p[2] for p in parts])
        J2s = np.concatenate([p[3] for p in parts])
        with P.GridContext(grid, goal, device=dev) as ref:
            ref.model_generate()
            ref.belief_set(b0)
            ref.mdp_reset()
            ref.loop_run(us, zs)
            ref.mdp_sweep(2)
            rb = ref.belief_get()
            rJ, rA = ref.mdp_get()
            rs, rn = ref.mdp_solve(max_sweeps=200)
            rJ2, _ = ref.mdp_get()
        err = np.abs(bs.astype(np.float64) - rb) / np.maximum(np.abs(rb), 1e-30)
        ok = bool(np.array_equal(Js, rJ) and np.array_equal(As, rA) and
                  np.array_equal(J2s, rJ2) and (err[rb > 0].max() <= 1e-5) and
                  all(p[4] == rs for p in parts) and all(p[5] == rn for p in parts))
        print(f"RCCL selftest ws={ws} N={N}: values/actions bit-exact="
              f"{np.array_equal(Js, rJ) and np.array_equal(As, rA)}, solve bit-exact="
              f"{np.array_equal(J2s, rJ2)}, belief max rel err={err[rb > 0].max():.2e} -> "
              f"{'PASS' if ok else 'FAIL'}", flush=True)
        if not ok:
            sys.exit(1)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
