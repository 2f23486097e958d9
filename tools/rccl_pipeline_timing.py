"""Per-step time of the RCCL row-shard loop pipeline on one GPU (a full-grid
shard with a 1-rank communicator: comm stream, events, async mass
all-reduce, deep-halo views; no neighbour transfers) against the plain loop,
at 1024^2.  A lower bound for the multi-GPU per-step cost."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = int(os.environ.get("PP2_N", "1024"))
    reps = 200
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, reps, seed=42)
    stream = torch.cuda.Stream()
    modes = os.environ.get("PP2_MODES", "plain,rccl1,rccl1-depth2,rccl1-depth1,rccl1-cs").split(",")
    for mode in modes:
        kw = {} if mode == "plain" else {"rows": (0, N)}
        with P.GridContext(grid, goal, gamma=0.95, **kw) as ctx:
            ctx.set_stream(stream.cuda_stream)
            if mode != "plain":
                ctx.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
                if "-depth" in mode:
                    ctx.set_tuning(ctx.TUNE_HALO_DEPTH, int(mode.split("-depth")[1]))
                if "-cs" in mode:
                    ctx.set_tuning(ctx.TUNE_COMM_STREAM, 1)
            ctx.model_generate()
            ctx.belief_set(S.uniform_belief(grid))
            ctx.mdp_reset()
            ctx.loop_run(us[:20], zs[:20])
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            ctx.loop_run(us, zs)
            e1.record(stream)
            torch.cuda.synchronize()
            print(f"{mode:14s} {e0.elapsed_time(e1) / reps * 1e3:7.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
