"""Event-timed fused loop steps at 1024^2 (A/B of kernel variants)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    for N in [int(v) for v in os.environ.get("PP2_NS", os.environ.get("PP2_N", "1024")).split(",")]:
        for res in [int(v) for v in os.environ.get("PP2_RESIDENT", "1,0").split(",")]:
            one(N, res)


def one(N, resident):
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    reps = int(os.environ.get("PP2_REPS", "100"))
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, reps, seed=42)
    stream = torch.cuda.Stream()
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.set_stream(stream.cuda_stream)
        ctx.set_tuning(ctx.TUNE_STEP_PAIRS, int(os.environ.get("PP2_PAIRS", "1")))
        ctx.set_tuning(ctx.TUNE_RESIDENT, resident)
        ctx.model_generate()
        ctx.belief_set(S.uniform_belief(grid))
        ctx.mdp_reset()
        ctx.loop_run(us[:10], zs[:10])
        ctx.synchronize()
        print(f"N={N} resident={resident} steps/launch={ctx.loop_steps_per_launch()}", flush=True)
        for what in ("loop", "sweep"):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if what == "loop":
                ctx.loop_run(us, zs)
            else:
                ctx.mdp_sweep(reps)
            e1.record(stream)
            torch.cuda.synchronize()
            ctx.synchronize()
            print(f"{what}: {e0.elapsed_time(e1) / reps * 1e3:.2f} us/step", flush=True)
        import time
        ctx.mdp_reset()
        ctx.synchronize()
        t0 = time.perf_counter()
        n_sw, nrm = ctx.mdp_solve()
        ctx.synchronize()
        print(f"mdp_solve: {n_sw} sweeps, norm {nrm:.6g}, {1e3 * (time.perf_counter() - t0):.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
