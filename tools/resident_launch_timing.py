"""Fixed cost of one resident loop launch at 1024^2: host enqueue time of
pp2_loop_run, event-timed GPU span and host wall time (enqueue .. stream
sync) for runs of n steps, so the per-launch constant and the per-step slope
can be read off.  Beside it the enqueue time of a single belief update (a
small-kernarg launch) as the floor."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = int(os.environ.get("PP2_N", "1024"))
    reps = int(os.environ.get("PP2_REPS", "15"))
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 2048, seed=42)
    stream = torch.cuda.Stream()
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.set_stream(stream.cuda_stream)
        ctx.model_generate()
        if os.environ.get("PP2_NORM_BLOCK"):
            ctx.set_tuning(ctx.TUNE_NORM_BLOCK, int(os.environ["PP2_NORM_BLOCK"]))
        ctx.belief_set(S.uniform_belief(grid))
        ctx.mdp_reset()
        ctx.loop_run(us[:10], zs[:10])
        ctx.synchronize()
        print(f"N={N} steps/launch={ctx.loop_steps_per_launch()} "
              f"norm block {os.environ.get('PP2_NORM_BLOCK', 'default')}", flush=True)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        for n in [int(v) for v in os.environ.get("PP2_NS", "2,4,8,20,50,100,400,2000").split(",")]:
            enq, gpu, wall = [], [], []
            for r in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                e0.record(stream)
                ctx.loop_run(us[:n], zs[:n])
                t1 = time.perf_counter()
                e1.record(stream)
                stream.synchronize()
                t2 = time.perf_counter()
                ctx.synchronize()
                enq.append((t1 - t0) * 1e6)
                gpu.append(e0.elapsed_time(e1) * 1e3)
                wall.append((t2 - t0) * 1e6)
            m = statistics.median
            print(f"n={n:5d}: enqueue {m(enq):7.1f} us  events {m(gpu):8.1f} us "
                  f"({m(gpu) / n:5.2f}/step)  wall {m(wall):8.1f} us ({m(wall) / n:5.2f}/step)",
                  flush=True)
        # back-to-back calls (a controller issuing runs of n steps): K runs
        # queued without a host sync between them (the resident chain), one
        # event span and one host wall time over all of them
        K = int(os.environ.get("PP2_CHAIN", "12"))
        for n in [int(v) for v in os.environ.get("PP2_NS", "2,4,8,20,50,100,400,2000").split(",")]:
            gpu, wall = [], []
            for r in range(max(3, reps // 3)):
                ctx.synchronize()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                e0.record(stream)
                for k in range(K):
                    ctx.loop_run(us[:n], zs[:n])
                e1.record(stream)
                stream.synchronize()
                ctx.synchronize()
                wall.append((time.perf_counter() - t0) * 1e6)
                gpu.append(e0.elapsed_time(e1) * 1e3)
            m = statistics.median
            print(f"chained x{K} n={n:5d}: events {m(gpu) / (K * n):5.2f} us/step  "
                  f"wall {m(wall) / (K * n):5.2f} us/step", flush=True)
        enq = []
        for r in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.belief_update(int(us[r]), int(zs[r]))
            enq.append((time.perf_counter() - t0) * 1e6)
        ctx.synchronize()
        print(f"belief_update enqueue {statistics.median(enq):.1f} us", flush=True)


if __name__ == "__main__":
    main()
