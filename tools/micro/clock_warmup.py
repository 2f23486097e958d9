"""Does a lone 20-step resident launch run slower on a GPU that was idle
before it?  Event-timed lone launches (host sync between them) in order:
after the setup, after an idle pause, and right after ~N ms of busy GPU work
(back-to-back resident launches), at 1024^2."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 2048, seed=42)
    stream = torch.cuda.Stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.set_stream(stream.cuda_stream)
        ctx.model_generate()
        ctx.belief_set(S.uniform_belief(grid))
        ctx.mdp_reset()
        ctx.loop_run(us[:5], zs[:5])
        ctx.synchronize()

        def lone(n=20):
            torch.cuda.synchronize()
            e0.record(stream)
            ctx.loop_run(us[:n], zs[:n])
            e1.record(stream)
            stream.synchronize()
            ctx.synchronize()
            return e0.elapsed_time(e1) * 1e3

        def busy(ms):
            t0 = time.perf_counter()
            while (time.perf_counter() - t0) * 1e3 < ms:
                for _ in range(8):
                    ctx.loop_run(us[:200], zs[:200])
                ctx.synchronize()

        print("first lone launches after setup:", " ".join(f"{lone():.1f}" for _ in range(8)),
              flush=True)
        for pause in (0.05, 0.5):
            time.sleep(pause)
            print(f"after {pause * 1e3:.0f} ms idle:", " ".join(f"{lone():.1f}" for _ in range(4)),
                  flush=True)
        for ms in (5, 20, 100, 300):
            time.sleep(0.5)
            busy(ms)
            print(f"after {ms} ms busy:", " ".join(f"{lone():.1f}" for _ in range(4)), flush=True)
        print("200-step lone after 300 ms busy:", " ".join(f"{lone(200):.1f}" for _ in range(4)),
              flush=True)
        time.sleep(0.5)
        print("200-step lone after 500 ms idle:", " ".join(f"{lone(200):.1f}" for _ in range(4)),
              flush=True)


if __name__ == "__main__":
    main()
