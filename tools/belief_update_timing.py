"""pp2_belief_update alone at 1024^2 (the beliefCallback path: one update per
message, mass finalised), event-timed over 100 calls, for same-box A/B of
library builds (PP2_LIBRARY)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 200, seed=42)
    stream = torch.cuda.Stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.set_stream(stream.cuda_stream)
        ctx.model_generate()
        ctx.belief_set(S.uniform_belief(grid))
        for k in range(20):
            ctx.belief_update(int(us[k]), int(zs[k]))
        ctx.synchronize()
        best = None
        for rep in range(5):
            e0.record(stream)
            for k in range(100):
                ctx.belief_update(int(us[k]), int(zs[k]))
            e1.record(stream)
            stream.synchronize()
            t = e0.elapsed_time(e1) * 1e3 / 100
            best = t if best is None else min(best, t)
        print(f"{os.path.basename(os.environ.get('PP2_LIBRARY', 'in-tree'))}: belief_update "
              f"{best:.2f} us per call (best of 5 x 100)", flush=True)


if __name__ == "__main__":
    main()
