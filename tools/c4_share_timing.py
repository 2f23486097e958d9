"""Config 4's per-rank share alone (bench.config4_rank_share: rank 3 of 8,
rows [768, 1024) x 2048 of the 2048^2 grid on a 1-rank RCCL communicator,
16 warm-up + 200 timed loop steps), and the unsharded 1024^2 loop (20-step
resident launches), on the library PP2_LIBRARY points at -- for same-box A/B
of builds (tools/ab_builds.sh).  Prints us per step (median of PP2_REPS runs)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import bench
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    reps = int(os.environ.get("PP2_REPS", "3"))
    lib = os.path.basename(os.environ.get("PP2_LIBRARY", "in-tree"))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    G, w, k = 2048, 16, 200
    grid = S.synth_grid(G, G, seed=G)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, w + k, seed=42)
    b0 = S.uniform_belief(grid)
    r0, r1 = 3 * G // 8, 4 * G // 8
    share = []
    for _ in range(reps):
        ctx = P.GridContext(grid, goal, gamma=bench.GAMMA, device=0, rows=(r0, r1))
        ctx.set_stream(stream.cuda_stream)
        ctx.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
        ctx.model_generate()
        ctx.belief_set(b0[r0 * G:r1 * G])
        ctx.mdp_reset()
        ctx.loop_run(us[:w], zs[:w])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.loop_run(us[w:], zs[w:])
        torch.cuda.synchronize()
        share.append(1e6 * (time.perf_counter() - t0) / k)
        tiling = ctx.resident_tiling()
        J, A = ctx.mdp_get()
        ctx.close()
    N = 1024
    g1 = S.synth_grid(N, N, seed=N)
    u1, z1, _ = S.synth_trajectory(g1, 40, seed=42)
    with P.GridContext(g1, S.synth_goal(g1), gamma=bench.GAMMA, device=0) as c1:
        c1.set_stream(stream.cuda_stream)
        c1.model_generate()
        c1.belief_set(S.uniform_belief(g1))
        c1.mdp_reset()
        c1.loop_run(u1[:20], z1[:20])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        loop = []
        for _ in range(reps):
            e0.record(stream)
            for _ in range(10):
                c1.loop_run(u1[:20], z1[:20])
            e1.record(stream)
            torch.cuda.synchronize()
            loop.append(e0.elapsed_time(e1) * 1e3 / 200)
    jsum = float(np.asarray(J, np.float64).sum())
    print(f"{lib}: c4 rank share {np.median(share):.3f} us/step (runs {', '.join(f'{v:.3f}' for v in share)}), "
          f"tiling {tiling}, J checksum {jsum:.6e}; 1024^2 loop {np.median(loop):.3f} us/step", flush=True)


if __name__ == "__main__":
    main()
