"""Config 4's per-rank share (rank 3 of 8: rows [768, 1024) x 2048 of the
2048^2 grid on a 1-rank RCCL communicator, bench.config4_rank_share) for
several resident halo depths e (PP2_TUNE_RESIDENT_HALO), tilings
(PP2_TUNE_RESIDENT_TILE_COLS), normalisation blocks and lagged / waited
block starts (PP2_TUNE_SHARD_LAG): a smaller e shrinks the view (256 + 2e rows)
and the cells per CU, at the price of more launches and RCCL rounds per call.
Prints, per setting, e, the plan's steps per launch, the measured us per
step and the projection at the assumed 10 / 30 us RCCL round."""
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
    G = int(os.environ.get("PP2_G", "2048"))
    w, k = 16, int(os.environ.get("PP2_STEPS", "200"))
    grid = S.synth_grid(G, G, seed=G)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, w + k, seed=42)
    b0 = S.uniform_belief(grid)
    r0, r1 = 3 * G // 8, 4 * G // 8
    stream = torch.cuda.Stream()
    # cases "e:tile cols:norm block:lag" (PP2_TUNE_RESIDENT_HALO, _TILE_COLS --
    # 3 = transposed tiles --, _NORM_BLOCK (0: default 8), _SHARD_LAG)
    spec = os.environ.get("PP2_CASES", "128:0:0:0,128:3:0:0,128:3:0:1,128:3:4:0,64:2:0:0,128:0:0:0")
    cases = [tuple(int(v) for v in c.split(":")) for c in spec.split(",")]
    for e_req, tc, nb, lag in cases:
        if True:
            ctx = P.GridContext(grid, goal, gamma=bench.GAMMA, device=0, rows=(r0, r1))
            ctx.set_stream(stream.cuda_stream)
            ctx.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
            ctx.set_tuning(P.GridContext.TUNE_RESIDENT_HALO, e_req)
            if tc:
                ctx.set_tuning(P.GridContext.TUNE_RESIDENT_TILE_COLS, tc)
            if nb:
                ctx.set_tuning(P.GridContext.TUNE_NORM_BLOCK, nb)
            ctx.set_tuning(P.GridContext.TUNE_SHARD_LAG, lag)
            ctx.model_generate()
            ctx.belief_set(b0[r0 * G:r1 * G])
            ctx.mdp_reset()
            ctx.synchronize()
            e = ctx.loop_steps_per_launch()
            tiling = ctx.resident_tiling()
            ts = []
            for rep in range(3):
                ctx.loop_run(us[:w], zs[:w])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ctx.loop_run(us[w:], zs[w:])
                torch.cuda.synchronize()
                ts.append(1e6 * (time.perf_counter() - t0) / k)
            ctx.close()
            t = float(np.median(ts))
            rounds = -(-k // e) + 1 if e > 0 else 0
            proj = [t + rounds * r / k for r in bench.RCCL_ROUND_US]
            print(f"e_req {e_req:4d} tc {tc} norm {nb or 8} lag {lag} -> e {e:4d} tiling {tiling}: {t:6.3f} us/step "
                  f"(runs {', '.join(f'{x:.3f}' for x in ts)}), rounds {rounds}, "
                  f"projection {proj[0]:.3f}-{proj[1]:.3f} us/step", flush=True)


if __name__ == "__main__":
    main()
