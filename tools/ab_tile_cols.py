"""A/B on one GPU: the resident loop's whole-row tiles vs 2-D tiles
(PP2_TUNE_RESIDENT_TILE_COLS 1 / 2) on config 4's per-rank share at 8 ranks
(rows [768, 1024) x 2048 of the 2048^2 grid, a 1-rank RCCL communicator, views
of 256 + 2e rows), alternated over several rounds; plus the 1024^2 grid
(whole rows either way) as a control.  Prints us per step."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import path_planning_2d_amd as P  # noqa: E402
from path_planning_2d_amd import synthetic as S  # noqa: E402

G, K, W = 2048, 200, 16
grid = S.synth_grid(G, G, seed=G)
goal = S.synth_goal(grid)
us, zs, _ = S.synth_trajectory(grid, W + K, seed=42)
b0 = S.uniform_belief(grid)
r0, r1 = 3 * G // 8, 4 * G // 8
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)


def share():
    c = P.GridContext(grid, goal, gamma=0.95, device=0, rows=(r0, r1))
    c.set_stream(stream.cuda_stream)
    c.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
    c.model_generate()
    return c


def timed(c, reset):
    reset(c)
    c.loop_run(us[:W], zs[:W])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c.loop_run(us[W:], zs[W:])
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / K


def reset_share(c):
    c.belief_set(b0[r0 * G:r1 * G])
    c.mdp_reset()
    c.synchronize()


ctx = share()
res = {1: [], 2: []}
for rnd in range(int(os.environ.get("AB_ROUNDS", "6"))):
    for tc in (1, 2) if rnd % 2 == 0 else (2, 1):
        ctx.set_tuning(ctx.TUNE_RESIDENT_TILE_COLS, tc)
        tiling = ctx.resident_tiling()
        res[tc].append(timed(ctx, reset_share))
        assert ctx.resident_status()[0] == 0
print(f"rank share 256x2048 (view tiling {ctx.resident_tiling()}):")
for tc in (1, 2):
    v = np.array(res[tc])
    print(f"  tile cols {tc}: median {np.median(v):.3f} us/step  min {v.min():.3f}  all "
          + " ".join(f"{x:.2f}" for x in v))
ctx.close()

g2 = S.synth_grid(1024, 1024, seed=1024)
u2, z2, _ = S.synth_trajectory(g2, W + K, seed=42)
c2 = P.GridContext(g2, S.synth_goal(g2), gamma=0.95, device=0)
c2.set_stream(stream.cuda_stream)
c2.model_generate()
bb = S.uniform_belief(g2)
t = []
for _ in range(4):
    c2.belief_set(bb)
    c2.mdp_reset()
    c2.loop_run(u2[:W], z2[:W])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c2.loop_run(u2[W:], z2[W:])
    torch.cuda.synchronize()
    t.append(1e6 * (time.perf_counter() - t0) / K)
print(f"1024^2 control (tiling {c2.resident_tiling()}): median {np.median(t):.3f} us/step")
c2.close()
