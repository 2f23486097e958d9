"""Diagnostic: sweeps and wall time of the 1024^2 MDP solve (ctx.mdp_solve)
fresh and after each other path has touched the context (resident loop,
sweeps, single belief updates, the pair loop, the dense model) -- a solve
must not depend on what ran before it."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import path_planning_2d_amd as P
from path_planning_2d_amd import synthetic as S
N = 1024
grid = S.synth_grid(N, N, seed=N); goal = S.synth_goal(grid)
us, zs, _ = S.synth_trajectory(grid, 200, seed=42)
stream = torch.cuda.Stream(); torch.cuda.set_stream(stream)
ctx = P.GridContext(grid, goal, gamma=0.95)
ctx.set_stream(stream.cuda_stream)
ctx.model_generate(); ctx.belief_set(S.uniform_belief(grid)); ctx.mdp_reset(); ctx.synchronize()
def solve(tag):
    ctx.mdp_reset(); torch.cuda.synchronize()
    t0 = time.perf_counter(); n, nrm = ctx.mdp_solve(); torch.cuda.synchronize()
    print(tag, n, nrm, f"{1e3*(time.perf_counter()-t0):.3f} ms", ctx.resident_launches(), flush=True)
solve("fresh")
ctx.loop_run(us[:25], zs[:25]); torch.cuda.synchronize()
solve("after loop")
ctx.mdp_sweep(100); torch.cuda.synchronize()
solve("after sweeps")
for k in range(100): ctx.belief_update(int(us[k]), int(zs[k]))
torch.cuda.synchronize()
solve("after belief updates")
ctx.set_tuning(ctx.TUNE_RESIDENT, 0); ctx.loop_run(us[:100], zs[:100]); ctx.set_tuning(ctx.TUNE_RESIDENT, 1); torch.cuda.synchronize()
solve("after pairs")
ctx.set_tuning(ctx.TUNE_CODED_MODEL, 0); ctx.loop_run(us[:100], zs[:100]); ctx.mdp_sweep(100); ctx.set_tuning(ctx.TUNE_CODED_MODEL, 1); torch.cuda.synchronize()
solve("after dense")
solve("again")
