"""Diagnostic: the bench's config4 rank-share leg in isolation -- rank 3's
256 x 2048 shard of the 2048^2 grid, 1-rank RCCL communicator, resident shard
path -- with a settle (synchronize + resident status) after every call, on
the context's own stream or on a torch stream (PP2_TORCH_STREAM=1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    G = int(os.environ.get("PP2_G", "2048"))
    r0, r1 = 3 * G // 8, 4 * G // 8
    grid = S.synth_grid(G, G, seed=G)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 216, seed=42)
    b0 = S.uniform_belief(grid)
    ctx = P.GridContext(grid, goal, gamma=0.95, device=0, rows=(r0, r1))
    if os.environ.get("PP2_TORCH_STREAM"):
        import torch
        st = torch.cuda.Stream()
        ctx.set_stream(st.cuda_stream)
    ctx.shard_comm_init(P.GridContext.rccl_unique_id(), 1, 0)
    if os.environ.get("PP2_HALO"):
        ctx.set_tuning(ctx.TUNE_RESIDENT_HALO, int(os.environ["PP2_HALO"]))
    ctx.model_generate()
    print("dict", ctx.model_dict_info(), "steps/launch", ctx.loop_steps_per_launch(), flush=True)
    ctx.belief_set(b0[r0 * G:r1 * G])
    ctx.mdp_reset()
    ctx.synchronize()
    for lo, hi in ((0, 16), (16, 216)):
        ctx.loop_run(us[lo:hi], zs[lo:hi])
        try:
            ctx.synchronize()
            print(f"steps [{lo},{hi}): ok, launches {ctx.resident_launches()}, "
                  f"status {ctx.resident_status()}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"steps [{lo},{hi}): {e}", flush=True)
            break
    print("mass", float(ctx.belief_get().astype(np.float64).sum()), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
