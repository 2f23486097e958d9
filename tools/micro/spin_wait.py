"""Host wall time of a lone 20-step resident launch (enqueue .. device
synchronize) against its event span, with the HIP runtime's default wait
(PP2_SPIN=0) or hipDeviceScheduleSpin set before the device is touched
(PP2_SPIN=1), on a warm GPU at 1024^2."""
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    spin = os.environ.get("PP2_SPIN", "0") == "1"
    if spin:
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipSetDevice(0) == 0
        rc = hip.hipSetDeviceFlags(1)  # hipDeviceScheduleSpin
        print("hipSetDeviceFlags(spin) ->", rc, flush=True)
    import torch
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    N = 1024
    grid = S.synth_grid(N, N, seed=N)
    goal = S.synth_goal(grid)
    us, zs, _ = S.synth_trajectory(grid, 2048, seed=42)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    with P.GridContext(grid, goal, gamma=0.95) as ctx:
        ctx.set_stream(stream.cuda_stream)
        ctx.model_generate()
        ctx.belief_set(S.uniform_belief(grid))
        ctx.mdp_reset()
        for _ in range(40):  # warm the GPU clock
            ctx.loop_run(us[:200], zs[:200])
        ctx.synchronize()
        e0.record(stream)
        e1.record(stream)
        wall, ev = [], []
        for r in range(30):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(stream)
            ctx.loop_run(us[:20], zs[:20])
            e1.record(stream)
            torch.cuda.synchronize()
            wall.append((time.perf_counter() - t0) * 1e6)
            ev.append(e0.elapsed_time(e1) * 1e3)
        m = statistics.median
        print(f"spin={int(spin)}: 20-step lone launch wall {m(wall):.1f} us, events {m(ev):.1f} us, "
              f"wall - events {m(wall) - m(ev):.1f} us", flush=True)


if __name__ == "__main__":
    main()
