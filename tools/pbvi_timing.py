"""Time PBVI phases on the GPU: belief-set expansion and backup iterations.

    python tools/pbvi_timing.py [--maps sparse_map_100x40,synth256] [--S 500] [--iters 5]
Prints one JSON line per map.  Run under rocprofv3 --kernel-trace --stats for
the per-kernel split."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402


def grid_of(name):
    from path_planning_2d_amd import synthetic as S
    if name.startswith("synth"):
        n = int(name[5:])
        g = S.synth_grid(n, n, n)
        return g, S.synth_goal(g)
    from conftest import golden, golden_map
    return golden_map(name), tuple(golden("model", name)["goal"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--maps", default="sparse_map_100x40,synth256")
    ap.add_argument("--S", type=int, default=500)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import path_planning_2d_amd as P
    from path_planning_2d_amd import synthetic as S
    for name in a.maps.split(","):
        g, goal = grid_of(name)
        with P.GridContext(g, goal, gamma=0.95) as ctx:
            ctx.model_generate()
            b0 = S.uniform_belief(g)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.pbvi_belief_set(b0, a.S)
            ctx.synchronize()
            t_set = time.perf_counter() - t0
            ctx.pbvi_backup(1)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.pbvi_backup(a.iters)
            ctx.synchronize()
            t_it = (time.perf_counter() - t0) / a.iters
            hw = g.size
            Sp = (a.S + 127) // 128 * 128
            gemm_flop = 2.0 * 144 * Sp * Sp * ((hw + 31) // 32 * 32)
            print(json.dumps({"map": name, "H": g.shape[0], "W": g.shape[1], "S": a.S,
                              "belief_set_s": round(t_set, 4),
                              "backup_iter_ms": round(t_it * 1e3, 3),
                              "backup_167_s": round(t_it * 167, 3),
                              "gemm_tflop_per_iter": gemm_flop / 1e12,
                              "iter_tflops_gemm_equiv": round(gemm_flop / t_it / 1e12, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
