"""Per-rank work of the weak-scaling bench at N >= 2 (bench.weak_rank_share)
for several owned-row counts: the resident view is owned rows + 2e halo rows
<= 1024, so fewer owned rows buy deeper halos (fewer RCCL rounds per step)."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    stream = torch.cuda.Stream()
    n1 = float(os.environ.get("PP2_N1_CELLS_PER_S", "244e9"))  # N = 1 bench value
    for R in (768, 896, 960):
        args = types.SimpleNamespace(size=1024, shard_rows=R, warmup=20, steps=200)
        r = bench.weak_rank_share(args, 0, stream, n1)
        print(R, r["steps_per_launch"], round(r["measured_us_per_step"], 3),
              [round(x, 3) for x in r["projection"]["weak_efficiency_vs_n1"]], flush=True)


if __name__ == "__main__":
    main()
