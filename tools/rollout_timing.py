"""bench.py's rollout leg alone (BASELINE configs[4]: 512^2, 4096 copies x
depth 5, fp16), for same-box A/B of library builds (PP2_LIBRARY)."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    stream = torch.cuda.Stream()
    args = types.SimpleNamespace(rollout_size=512, rollout_copies=4096, rollout_depth=5)
    r = bench.rollout_bench(args, 0, stream)
    print(f"{os.environ.get('PP2_LIBRARY', 'in-tree')}: {r['ms_per_rollout']:.3f} ms, "
          f"{r['algorithmic_GBps']:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
