"""GPU, >= 2 devices: the RCCL row-shard path across processes.

bench.py's config4 leg (BASELINE.json configs[3]) row-shards the 2048^2 grid
over the ranks of a torch.distributed.run job -- one process per GPU, RCCL
halo exchange and mass all-reduce over xGMI -- then gathers J, A and the
belief to rank 0 and compares them with the unsharded grid run on rank 0's GPU
(J/A bit for bit, belief rel 1e-5).  This test runs `bench.py --gpus 2` WITHOUT a launcher (bench.py starts
torch.distributed.run as a child) and asserts the gate passed and the RCCL
rounds were event-timed.  RCCL refuses two ranks on one device, so on a
1-GPU box it is skipped (the single-process shard group, test_gpu_shards.py,
covers the decomposition there).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_two_rank_rccl_config4_parity():
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs (RCCL rejects two ranks on one device)")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    # no launcher: bench.py itself starts torch.distributed.run as a child
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "16",
           "--warmup", "8", "--c4-steps", "24", "--c4-warmup", "8", "--kernel-reps", "8",
           "--plan-steps", "0", "--no-pbvi", "--rollout-copies", "0", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    c4 = res["config4"]
    assert c4["n_gpus"] == 2
    assert c4["parity"]["pass"], c4["parity"]
    assert c4["rccl_round_us"]["rounds"] >= 2, c4["rccl_round_us"]
    assert res["rccl_round_us"]["rounds"] >= 2, res["rccl_round_us"]
