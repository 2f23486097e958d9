"""CPU: `bench.py --gpus N` (N > 1) started without a launcher starts the
N-rank torch.distributed.run job as a child process, relays rank 0's JSON
line and exits with the child's code; a world-size-1 invocation stays in
process.  --launcher-selftest makes the ranks join a gloo group and
all-reduce one value, so nothing here touches a GPU."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
              "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    return env


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_launcher_cmd_shape():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "5"], 8, 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29999"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert cmd[-5] == os.path.abspath(BENCH)


def test_two_ranks_without_launcher_start_a_child_job():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launcher-selftest"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "starting 2 ranks" in r.stderr
    res = _json_line(r.stdout)
    assert res == {"launcher_selftest": True, "world_size": 2, "rank_sum": 3.0,
                   "launched_by": "torch.distributed.run"}


def test_one_rank_stays_in_process():
    r = subprocess.run([sys.executable, BENCH, "--launcher-selftest"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "starting" not in r.stderr
    res = _json_line(r.stdout)
    assert res["world_size"] == 1 and res["launched_by"] == "direct"


def test_child_exit_code_is_relayed():
    # WORLD_SIZE set but not matching --gpus: the ranks refuse, and the parent
    # returns their failure
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launcher-selftest"],
                       cwd=ROOT, env={**_env(), "PP2_BENCH_FORCE_FAIL": "1"},
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
