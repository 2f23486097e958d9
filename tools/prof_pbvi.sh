#!/bin/bash
# PBVI tests + timing + rocprof kernel stats (run via gpurun from the repo root).
# usage: tools/prof_pbvi.sh TAG
set -e
TAG=${1:-pbvi}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m pytest tests/test_gpu_pbvi.py -x -q -p no:cacheprovider > gpurun_out/gpu_pbvi.log 2>&1
timeout -k 10 300 python tools/pbvi_timing.py > gpurun_out/pbvi_timing.json 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python tools/pbvi_timing.py --iters 3 --maps synth256 > gpurun_out/pbvi_prof.log 2>&1
