#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_planner.py tests/test_gpu_pbvi.py tests/test_gpu_ros_nodes.py -x -q --timeout 150 --timeout-method thread \
  -p no:cacheprovider > $O/r04_t6.log 2>&1 || { tail -40 $O/r04_t6.log; exit 1; }
tail -2 $O/r04_t6.log
timeout -k 10 600 bash tools/ab_pbvi_plan.sh
