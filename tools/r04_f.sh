#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_planner.py tests/test_gpu_ros_nodes.py -x -q --timeout 150 --timeout-method thread \
  -p no:cacheprovider > $O/r04_t7.log 2>&1 || { tail -40 $O/r04_t7.log; exit 1; }
tail -2 $O/r04_t7.log
for i in 1 2; do PP2_REF=1 PP2_STEPS=200 timeout -k 10 120 python3 tools/prof_planner.py || exit 1; done
PP2_REF=1 PP2_STEPS=30 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_plan5 -o run -- python3 tools/prof_planner.py > $O/r04_prof_plan5.log 2>&1
