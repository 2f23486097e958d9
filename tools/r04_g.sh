#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fchain.py tests/test_gpu_planner.py -x -q --timeout 150 --timeout-method thread \
  -p no:cacheprovider > $O/r04_t8.log 2>&1 || { tail -40 $O/r04_t8.log; exit 1; }
tail -2 $O/r04_t8.log
timeout -k 10 60 python3 tools/fchain_timing.py || exit 1
for i in 1 2; do PP2_REF=1 PP2_STEPS=200 timeout -k 10 120 python3 tools/prof_planner.py || exit 1; done
