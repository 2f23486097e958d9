#!/bin/bash
# Quick GPU iteration: coded-path parity tests, then loop / sweep timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_coded.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_shards.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_quick.log 2>&1 &&
for n in 1024 2048 512; do PP2_N=$n timeout -k 10 60 python3 tools/coded_loop_timing.py; done > $OUT/timing.txt 2>&1
rc=$?
tail -3 $OUT/pytest_quick.log
cat $OUT/timing.txt
exit $rc
