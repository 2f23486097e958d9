#!/bin/bash
# Round-4 checks: full GPU suite, smoke, driver-style bench, rocprof of the
# bench, rocprof of reference-order plan steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --profile --steps 20 --warmup 20 > $OUT/prof.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log
cat $OUT/smoke.log | tail -3
echo "exit=$rc"
exit $rc
