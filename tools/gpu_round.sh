#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the
# script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEP=${1:-all}
run_tests() { timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; }
run_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; }
run_bench() { timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; }
run_prof()  { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --profile --steps 20 --warmup 20 > $OUT/prof.log 2>&1 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_roll -o run -- python3 tools/prof_rollout.py > $OUT/prof_roll.log 2>&1; }
case $STEP in
  all)   run_tests && run_smoke && run_bench && run_prof ;;
  tests) run_tests ;;
  bench) run_bench ;;
  prof)  run_prof ;;
  quick) run_smoke && run_bench ;;
esac
rc=$?
echo "exit=$rc"
exit $rc
