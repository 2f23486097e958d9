#!/bin/bash
# rocprofv3 kernel stats + HBM PMC counters for the bench workload.
# Counters are collected in their own passes (FETCH_SIZE, then WRITE_SIZE),
# with no tracing domains beside --pmc (MI355X_MICROARCH.md §rocprofv3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_DIR:-.}
ARGS="--profile --steps ${STEPS:-20} --warmup ${WARMUP:-20} ${EXTRA:-}"
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $ARGS > $OUT/prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
