#!/bin/bash
# FIB sweep evidence: rocprofv3 kernel stats of tools/fib_timing.py, then its
# SQ counters (tools/fib_sq.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fib_prof -o run -- python3 tools/fib_timing.py > gpurun_out/fib_prof.log 2>&1 &&
bash tools/fib_sq.sh
