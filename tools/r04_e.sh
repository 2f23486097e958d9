#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 60 python3 tools/fchain_timing.py > $O/r04_fct3.txt 2>&1 || { cat $O/r04_fct3.txt; exit 1; }
cat $O/r04_fct3.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fct -o run -- python3 tools/fchain_timing.py > $O/r04_prof_fct.log 2>&1
