#!/bin/bash
# Round-3 evidence pass: HBM PMC of the bench workload, SQ counters of the
# resident loop kernel, and the resident launch fixed cost (plain and under a
# kernel trace, so the event span can be split into kernel time and gaps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
bash tools/collect_pmc.sh &&
PP2_RESIDENT=1 PP2_REPS=200 bash tools/collect_lds_pmc.sh &&
timeout -k 10 120 python3 tools/resident_launch_timing.py > $OUT/launch_timing.txt 2>&1 &&
PP2_REPS=5 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/launch_prof -o run -- python3 tools/resident_launch_timing.py > $OUT/launch_prof.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
