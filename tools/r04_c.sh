#!/bin/bash
# Round 4: kernel trace of config 4's rank share (2-D tiles, e = 128; and
# e = 64): per-launch kernel time against the call's wall time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
PP2_CASES="128:0:0:0,64:2:0:0" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 tools/c4_halo_sweep.py > $O/r04_prof_c4.log 2>&1
rc=$?
grep -E "us/step" $O/r04_prof_c4.log
exit $rc
