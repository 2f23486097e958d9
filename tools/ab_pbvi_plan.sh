#!/bin/bash
# Same-box A/B of the PBVI-leaf plan step (tools/pbvi_plan_timing.py) over
# library builds: the in-tree one and tools/_var/*.so, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_pbvi_plan.txt
: > $OUT
for rep in 1 2; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    PP2_LIBRARY=$PWD/$lib timeout -k 10 120 python3 tools/pbvi_plan_timing.py 2>/dev/null | grep "p50" >> $OUT || exit 1
  done
done
cat $OUT
