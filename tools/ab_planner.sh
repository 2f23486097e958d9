#!/bin/bash
# Same-box A/B of the 256^2 plan step (tools/prof_planner.py) across library
# builds (tools/_var/*.so vs the in-tree one), interleaved three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_planner.txt
: > $OUT
for rep in 1 2 3; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    echo "== $lib rep $rep" >> $OUT
    PP2_LIBRARY=$PWD/$lib timeout -k 10 120 python3 tools/prof_planner.py 2>/dev/null | grep "plan steps" >> $OUT || exit 1
  done
done
cat $OUT
