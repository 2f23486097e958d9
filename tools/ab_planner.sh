#!/bin/bash
# Same-box A/B of the 256^2 plan step (tools/prof_planner.py) across library
# builds (tools/_var/*.so vs the in-tree one) and PP2_CDF_SKIP=0/1 (the
# in-tree planner's zero-block skip in the host cdf), interleaved three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_planner.txt
: > $OUT
for rep in 1 2 3; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    for skip in 1 0; do
      echo "== $lib PP2_CDF_SKIP=$skip rep $rep" >> $OUT
      PP2_CDF_SKIP=$skip PP2_LIBRARY=$PWD/$lib timeout -k 10 120 python3 tools/prof_planner.py 2>/dev/null | grep "plan steps" >> $OUT || exit 1
    done
  done
done
cat $OUT
