#!/bin/bash
# Same-box A/B of the 256^2 plan step (tools/prof_planner.py) across library
# builds (tools/_var/*.so vs the in-tree one; chain sets by k_fc_walk, PP2_FX=0)
# and, for the in-tree library, the fused chain sets (PP2_FX=1), interleaved
# three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_planner.txt
: > $OUT
for rep in 1 2 3; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    for fx in 0 1; do
      [ "$fx" = 1 ] && [ "$lib" != path_planning_2d_amd/libpp2_hip.so ] && continue
      echo "== $lib PP2_FX=$fx rep $rep" >> $OUT
      PP2_FX=$fx PP2_CASE=256 PP2_STEPS=200 PP2_LIBRARY=$PWD/$lib timeout -k 10 120 python3 tools/prof_planner.py 2>/dev/null | grep "plan steps" >> $OUT || exit 1
    done
  done
done
cat $OUT
