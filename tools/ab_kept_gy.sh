#!/bin/bash
# Same-box A/B of the config-2 plan step (tools/prof_planner.py, 256^2) over
# the kept children's FIB-table workgroup rows (PP2_FC_KEPT_GY; 0 = one per
# kept child, the default), interleaved three times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_kept_gy.txt; : > $OUT
for rep in 1 2 3; do
  for gy in 0 16 8; do
    PP2_FC_KEPT_GY=$gy PP2_CASE=256 PP2_STEPS=200 timeout -k 10 120 python3 tools/prof_planner.py 2>&1 | grep "plan steps" | sed "s/^/kept_gy=$gy /" >> $OUT || exit 1
  done
done
cat $OUT
