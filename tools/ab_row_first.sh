#!/bin/bash
# Same-box A/B of the config-2 plan step (tools/prof_planner.py, 256^2):
# the cdf chain enqueued before the predictions (PP2_ROW_FIRST=1) or after
# them (0, default), interleaved three times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_row_first.txt; : > $OUT
for rep in 1 2 3; do
  for rf in 1 0; do
    PP2_ROW_FIRST=$rf PP2_CASE=256 PP2_STEPS=200 timeout -k 10 120 python3 tools/prof_planner.py 2>&1 | grep "plan steps" | sed "s/^/row_first=$rf /" >> $OUT || exit 1
  done
done
cat $OUT
