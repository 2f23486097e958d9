#!/bin/bash
# A/B of library builds (tools/_var/*.so vs the in-tree one) on the coded
# loop / sweep timings at 1024^2 (pairs and single steps) and 2048^2,
# interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab.txt
: > $OUT
for rep in 1 2; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    for cfg in "1024 1" "1024 0" "2048 1"; do
      set -- $cfg
      echo "== $lib N=$1 pairs=$2 rep $rep" >> $OUT
      PP2_LIBRARY=$PWD/$lib PP2_N=$1 PP2_PAIRS=$2 timeout -k 10 60 python3 tools/coded_loop_timing.py >> $OUT 2>/dev/null || exit 1
    done
  done
done
cat $OUT
