#!/bin/bash
# Same-box A/B of library builds (the in-tree libpp2_hip.so against variant
# builds under tools/_var/, built here with make OUT=... OBJDIR=...
# EXTRA_FLAGS=...): AB_SCRIPT (default tools/c4_share_timing.py) per library,
# interleaved 3 times; AB_GREP picks its result lines (default "us/"), AB_GLOB
# the variant libraries (default tools/_var/*.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_r05.txt
: > $OUT
for rep in 1 2 3; do
  for lib in path_planning_2d_amd/libpp2_hip.so ${AB_GLOB:-tools/_var/*.so}; do
    PP2_LIBRARY=$PWD/$lib timeout -k 10 120 python3 ${AB_SCRIPT:-tools/c4_share_timing.py} 2>/dev/null | grep "${AB_GREP:-us/}" >> $OUT || exit 1
  done
done
cat $OUT
