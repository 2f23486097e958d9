#!/bin/bash
# Same-box A/B of library builds (the in-tree libpp2_hip.so against variant
# builds under tools/_var/, built here with make OUT=... OBJDIR=...
# EXTRA_FLAGS=...): tools/c4_share_timing.py per library, interleaved 3 times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_r05.txt
: > $OUT
for rep in 1 2 3; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    PP2_LIBRARY=$PWD/$lib timeout -k 10 120 python3 tools/c4_share_timing.py 2>/dev/null | grep "us/step" >> $OUT || exit 1
  done
done
cat $OUT
