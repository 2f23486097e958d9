#!/bin/bash
# Same-box A/B of resident-loop builds (tools/_var/*.so vs the in-tree one):
# resident launch timing at 1024^2, interleaved three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_resident.txt
: > $OUT
for rep in 1 2 3; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    echo "== $lib rep $rep" >> $OUT
    PP2_LIBRARY=$PWD/$lib timeout -k 10 60 python3 tools/resident_launch_timing.py 2>/dev/null | grep -E "n=   20|n=  400|n= 2000" >> $OUT || exit 1
    PP2_LIBRARY=$PWD/$lib PP2_RESIDENT=1 timeout -k 10 60 python3 tools/coded_loop_timing.py 2>/dev/null | grep -E "sweep:" >> $OUT || exit 1
  done
done
cat $OUT
