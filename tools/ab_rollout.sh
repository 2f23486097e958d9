#!/bin/bash
# Same-box A/B of the rollout leg (tools/rollout_timing.py) over library
# builds: the in-tree one and tools/_var/*.so, interleaved three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_rollout.txt
: > $OUT
for rep in 1 2 3; do
  for lib in path_planning_2d_amd/libpp2_hip.so ${AB_GLOB:-tools/_var/*.so}; do
    PP2_LIBRARY=$PWD/$lib timeout -k 10 90 python3 tools/rollout_timing.py 2>/dev/null | grep "ms," >> $OUT || exit 1
  done
done
cat $OUT
