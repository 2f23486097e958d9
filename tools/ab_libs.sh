#!/bin/bash
# A/B of library builds (tools/_var/*.so vs the in-tree one): coded loop /
# sweep timings at 1024^2 and 2048^2 and the 1-rank RCCL shard pipeline,
# interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab.txt
: > $OUT
for rep in 1 2; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    for n in 1024 2048; do
      echo "== $lib N=$n rep $rep" >> $OUT
      PP2_LIBRARY=$PWD/$lib PP2_N=$n timeout -k 10 60 python3 tools/coded_loop_timing.py 2>/dev/null | grep -v "^N=" >> $OUT || exit 1
    done
    echo "== $lib rccl1 rep $rep" >> $OUT
    PP2_LIBRARY=$PWD/$lib PP2_MODES=rccl1,rccl1-depth2,rccl1-depth4 timeout -k 10 120 python3 tools/rccl_pipeline_timing.py 2>/dev/null | grep "us/step" >> $OUT || exit 1
  done
done
cat $OUT
