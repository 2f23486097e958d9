#!/bin/bash
# Same-box A/B of the driver's headline command (bench.py --steps 20 --warmup 5,
# secondary legs skipped where a flag allows) across library builds
# (tools/_var/*.so vs the in-tree one), interleaved three times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_bench20.txt
: > $OUT
for rep in 1 2 3; do
  for lib in path_planning_2d_amd/libpp2_hip.so tools/_var/*.so; do
    PP2_LIBRARY=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 \
      --no-cpu-baseline --no-pbvi --plan-steps 0 --rollout-copies 0 --c4-size 0 --shard-rows 0 \
      > gpurun_out/ab_b.json 2> gpurun_out/ab_b.err || exit 1
    python3 -c "
import json
d = json.loads(open('gpurun_out/ab_b.json').read().strip().splitlines()[-1])
k = d['kernels']
print('$lib rep $rep: %.1f G cells/s, wall %.3f us/step, events %.3f, enqueue %.3f, launch %.1f us'
      % (d['value'] / 1e9, d['ms_per_step'] * 1e3, k['loop_step_us_events'],
         k['loop_enqueue_us_per_step'], d['roofline']['avg_launch_us']))" >> $OUT || exit 1
  done
done
cat $OUT
