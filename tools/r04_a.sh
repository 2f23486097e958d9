#!/bin/bash
# Round 4 GPU check: fchain + planner parity, chain-set timings, reference-order
# plan steps, then config 4's rank share over resident halo depths / tilings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fchain.py tests/test_gpu_planner.py tests/test_gpu_shards.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/r04_t4.log 2>&1 || { tail -30 $O/r04_t4.log; exit 1; }
tail -2 $O/r04_t4.log
timeout -k 10 60 python3 tools/fchain_timing.py > $O/r04_fct2.txt 2>&1 || { cat $O/r04_fct2.txt; exit 1; }
cat $O/r04_fct2.txt
PP2_REF=1 PP2_STEPS=100 timeout -k 10 120 python3 tools/prof_planner.py > $O/r04_plan3.log 2>&1 || { cat $O/r04_plan3.log; exit 1; }
cat $O/r04_plan3.log
timeout -k 10 300 python3 tools/c4_halo_sweep.py > $O/r04_c4halo.txt 2>&1 || { cat $O/r04_c4halo.txt; exit 1; }
cat $O/r04_c4halo.txt
timeout -k 10 60 tools/micro/copy_bw > $O/r04_copy_bw2.txt 2>&1 || { cat $O/r04_copy_bw2.txt; exit 1; }
PP2_REF=1 PP2_STEPS=30 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_plan4 -o run -- python3 tools/prof_planner.py > $O/r04_prof_plan4.log 2>&1
rc=$?
cat $O/r04_copy_bw2.txt
exit $rc
