#!/bin/bash
# The rollout's leaf pass on the matrix cores: rollout parity, then the
# rollout leg (512^2, 4096 copies x 5) with the MFMA pass (stage 2 / 1) and
# the fmaf pass, interleaved, and a kernel trace of the product build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/leaf_tests.log 2>&1 || { tail -30 $O/leaf_tests.log; exit 1; }
tail -2 $O/leaf_tests.log
for lib in ${PP2_LIBS:-product tools/_var/leaf_fmaf.so}; do
  [ "$lib" = product ] && l= || l=$lib
  PP2_LIBRARY=$l timeout -k 10 120 python3 tools/rollout_timing.py || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_leaf -o run -- python3 tools/rollout_timing.py > $O/leaf_prof.log 2>&1 || { tail $O/leaf_prof.log; exit 1; }
f=$(ls $O/prof_leaf/*kernel_stats.csv $O/prof_leaf/*/*kernel_stats.csv 2>/dev/null | head -1); python3 tools/kstats.py "$f" 12
