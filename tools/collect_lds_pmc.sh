#!/bin/bash
# SQ counters (LDS, VALU, wait states) of the coded loop and sweep kernels
# (DRIVER: another driver script and its arguments, e.g. "tools/prof_rollout.py
# --reps 2" for the rollout's band kernel), one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md rocprofv3:
# at most 8 SQ counters per pass; no tracing domains beside --pmc).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_OUT:-lds_pmc}
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $OUT/p1 -o run -- python3 ${DRIVER:-tools/coded_loop_timing.py} > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $OUT/p2 -o run -- python3 ${DRIVER:-tools/coded_loop_timing.py} > $OUT/p2.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
