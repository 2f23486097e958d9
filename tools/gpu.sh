#!/bin/bash
# The GPU driver: one script, one mode per step argument (tools/README.md);
# ROUND (default r06) names the PMC summary directories.
#   tests    full `pytest -m gpu` suite
#   planner  tests/test_gpu_planner.py only
#   bench    driver-style bench (N=1, 20 steps)
#   prof     rocprofv3 kernel trace of the bench's timed loop + the plan-step legs
#   pmc      HBM counters of the resident loop / solve (tools/collect_pmc.sh)
#   fchain   tests/test_gpu_fchain.py (the exact chain sets, FC_LIST included)
#   pbvi     tools/pbvi_plan_timing.py (PBVI-leaf plan steps: packed / one-chain / k_pair_seq dots)
#   profplan rocprofv3 kernel traces of the node and 256^2 PBVI-leaf plan steps
#   shards   tests/test_gpu_shards.py + test_gpu_resident.py (the resident / shard kernels)
#   ab       tools/ab_builds.sh: config-4 rank share + 1024^2 loop, in-tree vs tools/_var/*.so
#   copy     tools/micro/copy_bw (the one-shot copy ceiling, built here with hipcc)
#   pbvitests tests/test_gpu_pbvi.py (the PBVI kernels, the leaf-dot shapes)
#   dots     tools/micro/pair_dots (the leaf-dot shapes in isolation, built here with hipcc)
#   rollsq   SQ counters of the rollout's band kernel (tools/collect_lds_pmc.sh)
#   abroll   tests/test_gpu_rollout.py on each tools/_var/roll_*.so, then tools/ab_rollout.sh
#   abfib    tools/fib_ab_timing.py on the in-tree library and tools/_var/fib_*.so
#   quick    the shard / coded / rollout GPU test files (the round's changed paths)
#   p256     rocprofv3 kernel trace of the config-2 plan step (256^2, depth 3, FIB leaves)
#   fxab     config-2 plan steps with the fused chain sets (PP2_FX=1) and without (0), interleaved
#   fxtests  tests/test_gpu_fchain.py + test_gpu_planner.py (the chain sets and the planner)
#   candab   config-2 plan steps with the FIB candidate masks (PP2_FIB_CANDS=1) and without (0), interleaved
# Every GPU step has its own time limit, steps are chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
T="--timeout 150 --timeout-method thread -p no:cacheprovider"
run_tests()   { timeout -k 10 900 python -u -m pytest tests -m gpu -x -v $T > $OUT/pytest_gpu.log 2>&1; }
run_planner() { timeout -k 10 600 python -u -m pytest tests/test_gpu_planner.py -x -v $T > $OUT/pytest_planner.log 2>&1; }
run_smoke()   { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; }
run_bench()   { timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; }
run_prof()    { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --profile --steps 20 --warmup 20 > $OUT/prof.log 2>&1; }
run_pmc()     { PMC_DIR=pmc_${ROUND:-r06} timeout -k 10 900 bash tools/collect_pmc.sh > $OUT/pmc.log 2>&1; }
run_pmcx()    { PP2_LIBRARY=$PWD/tools/_var/c_xcd.so PMC_DIR=pmc_${ROUND:-r06}x timeout -k 10 900 bash tools/collect_pmc.sh > $OUT/pmcx.log 2>&1; }
run_shards()  { timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py tests/test_gpu_resident.py -x -v $T > $OUT/pytest_shards.log 2>&1; }
run_ab()      { timeout -k 10 900 bash tools/ab_builds.sh > $OUT/ab.log 2>&1; }
run_copy()    { timeout -k 10 120 tools/micro/copy_bw 2048 > $OUT/copy_bw.txt 2>&1; }
run_pbvitests() { timeout -k 10 300 python -u -m pytest tests/test_gpu_pbvi.py -x -v $T > $OUT/pytest_pbvi.log 2>&1; }
run_dots()    { timeout -k 10 120 tools/micro/pair_dots > $OUT/pair_dots.txt 2>&1; }
run_rollsq()  { PMC_OUT=rollout_sq DRIVER="tools/prof_rollout.py --reps 2" timeout -k 10 300 bash tools/collect_lds_pmc.sh > $OUT/rollout_sq.log 2>&1; }
run_abroll()  { for lib in tools/_var/roll_*.so; do PP2_LIBRARY=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -q $T > $OUT/pytest_rollout_$(basename $lib .so).log 2>&1 || return 1; done &&
                AB_GLOB="tools/_var/roll_*.so" timeout -k 10 600 bash tools/ab_rollout.sh > $OUT/ab_rollout.log 2>&1; }
run_abfib()   { AB_SCRIPT=tools/fib_ab_timing.py AB_GLOB="tools/_var/fib_*.so" timeout -k 10 600 bash tools/ab_builds.sh > $OUT/ab_fib.log 2>&1; }
run_fchain()  { timeout -k 10 300 python -u -m pytest tests/test_gpu_fchain.py -x -v $T > $OUT/pytest_fchain.log 2>&1; }
run_pbvi()    { PP2_PBVI_STATS=1 timeout -k 10 300 python3 tools/pbvi_plan_timing.py > $OUT/pbvi_plan_timing.txt 2>&1; }
run_profplan() { PP2_CASE=node PP2_STEPS=30 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_node -o run -- python3 tools/prof_planner.py > $OUT/prof_node.log 2>&1 &&
                 PP2_CASE=256 PP2_LB=1 PP2_STEPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pbvi256 -o run -- python3 tools/prof_planner.py > $OUT/prof_pbvi256.log 2>&1; }
run_quick()   { timeout -k 10 900 python -u -m pytest tests/test_gpu_shards.py tests/test_gpu_coded.py tests/test_gpu_rollout.py -x -v $T > $OUT/pytest_quick.log 2>&1; }
run_p256()    { PP2_CASE=256 PP2_STEPS=60 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p256 -o run -- python3 tools/prof_planner.py > $OUT/prof_p256.log 2>&1; }
run_fxab()    { for rep in 1 2; do for fx in 1 0; do PP2_FX=$fx PP2_CASE=256 PP2_STEPS=200 timeout -k 10 120 python3 tools/prof_planner.py 2>&1 | sed "s/^/fx=$fx /" >> $OUT/fxab.txt || return 1; done; done; cat $OUT/fxab.txt; }
run_candab()  { for rep in 1 2 3; do for c in 1 0; do PP2_FIB_CANDS=$c PP2_CASE=256 PP2_STEPS=200 timeout -k 10 120 python3 tools/prof_planner.py 2>&1 | sed "s/^/cands=$c /" >> $OUT/candab.txt || return 1; done; done; cat $OUT/candab.txt; }
run_fxtests() { timeout -k 10 900 python -u -m pytest tests/test_gpu_fchain.py tests/test_gpu_planner.py -x -v $T > $OUT/pytest_fx.log 2>&1; }
rc=0
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests) run_tests ;; planner) run_planner ;; smoke) run_smoke ;; bench) run_bench ;;
    prof) run_prof ;; pmc) run_pmc ;; pbvitests) run_pbvitests ;; dots) run_dots ;; rollsq) run_rollsq ;; abroll) run_abroll ;; abfib) run_abfib ;; pmcx) run_pmcx ;; fchain) run_fchain ;; copy) run_copy ;; shards) run_shards ;; ab) run_ab ;; pbvi) run_pbvi ;; profplan) run_profplan ;; quick) run_quick ;; p256) run_p256 ;; fxab) run_fxab ;; fxtests) run_fxtests ;; candab) run_candab ;;
    *) echo "unknown step $step"; false ;;
  esac
  rc=$?
  [ $rc -ne 0 ] && break
done
for f in pytest_fx.log pytest_quick.log pytest_gpu.log pytest_planner.log pytest_fchain.log pytest_shards.log pytest_pbvi.log; do [ -f $OUT/$f ] && tail -3 $OUT/$f; done
echo "exit=$rc"
exit $rc
