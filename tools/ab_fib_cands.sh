cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab3.txt; : > $OUT
for rep in 1 2 3; do
  for cfg in "0 0 0" "1 0 0" "1 1 0"; do
    set -- $cfg
    PP2_FIB_CANDS=$1 PP2_FC_PLAN9=$2 PP2_FC_K9WAVE=$3 PP2_CASE=256 PP2_STEPS=200 timeout -k 10 120 python3 tools/prof_planner.py 2>&1 | grep "plan steps" | sed "s/^/cands=$1 plan9=$2 k9wave=$3 /" >> $OUT || exit 1
  done
done
cat $OUT
