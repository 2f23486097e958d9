#!/bin/bash
# Round 4: transposed resident tiles on shard views -- parity (shard group and
# 1-rank RCCL config-4 shares), then the rank share's timing per tiling.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shards.py -x -v --timeout 150 --timeout-method thread \
  -p no:cacheprovider > $O/r04_t5.log 2>&1 || { tail -40 $O/r04_t5.log; exit 1; }
tail -3 $O/r04_t5.log
timeout -k 10 300 python3 tools/c4_halo_sweep.py > $O/r04_c4tr.txt 2>&1
rc=$?
cat $O/r04_c4tr.txt
exit $rc
