#!/bin/bash
# 2-D resident tiles: the tile-column A/B, then parity (resident + shard tests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python3 tools/ab_tile_cols.py > $OUT/ab_tile_cols2.txt 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_shards.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_2d.log 2>&1
rc=$?
tail -5 $OUT/pytest_2d.log
echo "exit=$rc"
exit $rc
