#!/bin/bash
# The automatic shard halo (halved while the tiles get fewer rows) and the
# 2-D sweep grouping: shard / resident / config parity, then config 4's rank
# share at the automatic and the explicit depths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_shards.py tests/test_gpu_configs.py tests/test_gpu_coded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/hr_tests.log 2>&1 || { tail -30 $O/hr_tests.log; exit 1; }
tail -2 $O/hr_tests.log
PP2_LIBS="product" PP2_CASES=0:0:0:0,128:0:0:0,0:0:0:0,128:0:0:0 bash tools/micro/nowait_run.sh
