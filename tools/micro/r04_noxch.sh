#!/bin/bash
# rollout parity plus config-4 / 1024^2 timings: product, no-wait and no-exchange diagnostic builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -12 gpurun_out/rt.log
PP2_LIBS="product tools/micro/_nowait/libpp2_nowait.so tools/micro/_nowait/libpp2_noxch.so product tools/micro/_nowait/libpp2_noxch.so" PP2_CASES=0:0:0:0,128:0:0:0 bash tools/micro/nowait_run.sh
