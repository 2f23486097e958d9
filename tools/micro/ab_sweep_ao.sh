set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_shards.py tests/test_gpu_configs.py tests/test_gpu_coded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/g4_tests.log 2>&1 || { tail -30 $O/g4_tests.log; exit 1; }
tail -2 $O/g4_tests.log
PP2_LIBS="product tools/_var/sweep_ao0.so product tools/_var/sweep_ao0.so" PP2_CASES=128:0:0:0,96:2:0:0,64:2:0:0 bash tools/micro/nowait_run.sh
