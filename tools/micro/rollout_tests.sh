set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -15
