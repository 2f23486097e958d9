#!/bin/bash
# GPU side of tools/micro/resident_nowait.sh: the same timings with the
# product library and with the no-wait diagnostic build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
mkdir -p $O
export PP2_CASES=${PP2_CASES:-128:0:0:0,128:1:0:0,64:0:0:0}
for lib in ${PP2_LIBS:-product tools/micro/_nowait/libpp2_nowait.so}; do
  echo "== library $lib"
  [ "$lib" = product ] && lib=
  PP2_LIBRARY=$lib timeout -k 10 120 python3 tools/micro/loop_1024.py || exit 1
  PP2_LIBRARY=$lib timeout -k 10 200 python3 tools/c4_halo_sweep.py || exit 1
done
