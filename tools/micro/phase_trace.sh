#!/bin/bash
# Phase timestamps of the coded fused loop kernel: builds a diagnostic copy of
# the library with -DPP2_PHASE_TRACE into tools/micro/_trace/ (run here, on the
# build host) -- then on the GPU box: python3 tools/micro/phase_trace.py
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
CS=$ROOT/path_planning_2d_amd/csrc
mkdir -p "$HERE/_trace"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fgpu-flush-denormals-to-zero \
  -ffp-contract=off -DPP2_PHASE_TRACE -I"$ROOT/include" -I"$CS" -shared \
  -o "$HERE/_trace/libpp2_trace.so" "$CS/pp2_kernels.hip" "$CS/pp2_coded.hip" \
  "$CS/pp2_runtime.cpp" "$CS/pp2_tree.cpp" "$CS/pp2_shards.cpp" "$CS/pp2_rollout.cpp" -lrccl
