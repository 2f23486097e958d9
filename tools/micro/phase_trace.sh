#!/bin/bash
# Phase timestamps of the coded fused loop kernel: builds a diagnostic copy of
# the library with -DPP2_PHASE_TRACE into tools/micro/_trace/ (run here, on the
# build host) -- then on the GPU box: python3 tools/micro/phase_trace.py
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
CS=$ROOT/path_planning_2d_amd/csrc
mkdir -p "$HERE/_trace"
make -C "$CS" -j8 OUT="$HERE/_trace/libpp2_trace.so" OBJDIR="$HERE/_trace/obj" \
  EXTRA_FLAGS=-DPP2_PHASE_TRACE "$HERE/_trace/libpp2_trace.so"
