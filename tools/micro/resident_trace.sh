#!/bin/bash
# Per-step phase timestamps of the tile-resident loop: builds a diagnostic
# copy of the library with -DPP2_RES_TRACE into tools/micro/_rtrace/ (run
# here, on the build host) -- then on the GPU box: python3 tools/micro/resident_trace.py
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
CS=$ROOT/path_planning_2d_amd/csrc
mkdir -p "$HERE/_rtrace"
make -C "$CS" -j8 OUT="$HERE/_rtrace/libpp2_rtrace.so" OBJDIR="$HERE/_rtrace/obj" \
  EXTRA_FLAGS=-DPP2_RES_TRACE "$HERE/_rtrace/libpp2_rtrace.so"
