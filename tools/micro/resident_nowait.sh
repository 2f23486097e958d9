#!/bin/bash
# Diagnostic: the tile-resident loop with its hand-off polls turned off
# (-DPP2_RES_NOWAIT: every poll takes its first loads, wrong results) -- the
# per-step time of compute + barriers alone, to split a step into compute and
# hand-off latency; the same without the step-end barrier.  Builds tools/micro/_nowait/libpp2_nowait.so here; on the
# GPU box: PP2_LIBRARY=tools/micro/_nowait/libpp2_nowait.so python3 tools/c4_halo_sweep.py
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
CS=$ROOT/path_planning_2d_amd/csrc
mkdir -p "$HERE/_nowait"
make -C "$CS" -j8 OUT="$HERE/_nowait/libpp2_nowait.so" OBJDIR="$HERE/_nowait/obj" \
  EXTRA_FLAGS=-DPP2_RES_NOWAIT "$HERE/_nowait/libpp2_nowait.so"
# ... and without the step-end barrier (-DPP2_RES_NOBAR, races: timing only)
make -C "$CS" -j8 OUT="$HERE/_nowait/libpp2_nobar.so" OBJDIR="$HERE/_nowait/obj_nobar" \
  EXTRA_FLAGS=-DPP2_RES_NOBAR "$HERE/_nowait/libpp2_nobar.so"
make -C "$CS" -j8 OUT="$HERE/_nowait/libpp2_nowait_nobar.so" OBJDIR="$HERE/_nowait/obj_both" \
  EXTRA_FLAGS="-DPP2_RES_NOWAIT -DPP2_RES_NOBAR" "$HERE/_nowait/libpp2_nowait_nobar.so"
# ... and with no hand-off loads at all (-DPP2_RES_NOXCH: the neighbours' rows read as zeros)
make -C "$CS" -j8 OUT="$HERE/_nowait/libpp2_noxch.so" OBJDIR="$HERE/_nowait/obj_noxch" \
  EXTRA_FLAGS=-DPP2_RES_NOXCH "$HERE/_nowait/libpp2_noxch.so"
