"""CPU: the hand-counted waits of the built library's kernels cover every
load they pace (tools/asm_hazard_check.py, round-5 ADVICE).

k_pair_dot_bq, k_chain_walk, k_rollout_band and k_rollout_leaf_mfma issue
memory instructions in inline asm and wait for them with hand-counted
`s_waitcnt`; the compiler does not see those loads, so nothing but this
check stops it from touching their destination registers before the wait
(the round-5 rollout fault).  The checker disassembles every
gfx950 code object in libpp2_hip.so and simulates the wait counters over
each kernel's control flow; any instruction that reads or writes an
in-flight load's destination is reported.  Compiler-scheduled code passes
by construction; the asm kernels must too."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "path_planning_2d_amd", "libpp2_hip.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpp2_hip.so not built")
@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="no llvm-objdump")
def test_no_instruction_touches_an_inflight_load():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asm_hazard_check.py"), LIB],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    n = int(r.stdout.strip().splitlines()[-1].split()[0])
    assert n > 100  # every kernel of the library was disassembled


def test_checker_flags_a_hazard():
    """The checker itself: a load whose destination is read before its wait
    is reported; the same code with the wait in place is not; a second load
    into the same registers (in-order return) is not."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import asm_hazard_check as H
    bad = [(0, "global_load_dwordx4", "v[4:7], v[0:1], off", None),
           (8, "v_add_f32_e32", "v8, v4, v9", None),
           (12, "s_waitcnt", "vmcnt(0)", None),
           (16, "s_endpgm", "", None)]
    assert H.check_function("k", bad)
    good = [bad[0], bad[2], bad[1], bad[3]]
    assert not H.check_function("k", good)
    waw = [bad[0], (8, "global_load_dwordx4", "v[4:7], v[2:3], off", None), bad[2], bad[1],
           bad[3]]
    assert not H.check_function("k", waw)
    # a loop carrying a load into the next iteration without a wait
    loop = [(0, "s_mov_b32", "s0, 0", None),
            (4, "v_mul_f32_e32", "v8, v4, v4", None),        # uses last iteration's load
            (8, "global_load_dword", "v4, v[0:1], off", None),
            (16, "s_cbranch_scc1", "", 4),
            (20, "s_waitcnt", "vmcnt(0)", None),
            (24, "s_endpgm", "", None)]
    assert H.check_function("k", loop)
