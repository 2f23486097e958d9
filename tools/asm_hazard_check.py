#!/usr/bin/env python3
"""Static check of the hand-counted memory waits in the built library.

Several kernels issue memory instructions the compiler does not track --
inline-asm `ds_read` / `global_load` with hand-counted `s_waitcnt`
(k_pair_dot_bq, k_chain_walk, k_rollout_band, k_rollout_leaf_mfma) -- and
are correct only if no instruction touches a destination register of such a
load before the wait that covers it.  The round-5 rollout fault was exactly
that: the compiler moved an in-flight load's destination registers and the
late load overwrote an address.  This tool disassembles every
gfx950 code object embedded in libpp2_hip.so and simulates the wait counters
over each kernel:

  * VMEM ops (loads, stores, LDS-DMA) retire in order under `vmcnt`, LDS ops
    under `lgkmcnt`; an SMEM op (out-of-order) makes only `lgkmcnt(0)` retire;
  * any instruction that reads or writes a VGPR / AGPR that is the
    destination of a load not yet retired is a hazard;
  * control flow: a forward dataflow over the kernel's basic blocks to a
    fixpoint -- at a join a load is outstanding if it is on either path, with
    the fewer younger ops of the two (a pipeline's loads issued in one loop
    iteration and used in the next are followed around the back edge).

Compiler-scheduled code satisfies this by construction, so every report
points at hand-counted code.  Usage:

    python tools/asm_hazard_check.py [path/to/libpp2_hip.so] [kernel-substring ...]

Exit status 1 when a hazard is found (tests/test_asm_hazards.py runs it).
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so_path, arch="gfx950"):
    """The ELF code objects for `arch` in the clang offload bundles of a
    host shared library."""
    data = open(so_path, "rb").read()
    pos = 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return
        n = struct.unpack_from("<Q", data, i + 24)[0]
        off = i + 32
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode()
            off += tl
            if arch in triple:
                yield data[i + o:i + o + sz]
        pos = i + 1


def disassemble(blob):
    with tempfile.NamedTemporaryFile(suffix=".elf", delete=False) as f:
        f.write(blob)
        path = f.name
    try:
        return subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", path], check=True,
                              capture_output=True, text=True).stdout
    finally:
        os.unlink(path)


FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
INSN = re.compile(r"^\t(\S+)\s*(.*?)\s*// ([0-9A-F]+):")
TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")
REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")


def functions(text):
    name, body = None, []
    for line in text.splitlines():
        m = FUNC.match(line)
        if m:
            if name:
                yield name, body
            name, body = m.group(2), []
            base = int(m.group(1), 16)
            continue
        m = INSN.match(line)
        if m and name:
            addr = int(m.group(3), 16)
            ops = m.group(2)
            t = TARGET.search(line)
            tgt = base + int(t.group(2), 16) if t and t.group(1) == name else None
            body.append((addr, m.group(1), ops, tgt))
    if name:
        yield name, body


def regs(ops):
    """VGPR / AGPR numbers referenced by an operand string (AGPRs offset by 512)."""
    out = set()
    for kind, one, lo, hi in REG.findall(ops):
        off = 512 if kind == "a" else 0
        if one:
            out.add(off + int(one))
        else:
            out.update(range(off + int(lo), off + int(hi) + 1))
    return out


def first_operand_regs(ops):
    first = ops.split(",")[0] if ops else ""
    return regs(first)


VMEM = ("global_", "buffer_", "flat_", "scratch_")
SMEM = ("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_dcache", "s_scratch_load")


def classify(mn, ops):
    """('vm' | 'lds' | 'smem' | None, destination registers)."""
    if mn.startswith(VMEM):
        if "_lds" in mn or re.search(r"\blds\b", ops):
            return "vm", set()  # LDS-DMA: no VGPR destination
        if "load" in mn:
            return "vm", first_operand_regs(ops)
        if "atomic" in mn and re.search(r"\b(glc|sc0)\b", ops):
            return "vm", first_operand_regs(ops)
        return "vm", set()  # stores, atomics without return, cache ops
    if mn.startswith("ds_"):
        if any(k in mn for k in ("read", "load", "_rtn", "permute", "swizzle", "consume",
                                 "append", "bpermute")):
            return "lds", first_operand_regs(ops)
        return "lds", set()
    if mn.startswith(SMEM):
        return "smem", set()
    return None, set()


WAIT = re.compile(r"(vmcnt|lgkmcnt)\((\d+)\)")


def transfer(state, insn, report=None):
    """One instruction on a state {("vm"|"lgkm", load address): (younger ops, dst,
    is_smem)}; report(insn, load address, registers) for each hazard."""
    addr, mn, ops, _ = insn
    if mn == "s_waitcnt":
        w = dict((c, int(v)) for c, v in WAIT.findall(ops))
        if ops.strip() == "0":
            w = {"vmcnt": 0, "lgkmcnt": 0}
        smem = any(v[2] for (q, _), v in state.items() if q == "lgkm")
        out = {}
        for (q, a), v in state.items():
            if q == "vm" and "vmcnt" in w and v[0] >= w["vmcnt"]:
                continue
            if q == "lgkm" and "lgkmcnt" in w:
                m = w["lgkmcnt"]
                if m == 0 or (not smem and v[0] >= m):
                    continue
            out[(q, a)] = v
        return out
    if mn == "s_endpgm":
        return {}
    used = regs(ops)
    kind, dst = classify(mn, ops)
    q = None if kind is None else "vm" if kind == "vm" else "lgkm"
    if used and report:
        for (oq, a), (_, odst, _) in state.items():
            # a load of the same counter may overwrite an outstanding load's
            # destination: they return in issue order (its sources may not)
            hit = (used - dst if oq == q else used) & odst
            if hit:
                report(insn, a, hit)
    if kind is None:
        return state
    out = {}
    for key, (k, d, sm) in state.items():
        out[key] = (k + 1, d, sm) if key[0] == q else (k, d, sm)
    out[(q, addr)] = (0, dst, kind == "smem")
    return out


def merge(a, b):
    """Outstanding on either path, as young as on the younger path."""
    out = dict(a)
    for key, v in b.items():
        if key in out:
            u = out[key]
            out[key] = (min(u[0], v[0]), u[1] | v[1], u[2] or v[2])
        else:
            out[key] = v
    return out


def check_function(name, body):
    """Forward dataflow over the function's basic blocks to a fixpoint, then
    one reporting pass."""
    if not body:
        return []
    idx = {a: k for k, (a, _, _, _) in enumerate(body)}
    leaders = {0}
    for k, (a, mn, ops, tgt) in enumerate(body):
        if mn.startswith(("s_branch", "s_cbranch")) or mn == "s_endpgm":
            if k + 1 < len(body):
                leaders.add(k + 1)
            if tgt is not None and tgt in idx:
                leaders.add(idx[tgt])
    starts = sorted(leaders)
    blocks = {s: (s, (starts[i + 1] if i + 1 < len(starts) else len(body)))
              for i, s in enumerate(starts)}

    def succ(s):
        e = blocks[s][1]
        a, mn, ops, tgt = body[e - 1]
        out = []
        if mn == "s_endpgm":
            return out
        if mn.startswith(("s_branch", "s_cbranch")) and tgt is not None and tgt in idx:
            out.append(idx[tgt])
        if not mn.startswith("s_branch") and e < len(body):
            out.append(e)
        return out

    ins = {0: {}}
    work = [0]
    rounds = 0
    while work and rounds < 200000:
        rounds += 1
        s = work.pop()
        st = ins[s]
        for k in range(*blocks[s]):
            st = transfer(st, body[k])
        for t in succ(s):
            old = ins.get(t)
            new = st if old is None else merge(old, st)
            if old is None or new != old:
                ins[t] = new
                work.append(t)
    hazards = []

    def report(insn, load_addr, hit):
        hazards.append((name, insn[0], insn[1], insn[2], load_addr, sorted(hit)))

    for s in starts:
        if s not in ins:
            continue
        st = ins[s]
        for k in range(*blocks[s]):
            st = transfer(st, body[k], report)
    return hazards


def main(argv):
    so = os.path.join(ROOT, "path_planning_2d_amd", "libpp2_hip.so")
    pats = []
    for a in argv:
        if a.endswith(".so"):
            so = a
        else:
            pats.append(a)
    found = 0
    nfun = 0
    for blob in code_objects(so):
        for name, body in functions(disassemble(blob)):
            if pats and not any(p in name for p in pats):
                continue
            nfun += 1
            seen = set()
            for h in check_function(name, body):
                key = (h[1], h[4])
                if key in seen:
                    continue
                seen.add(key)
                found += 1
                print(f"HAZARD {h[0]}: {h[1]:#x} {h[2]} {h[3]} touches v{h[5]} of the load at "
                      f"{h[4]:#x}")
    print(f"{nfun} kernels checked, {found} hazards")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
