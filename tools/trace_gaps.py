"""Busy and idle time of a rocprofv3 kernel trace: the union of all kernels'
[start, end) intervals against the span from the first start to the last end,
the idle gaps between them (count, total, the largest), and per kernel the
time it alone kept the GPU busy (no other kernel running) -- which kernels
sit on the critical path.  With a name substring, only the span from that
kernel's first launch on is counted (skip a setup phase).
    python tools/trace_gaps.py gpurun_out/prof_p256/run_kernel_trace.csv [first-kernel-substring]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    if not name:
        return "-"
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("pp2::", "")
    return n.split("(")[0][:28]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if len(sys.argv) > 2:
        first = next(i for i, e in enumerate(ev) if sys.argv[2] in e[2])
        ev = ev[first:]
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    # sweep: busy union, gaps, and the time each kernel ran alone
    points = []
    for i, (s, e, n) in enumerate(ev):
        points.append((s, 1, i))
        points.append((e, -1, i))
    points.sort()
    active = set()
    busy = 0
    gaps = []
    gap_kinds = defaultdict(lambda: [0, 0])  # (kernel that ended, kernel that starts) -> count, time
    last_end_name = None
    alone = defaultdict(int)
    last = t0
    for t, kind, i in points:
        if active:
            busy += t - last
            if len(active) == 1:
                alone[ev[next(iter(active))][2]] += t - last
        elif t > last:
            gaps.append(t - last)
            key = (short(last_end_name), short(ev[i][2]))
            gap_kinds[key][0] += 1
            gap_kinds[key][1] += t - last
        last = t
        if kind == 1:
            active.add(i)
        else:
            active.discard(i)
            last_end_name = ev[i][2]
    span = t1 - t0
    print(f"span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({busy / span:.1%}), "
          f"idle {(span - busy) / 1e6:.2f} ms in {len(gaps)} gaps, "
          f"largest {max(gaps) / 1e3 if gaps else 0:.1f} us, "
          f"median {sorted(gaps)[len(gaps) // 2] / 1e3 if gaps else 0:.1f} us")
    print("idle gaps by (kernel that ended -> kernel that started):")
    for (a, b), (c, v) in sorted(gap_kinds.items(), key=lambda kv: -kv[1][1])[:10]:
        print(f"  {a:28s} -> {b:28s} {c:6d} gaps {v / 1e6:8.2f} ms")
    print("kernel time alone on the GPU (the critical path's share):")
    for name, v in sorted(alone.items(), key=lambda kv: -kv[1])[:14]:
        print(f"  {name[:70]:70s} {v / 1e6:8.2f} ms ({v / span:.1%})")


if __name__ == "__main__":
    main()
