"""Per-expansion kernel timeline of a rocprofv3 --kernel-trace CSV of
tools/prof_planner.py: expansions start at k_tree_pred; for each kernel (by
its order of appearance in an expansion) the median start, end and duration
relative to the expansion's start, and the median expansion span."""
import csv
import statistics as st
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("pp2::", "")
    return n.split("(")[0][:28]


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    idx = [i for i, e in enumerate(ev) if "k_tree_pred" in e[2]]
    # skip the warm-up third
    idx = idx[len(idx) // 3:]
    per = {}
    spans = []
    for a, b in zip(idx, idx[1:]):
        t0 = ev[a][0]
        seen = {}
        for s, e, n in ev[a:b]:
            key = short(n)
            seen[key] = seen.get(key, 0) + 1
            k = (key, seen[key])
            per.setdefault(k, []).append(((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
        spans.append((ev[b][0] - t0) / 1e3)
    print(f"{len(spans)} expansions; median span to the next expansion {st.median(spans):.1f} us")
    order = sorted(per, key=lambda k: st.median(x[0] for x in per[k]))
    for k in order:
        v = per[k]
        if len(v) < len(spans) // 2:
            continue
        print(f"{st.median(x[0] for x in v):8.1f} {st.median(x[1] for x in v):8.1f} "
              f"{st.median(x[2] for x in v):7.1f}  {k[0]}#{k[1]}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
