"""Summarise a rocprofv3 run of `bench.py --profile` into profiles/pmc_<tag>.json.

Inputs (merged back from the GPU box by gpurun): gpurun_out/prof/
run_kernel_stats.csv (kernel durations), gpurun_out/pmc_fetch/ and
gpurun_out/pmc_write/ run_counter_collection.csv (separate --pmc passes).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of
a wide (16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane streaming stores.
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
Usage: python profiles/parse_pmc.py <tag> [cells] [steps per resident launch]
       [directory under gpurun_out (tools/collect_pmc.sh's PMC_DIR)]
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
# algorithmic HBM bytes per cell (bench.py docstring / DESIGN.md)
ALGO = {"k_mdp_sweep": 369, "k_belief_update": 48, "k_loop_step": 381,
        "k_loop_step_coded": 19, "k_mdp_sweep_coded": 11,
        "k_loop_pair_coded": 19,  # two steps per launch, intermediate in LDS
        "k_loop_resident": 19}  # the whole trajectory per launch, tiles in LDS


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "").replace("pp2::", "")


def counter(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


def main():
    tag = sys.argv[1]
    cells = int(sys.argv[2]) if len(sys.argv) > 2 else 1024 * 1024
    spl = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    src = os.path.join(OUT, sys.argv[4]) if len(sys.argv) > 4 else OUT
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "prof", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = r
    fetch = counter(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = counter(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    kernels = {}
    for k, r in stats.items():
        base = k.split("<")[0]
        d = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
             "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3,
             "pct_time": float(r["Percentage"])}
        if k in fetch and k in write:
            f = sorted(fetch[k])[len(fetch[k]) // 2]
            w = sorted(write[k])[len(write[k]) // 2]
            d["FETCH_SIZE_KiB_median"] = f
            d["WRITE_SIZE_KiB_median"] = w
            d["hbm_bytes_per_launch"] = (2 * f + w) * 1024
        if base in ALGO:
            d["cells"] = cells
            if base == "k_loop_resident":
                d["steps_per_launch"] = spl
            d["algorithmic_bytes_per_launch"] = ALGO[base] * cells
            d["algorithmic_GBps"] = ALGO[base] * cells / (d["avg_us"] * 1e-6) / 1e9
            if "hbm_bytes_per_launch" in d:
                d["hbm_over_algorithmic"] = d["hbm_bytes_per_launch"] / d["algorithmic_bytes_per_launch"]
        kernels[k] = d
    res = {"tag": tag, "source": "rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE "
                               "(separate passes) of `python3 bench.py --profile`",
           "hbm_bytes_formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)",
           "kernels": kernels}
    path = os.path.join(ROOT, "profiles", f"pmc_{tag}.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
