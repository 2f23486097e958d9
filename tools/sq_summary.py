"""Summarise tools/collect_lds_pmc.sh (two SQ/GRBM --pmc passes over
tools/coded_loop_timing.py) into profiles/<round>/resident_sq.json, the LDS /
VALU busy fractions bench.py reports beside the resident kernel's roofline.

Counter semantics (MI355X_MICROARCH.md, rocprofv3 PMC slots): SQ wave-cycle
counters are chip sums in units of 4 cycles; SQ_ACTIVE_INST_VALU counts one
per VALU instruction (a wave64 fp32 op holds its 16-lane SIMD 4 cycles);
SQ_LDS_IDX_ACTIVE counts LDS-array cycles; GRBM_GUI_ACTIVE is the sum over
the 8 XCDs, so GRBM_GUI_ACTIVE / 8 is the dispatch's wall clock in cycles.
    valu_busy = 4 * SQ_ACTIVE_INST_VALU / (4 SIMDs * CUs * wall)
    lds_busy  = SQ_LDS_IDX_ACTIVE / (CUs * wall)
Usage: python tools/sq_summary.py <round dir, e.g. r03> <steps per launch>
       [kernel substring, default k_loop_resident] [pmc dir under gpurun_out]
       [output name, default resident_sq.json] [driver, as collect_lds_pmc.sh's
       DRIVER, default "tools/coded_loop_timing.py at 1024^2"]
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUS = 256


def dispatches(path, kernel):
    """{dispatch id: {counter: value}} of the named kernel's dispatches."""
    acc = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            acc[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    return acc


def longest(d):
    return max(d.values(), key=lambda v: v.get("SQ_WAVE_CYCLES", v.get("GRBM_GUI_ACTIVE", 0.0)))


def main():
    rnd, steps = sys.argv[1], int(sys.argv[2])
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_loop_resident"
    src = os.path.join(ROOT, "gpurun_out", sys.argv[4] if len(sys.argv) > 4 else "lds_pmc")
    c = {}
    for p in ("p1", "p2"):
        c.update(longest(dispatches(os.path.join(src, p, "run_counter_collection.csv"), kernel)))
    wall = c["GRBM_GUI_ACTIVE"] / 8.0
    waves = c["SQ_WAVES"]
    out = {
        "kernel": kernel,
        "steps_per_launch": steps,
        "source": "tools/collect_lds_pmc.sh (rocprofv3 --pmc, two passes) of "
                  + (sys.argv[6] if len(sys.argv) > 6 else "tools/coded_loop_timing.py at 1024^2")
                  + "; the longest dispatch",
        "counters": c,
        "wall_cycles_per_step": wall / steps,
        "valu_busy": 4.0 * c["SQ_ACTIVE_INST_VALU"] / (4 * CUS * wall),
        "lds_busy": c["SQ_LDS_IDX_ACTIVE"] / (CUS * wall),
        "lds_bank_conflict_share": (c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1.0)
                                    if "SQ_LDS_BANK_CONFLICT" in c else None),
        "per_wave_per_step": {k: c[f"SQ_INSTS_{k}"] / waves / steps
                              for k in ("VALU", "LDS", "SALU", "VMEM_RD") if f"SQ_INSTS_{k}" in c},
        "wave_time_split": {k: c[f"SQ_{k}"] / c["SQ_WAVE_CYCLES"]
                            for k in ("ACTIVE_INST_ANY", "WAIT_INST_ANY", "WAIT_ANY")},
        "formulas": {"valu_busy": "4*SQ_ACTIVE_INST_VALU / (4 SIMDs * 256 CUs * GRBM_GUI_ACTIVE/8)",
                     "lds_busy": "SQ_LDS_IDX_ACTIVE / (256 CUs * GRBM_GUI_ACTIVE/8)"},
    }
    d = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(d, exist_ok=True)
    name = sys.argv[5] if len(sys.argv) > 5 else "resident_sq.json"
    json.dump(out, open(os.path.join(d, name), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
