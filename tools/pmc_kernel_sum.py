#!/usr/bin/env python3
"""Per-dispatch means of every counter in one or more rocprofv3 --pmc output dirs, for the kernels
whose name contains a substring, plus derived figures (clock, MFMA / VALU busy fractions).

Usage: pmc_kernel_sum.py <name substring> <pmc dir> [<pmc dir> ...]
SQ_*_CYCLES that count quad-cycles (SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_*) are
reported raw; SQ_VALU_MFMA_BUSY_CYCLES counts cycles (MI355X_MICROARCH.md, per-instruction constants).
"""
import csv
import glob
import json
import os
import sys


def main():
    sub, dirs = sys.argv[1], sys.argv[2:]
    per = {}  # counter -> {dispatch: value}
    names = set()
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if sub not in r["Kernel_Name"]:
                    continue
                names.add(r["Kernel_Name"][:120])
                key = (d, r.get("Dispatch_Id") or r.get("Correlation_Id"))
                c = per.setdefault(r["Counter_Name"], {})
                c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
    out = {"kernels": sorted(names)}
    for k, v in sorted(per.items()):
        out[k] = {"dispatches": len(v), "mean": sum(v.values()) / max(len(v), 1)}
    m = {k: v["mean"] for k, v in out.items() if isinstance(v, dict)}
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        # MFMA-busy per SIMD: SQ_VALU_MFMA_BUSY_CYCLES sums over the chip's 1 024 SIMDs, GRBM_GUI_ACTIVE
        # over its 8 XCDs (one XCD's active cycles = GRBM_GUI_ACTIVE / 8; MI355X_MICROARCH.md, DVFS
        # give-back), so the busy fraction is MFMA cycles / (1 024 x GRBM_GUI_ACTIVE / 8) -- the same
        # normalisation as tools/pmc_gemm_util.sh (round 4 divided by 1 024 x GRBM_GUI_ACTIVE: 8x low)
        out["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
        out["xcd_active_cycles"] = m["GRBM_GUI_ACTIVE"] / 8
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
