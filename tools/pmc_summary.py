#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel family.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B
request of a wide (16 B/lane) coalesced stream, i.e. half the bytes; the GEMM's
LDS-DMA staging is exactly that access shape, so FETCH_SIZE is doubled.
WRITE_SIZE is exact for 16-B-per-lane stores. Units: KB (x1024).
"""
import csv
import glob
import json
import os
import sys


def load(d, counter):
    rows = {}
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (r["Kernel_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))
            rows[key] = rows.get(key, 0.0) + float(r["Counter_Value"])
    return rows


def family(name):
    for k in ("gemm_pipe9_kernel", "gemm_pipe8_kernel", "gemm_pipe6_kernel", "gemm_pipe4_kernel", "gemm_pipe3_kernel",
              "gemm_tn_kernel", "gemm_mx_kernel", "attn_hyb_kernel", "attn_m32_kernel", "attn_short_kernel",
              "attn_fwd_kernel", "attn_pipe_kernel", "attn_dma_kernel", "layernorm_kernel", "sim_topk_kernel",
              "resample_patch_p_kernel", "resample_patch_fused_kernel", "resample_v_patch_kernel",
              "probe_attn_img_kernel", "probe_attn_kernel", "row_part_combine_lds_kernel"):
        if k in name:
            return k
    return "other"


def main(d):
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    fam = {}
    for (name, _), v in fetch.items():
        f = fam.setdefault(family(name), {"launches": 0, "fetch_kb": 0.0, "write_kb": 0.0})
        f["launches"] += 1
        f["fetch_kb"] += v
    for (name, _), v in write.items():
        fam.setdefault(family(name), {"launches": 0, "fetch_kb": 0.0, "write_kb": 0.0})["write_kb"] += v
    out = {}
    for k, f in fam.items():
        n = max(f["launches"], 1)
        out[k] = {"launches": f["launches"],
                  "hbm_bytes_per_launch": (2 * f["fetch_kb"] + f["write_kb"]) * 1024 / n,
                  "fetch_bytes_per_launch_corrected": 2 * f["fetch_kb"] * 1024 / n,
                  "write_bytes_per_launch": f["write_kb"] * 1024 / n}
    # the mme_gemm entry point as bench.py's KernelTimer sees it: every GEMM kernel together
    fams = [f for k, f in fam.items() if k.startswith("gemm_")]
    n = sum(f["launches"] for f in fams)
    if n:
        out["mme_gemm"] = {"launches": n,
                           "hbm_bytes_per_launch": sum(2 * f["fetch_kb"] + f["write_kb"] for f in fams) * 1024 / n}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
