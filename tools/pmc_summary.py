#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel family.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B
request of a wide (16 B/lane) coalesced stream, i.e. half the bytes; the GEMMs'
LDS-DMA staging and the 16-B loads of the HBM-bound kernels are that access shape,
so FETCH_SIZE is doubled. WRITE_SIZE is exact for 16-B-per-lane stores. Units: KB (x1024).

Families: "gemm" = every bf16 GEMM kernel (gemm_pipe9 / pipe6 / tn: what bench.py's
KernelTimer "gemm" family times through mme_gemm), "gemm_mx" = the mx8 GEMMs, and the
HBM-bound kernels by name (bench.py HBM_FAMILIES).

Usage: pmc_summary.py <pmc dir> [--config JSON --build LABEL --merge profiles/hbm_traffic.json]
"""
import argparse
import csv
import glob
import json
import os

NAMED = ("resample_patch_p_kernel", "rowstats_kernel", "layernorm_kernel", "l2norm_kernel", "attn_short_kernel",
         "attn_short2_kernel",
         "attn_hyb_kernel", "attn_m32_kernel", "attn_fwd_kernel", "sim_topk_kernel", "map_pool_kernel",
         "row_part_combine_lds_kernel", "layernorm_mx_kernel", "token_embed_kernel", "clip_embed_ln_kernel")


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
    if "gemm_mx" in name:
        return "gemm_mx"
    if "gemm_" in name:
        return "gemm"
    for k in NAMED:
        if k in name:
            return k
    return "other"


def summarize(d):
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
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--config", default=None, help="JSON of the bench configuration the passes ran")
    p.add_argument("--build", default="", help="label of the measured build (commit / round step)")
    p.add_argument("--merge", default=None, help="hbm_traffic.json to add / replace this configuration's entry in")
    a = p.parse_args()
    fams = summarize(a.dir)
    if not a.merge:
        print(json.dumps(fams, indent=1))
        return
    cfg = json.loads(a.config)
    try:
        doc = json.load(open(a.merge))
    except (OSError, ValueError):
        doc = {"note": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch, one job per configuration "
                       "(tools/pmc_job.sh); bench.py reports them where its launch counts match",
               "configs": []}
    doc["configs"] = [e for e in doc["configs"] if e.get("config") != cfg]
    doc["configs"].append({"config": cfg, "build": a.build, "families": fams})
    json.dump(doc, open(a.merge, "w"), indent=1)
    print(json.dumps(fams, indent=1))


if __name__ == "__main__":
    main()
