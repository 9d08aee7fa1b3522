#!/usr/bin/env python3
"""Cross-check bench.py's live HIP-event GEMM timing against a rocprofv3 summary.

usage: check_profile.py <kernel_stats.csv> <bench json line file>
Prints the rocprof average duration of the GEMM kernels (all mme_gemm kernels
pooled, like bench.py's KernelTimer) next to the bench's avg_launch_ms.
"""
import csv
import json
import sys


def main(stats, bench):
    calls = tot = 0
    per = {}
    for r in csv.DictReader(open(stats)):
        name = r["Name"]
        if "gemm_" in name and "_kernel" in name:
            c, t = int(r["Calls"]), float(r["TotalDurationNs"])
            calls += c
            tot += t
            per[name.split("<")[0].split("::")[-1]] = per.get(name.split("<")[0].split("::")[-1], 0) + c
    line = [l for l in open(bench) if l.startswith("{")][-1]
    b = json.loads(line)["roofline"]
    rp = tot / calls / 1e6
    print(json.dumps({"rocprof_gemm_calls": calls, "rocprof_gemm_avg_ms": round(rp, 4),
                      "bench_gemm_launches": b["launches"], "bench_avg_launch_ms": b["avg_launch_ms"],
                      "ratio": round(b["avg_launch_ms"] / rp, 4), "kernels": per}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
