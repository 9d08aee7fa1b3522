#!/usr/bin/env python3
"""Attribute kernel dispatches of a rocprofv3 kernel trace (bench.py --steps K --warmup W) to the
bench phases: every mme_sim_topk launch is listed in dispatch order with its duration, start time
and phase (warmup / timed step / post-timed parity checker / post-timed host-inputs job: bench.py runs
sim_topk 3 times per job step, 3 more times in retrieval_parity after the timed region, and 3 more in
the streamed host-inputs job that follows it). Also buckets the torch copy kernels
(__amd_rocclr_copyBuffer) by phase, so copies inside the timed region would show.

usage: trace_phases.py <kernel_trace.csv> <warmup> <steps>"""
import csv
import json
import sys


def main(path, warmup, steps):
    rows = list(csv.DictReader(open(path)))
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    sim = [r for r in rows if "sim_topk_kernel" in r["Kernel_Name"]]
    sim.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = []
    for i, r in enumerate(sim):
        job = i // 3
        phase = ("warmup" if job < warmup else "timed" if job < warmup + steps else
                 "parity (post-timed)" if job == warmup + steps else "host-inputs job (post-timed)")
        out.append({"dispatch": int(r["Dispatch_Id"]), "phase": phase,
                    "ms": round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 3),
                    "start_s": round((int(r["Start_Timestamp"]) - t0) / 1e9, 3)})
    # phase boundaries by time: end of the last warmup / timed sim_topk triple
    ends = [int(sim[3 * j + 2]["End_Timestamp"]) for j in range(len(sim) // 3)]
    copies = {}
    for r in rows:
        if "copyBuffer" not in r["Kernel_Name"]:
            continue
        t = int(r["Start_Timestamp"])
        j = next((i for i, e in enumerate(ends) if t <= e), len(ends))
        ph = ("warmup" if j < warmup else "timed" if j < warmup + steps else "post-timed")
        c = copies.setdefault(ph, [0, 0.0])
        c[0] += 1
        c[1] += (int(r["End_Timestamp"]) - t) / 1e6
    print(json.dumps({"sim_topk_dispatches": out,
                      "copy_kernels_by_phase": {k: {"calls": v[0], "ms": round(v[1], 2)} for k, v in copies.items()}},
                     indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
