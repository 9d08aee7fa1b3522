#!/bin/bash
# Issue / MFMA-busy / clock counters of the production GEMM (pipe8) on one encoder shape
# (tools/gemm_bench.py, default fc1 at M = 186 624), one rocprofv3 --pmc pass per counter
# group (kernel trace only). Per dispatch: GRBM_GUI_ACTIVE / 8 XCDs / kernel time = the clock
# the chip held; SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x those cycles) = MFMA pipe utilisation.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm_util
mkdir -p $OUT
CMD="python3 tools/gemm_bench.py --iters 2 --epi ${EPI:-bias} --shapes ${SHAPES:-fc1} --variants=${VARIANTS:--1}"
i=0
for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
dur = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_gemm_util/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_pipe" not in k:
            continue
        k = k[:100]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])].add((f, r.get("Dispatch_Id")))
for f in glob.glob("gpurun_out/pmc_gemm_util/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_pipe" in r["Kernel_Name"]:
            dur[r["Kernel_Name"][:100]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for k, d in acc.items():
    # each counter comes from one pass: average over the dispatches of that pass
    row = {"dispatches": max(len(cnt[(k, c)]) for c in d),
           **{c: v / max(len(cnt[(k, c)]), 1) for c, v in sorted(d.items())}}
    if dur[k]:
        ns = sum(dur[k]) / len(dur[k])
        row["avg_ns"] = ns
        if "GRBM_GUI_ACTIVE" in row:  # summed over the 8 XCDs
            row["clock_ghz"] = row["GRBM_GUI_ACTIVE"] / 8 / ns
            if "SQ_VALU_MFMA_BUSY_CYCLES" in row:  # over 256 CUs x 4 SIMDs at that clock
                row["mfma_busy_frac"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * row["GRBM_GUI_ACTIVE"] / 8)
    out[k] = row
json.dump(out, open("gpurun_out/pmc_gemm_util/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
