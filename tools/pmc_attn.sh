#!/bin/bash
# Issue / stall / LDS counters of the production attention kernel on SigLIP vision
# (B 256, T 729, 16 heads x 72), one rocprofv3 --pmc pass per counter group (kernel trace only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_attn
mkdir -p $OUT
CMD="python3 tools/attn_bench.py --cases ${CASES:-siglip_vision} --variants ${VARIANTS:-0}"
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob("gpurun_out/pmc_attn/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "attn" not in k:
            continue
        k = k[:110]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r.get("Dispatch_Id"))
out = {}
for k, d in acc.items():
    n = max(len(cnt[k]), 1)
    out[k] = {"dispatches": n, **{c: v / n for c, v in sorted(d.items())}}
json.dump(out, open("gpurun_out/pmc_attn/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
