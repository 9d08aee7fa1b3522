#!/bin/bash
# Stall / LDS / cache counters of the GEMM microbenchmark (fc1 shape), one pass per group.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ctr
mkdir -p $OUT
CMD="python3 tools/gemm_bench.py --shapes ${SHAPES:-fc1} --iters 3"
i=0
for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob("gpurun_out/pmc_ctr/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r.get("Dispatch_Id"))
for k, d in acc.items():
    n = len(cnt[k])
    print(k, "dispatches", n)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v / max(n,1):.4g}")
PY
