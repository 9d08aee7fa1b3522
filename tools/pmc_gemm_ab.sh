#!/bin/bash
# L2-miss traffic of two GEMM kernel forms on one shape (tools/gemm_bench.py variants, e.g.
# VARIANTS=70,-1 = pipe8 vs pipe9 in libmme_dev.so): FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes (kernel trace only), summed per kernel name and divided by dispatches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ab
mkdir -p $OUT
CMD="python3 tools/gemm_bench.py --iters 2 --epi ${EPI:-bias} --shapes ${SHAPES:-fc1} --variants=${VARIANTS:-70,-1}"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $OUT/$C -o run -- $CMD > $OUT/$C.log 2>&1 || { echo "pass $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(lambda: collections.defaultdict(set))
for f in glob.glob("gpurun_out/pmc_ab/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_pipe" not in k:
            continue
        k = k.split("(")[0][-40:] + " " + k[k.find("<"):k.find("<") + 60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k][r["Counter_Name"]].add(r.get("Dispatch_Id"))
out = {}
for k, d in acc.items():
    row = {c: v / max(len(n[k][c]), 1) for c, v in d.items()}
    # gfx950: FETCH_SIZE reports half the bytes of wide streaming reads (MI355X_MICROARCH.md) -> x2; units KiB
    row["fetch_GB_corrected"] = row.get("FETCH_SIZE", 0) * 2 * 1024 / 1e9
    row["write_GB"] = row.get("WRITE_SIZE", 0) * 1024 / 1e9
    row["dispatches"] = max(len(s) for s in n[k].values())
    out[k] = row
print(json.dumps(out, indent=1))
PY
