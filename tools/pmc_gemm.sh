#!/bin/bash
# HBM traffic of the GEMM kernel: two separate rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE; they do not fit one pass on gfx950), kernel-trace only, over one full
# bench job (the launch mix bench.py's per-launch algorithmic bytes average over;
# PMC_IMAGES=512 for a quicker, differently batched one). Aggregated by tools/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS="--n-images ${PMC_IMAGES:-5000} --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timer"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PMC_TIMEOUT:-400} rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run \
      -- python3 bench.py $ARGS > $OUT/$C.log 2>&1 || { echo "pmc pass $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
