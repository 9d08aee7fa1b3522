#!/bin/bash
# HBM traffic per kernel family over ONE job of the bench geometry: two separate rocprofv3 --pmc
# passes (FETCH_SIZE, WRITE_SIZE: they do not share a pass on gfx950), kernel-trace only, each over
# `bench.py --steps 1 --warmup 0` without the host-streamed job and the parity checkers, so the
# launches are exactly one timed step's. Aggregated and merged into gpurun_out/hbm_traffic.json
# (copied to profiles/hbm_traffic.json) by tools/pmc_summary.py under the configuration key
# bench.py looks it up by. Env: PMC_MODEL (SigLIP-400M), PMC_ARGS (extra bench args, e.g. --fp8),
# PMC_CONFIG (the JSON key), PMC_BUILD (label).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
M=${PMC_MODEL:-SigLIP-400M}
OUT=gpurun_out/pmc_${PMC_TAG:-$M}
mkdir -p $OUT
ARGS="--model $M --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timer --no-parity --no-host-inputs ${PMC_ARGS}"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PMC_TIMEOUT:-400} rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run \
      -- python3 bench.py $ARGS > $OUT/$C.log 2>&1 || { echo "pmc pass $C failed"; tail -5 $OUT/$C.log; exit 1; }
done
[ -f gpurun_out/hbm_traffic.json ] || cp profiles/hbm_traffic.json gpurun_out/hbm_traffic.json 2>/dev/null
python3 tools/pmc_summary.py $OUT --config "$PMC_CONFIG" --build "${PMC_BUILD:-}" --merge gpurun_out/hbm_traffic.json \
    > $OUT/summary.json && cat $OUT/summary.json
