set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
( for e in bias res resstats resper bias res resstats resper; do timeout -k 10 120 python -u tools/gemm_bench.py --shapes o_proj,fc2 --iters 10 --epi $e || exit 1; done ) > gpurun_out/r02_res_cost.log 2>&1
