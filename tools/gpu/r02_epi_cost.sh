set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
( for e in none bias gelu none bias gelu; do timeout -k 10 120 python -u tools/gemm_bench.py --shapes fc1,qkv --iters 10 --epi $e || exit 1; done ) > gpurun_out/r02_epi_cost.log 2>&1
