set -o pipefail
export PYTHONUNBUFFERED=1
for e in none bias res; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 174231 --shapes o_proj,1280:1280,fc1 --epi $e --variants=-1,38,39 --iters 10 >> gpurun_out/r02_epi.log 2>&1 || exit 1
done
