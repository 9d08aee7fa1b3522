set -o pipefail
export PYTHONUNBUFFERED=1
for e in bias res resper; do
timeout -k 10 300 python -u tools/gemm_bench.py --rows 174231 --shapes o_proj,1280:1280 --epi $e --variants=-1 --iters 10 >> gpurun_out/r02_resper.log 2>&1 || exit 1
done
