set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/gemm_bench.py --rows 174231 --shapes o_proj,1280:1280,fc2 --epi res --variants=-1,40,41,42,43,39 --iters 10 >> gpurun_out/r02_stag.log 2>&1
