set -o pipefail
export PYTHONUNBUFFERED=1
# production (-1: pipe8 + per-wave epilogue) vs 74 (persistent pipe8); max|diff| must be 0
timeout -k 10 300 python -u tools/gemm_bench.py --epi bias --shapes fc1,qkv,o_proj,fc2 --variants=-1,74,-1,74 > gpurun_out/r02_pers8.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --epi gelu --shapes fc1 --variants=-1,74,-1,74 >> gpurun_out/r02_pers8.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --rows 100032 --epi bias --shapes fc1,qkv --variants=-1,74,-1,74 >> gpurun_out/r02_pers8.log 2>&1
