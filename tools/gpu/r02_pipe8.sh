set -o pipefail
export PYTHONUNBUFFERED=1
# pipe6 (production, -1) vs pipe8 (64) vs epilogue-free builds (39 = pipe6, 65 = pipe8)
timeout -k 10 200 python -u tools/gemm_bench.py --epi bias --shapes fc1,qkv,o_proj,fc2 --variants=-1,64,-1,64 > gpurun_out/r02_pipe8.log 2>&1 && \
timeout -k 10 200 python -u tools/gemm_bench.py --epi gelu --shapes fc1 --variants=-1,64,39,65 >> gpurun_out/r02_pipe8.log 2>&1
