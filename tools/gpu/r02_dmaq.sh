set -o pipefail
export PYTHONUNBUFFERED=1
# production (-1: pipe8 + per-wave epilogue) vs 72 (2 of 4 DMA pieces per step in the compute phase) vs 73 (all 4)
timeout -k 10 300 python -u tools/gemm_bench.py --epi bias --shapes fc1,qkv,fc2 --variants=-1,72,73,-1,72,73 > gpurun_out/r02_dmaq.log 2>&1
