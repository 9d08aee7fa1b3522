set -o pipefail
export PYTHONUNBUFFERED=1
# pipe8 block-wide epilogue (64) vs per-wave epilogue (71); max|diff| vs the first variant must be 0
timeout -k 10 300 python -u tools/gemm_bench.py --epi bias --shapes fc1,qkv,o_proj,fc2 --variants=64,71,64,71 > gpurun_out/r02_wepi.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --epi gelu --shapes fc1 --variants=64,71,64,71 >> gpurun_out/r02_wepi.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --epi res --shapes o_proj,fc2 --variants=64,71,64,71 >> gpurun_out/r02_wepi.log 2>&1
