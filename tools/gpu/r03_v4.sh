set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out

MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --variants=-1,80,-1,80 --epi gelu --shapes qkv,fc1 > gpurun_out/r03_v4_gemm_gelu.log 2>&1 && \
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --variants=-1,80,-1,80 --epi bias --shapes qkv,o_proj,fc1,fc2 > gpurun_out/r03_v4_gemm_bias.log 2>&1 && \
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --variants=-1,80,-1,80 --epi res --shapes o_proj,fc2 > gpurun_out/r03_v4_gemm_res.log 2>&1 && \
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --variants 92,93,92,93 --cases siglip_vision > gpurun_out/r03_v4_attn.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 > gpurun_out/r03_v4_colpali_bench.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu -k "fp8_dfn5b_full_size or colpali_full_geometry" tests/ > gpurun_out/r03_v4_fp8_colpali_tests.log 2>&1
