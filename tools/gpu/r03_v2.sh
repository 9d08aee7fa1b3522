# dev A/B: pipe9 GEMM (variant 80) vs production pipe8; attention kind 63 vs 62 (variants 93 / 92)
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
export MME_DEV=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "pipe9 or attention_m32" tests/test_gpu_kernels.py > gpurun_out/r03_v2_devtests.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --variants -1,80,-1,80 --epi gelu --shapes qkv,fc1 > gpurun_out/r03_v2_gemm_gelu.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --variants -1,80,-1,80 --epi bias --shapes qkv,o_proj,fc1,fc2 > gpurun_out/r03_v2_gemm_bias.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --variants -1,80,-1,80 --epi res --shapes o_proj,fc2 > gpurun_out/r03_v2_gemm_res.log 2>&1 && \
timeout -k 10 300 python -u tools/attn_bench.py --variants 92,93,92,93 --cases siglip_vision > gpurun_out/r03_v2_attn.log 2>&1
