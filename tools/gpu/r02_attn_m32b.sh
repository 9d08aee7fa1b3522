set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention" > gpurun_out/r02_attn_m32b_pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/attn_bench.py --cases siglip_vision,dfn5b_vision,vitH_vision --variants 0,60,68,73,75,76,0,60,68,73,75,76 > gpurun_out/r02_attn_m32b_bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > gpurun_out/r02_m32_laion_clip_h_bench.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model Apple-DFN5B-H --no-cpu-baseline > gpurun_out/r02_m32_dfn5b_bf16_bench.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r02_m32_dfn5b_fp8_bench.log 2>&1
