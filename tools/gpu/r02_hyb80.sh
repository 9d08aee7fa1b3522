set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention_m32 and (58 or 59 or 60 or 61)" > gpurun_out/r02_hyb80_pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/attn_bench.py --cases dfn5b_vision,vitH_vision,siglip_vision --variants 0,90,89,91,0,90,89,91,0,90 > gpurun_out/r02_hyb80_bench.log 2>&1
