set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention_m32 and (54 or 55 or 56 or 57)" > gpurun_out/r02_attn_pf_pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/attn_bench.py --cases siglip_vision,dfn5b_vision,vitH_vision,clipL_vision --variants 0,68,84,85,86,87,0,68,84,85,87 > gpurun_out/r02_attn_pf_bench.log 2>&1
