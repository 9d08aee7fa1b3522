set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision,dfn5b_vision,vitH_vision --variants 47,57,47,57 > gpurun_out/r02_attn_skip.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k attention >> gpurun_out/r02_attn_skip.log 2>&1
