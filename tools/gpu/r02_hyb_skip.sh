set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention_m32 and 62" > gpurun_out/r02_hyb_skip_pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/attn_bench.py --cases siglip_vision --variants 0,92,0,92,0,92,0,92 > gpurun_out/r02_hyb_skip_bench.log 2>&1
