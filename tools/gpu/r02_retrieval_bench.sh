set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_retrieval.py -s > gpurun_out/r02_g1_pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 > gpurun_out/r02_g1_bench.log 2>&1
