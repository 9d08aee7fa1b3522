set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_encoders.py > gpurun_out/r02_v4_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --epi resstats --shapes o_proj,fc2 --variants=-1,47,-1,47 > gpurun_out/r02_v4_resstats_ab.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r02_v4_pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r02_v4_bench.log 2>&1
