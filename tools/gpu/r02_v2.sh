set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
# pipe8 in production: kernel tests first (bit-identity vs pipe6), then the full suite, smoke, bench
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py > gpurun_out/r02_v2_kernels.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r02_v2_pytest.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_v2_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r02_v2_bench.log 2>&1
