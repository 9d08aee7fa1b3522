set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -rs --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03_v1_pytest.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_v1_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 > gpurun_out/r03_v1_colpali_bench.log 2>&1
