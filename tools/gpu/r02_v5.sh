set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r02_v5_pytest.log 2>&1
