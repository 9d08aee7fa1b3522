set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "res_stats or row_part or pipe8 or rowstats" > gpurun_out/r02_s2c_pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r02_s2c_bench.log 2>&1 && \
PROF_TIMEOUT=500 bash tools/profile_bench.sh > gpurun_out/r02_s2c_prof.log 2>&1
