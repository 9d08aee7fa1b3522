set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc gpurun_out/pmc_gemm_util
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_encoders.py > gpurun_out/r02_v2b_tests.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r02_v2b_bench.log 2>&1 && \
PROF_TIMEOUT=500 bash tools/profile_bench.sh > gpurun_out/r02_v2b_prof.log 2>&1 && \
PMC_TIMEOUT=400 bash tools/pmc_gemm.sh > gpurun_out/r02_v2b_pmc.log 2>&1 && \
VARIANTS=-1 bash tools/pmc_gemm_util.sh > gpurun_out/r02_v2b_pmc_util.log 2>&1
