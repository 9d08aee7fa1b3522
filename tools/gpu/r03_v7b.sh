set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/preprocess_bench.py > gpurun_out/r03_v7_preprocess.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r03_v7_dfn5b_fp8_bench.log 2>&1 && \
SHAPES=fc1 timeout -k 10 500 bash tools/pmc_gemm_util.sh > gpurun_out/r03_v7_pmc_gemm_util_fc1.log 2>&1 && \
PMC_TIMEOUT=400 timeout -k 10 900 bash tools/pmc_gemm.sh > gpurun_out/r03_v7_pmc_traffic.log 2>&1
rc=$?
cat gpurun_out/r03_v7_preprocess.log | grep -v amdgpu
exit $rc
