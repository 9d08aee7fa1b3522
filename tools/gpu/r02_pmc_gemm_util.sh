set -o pipefail
export PYTHONUNBUFFERED=1
VARIANTS=-1 bash tools/pmc_gemm_util.sh > gpurun_out/r02_pmc_gemm_util.log 2>&1
