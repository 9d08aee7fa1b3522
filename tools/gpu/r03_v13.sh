set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
MME_DEV=1 VARIANTS=70,-1 SHAPES=fc1 timeout -k 10 300 bash tools/pmc_gemm_ab.sh > gpurun_out/r03_v13_pmc_ab_fc1.log 2>&1
rc=$?; tail -30 gpurun_out/r03_v13_pmc_ab_fc1.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/pmc_ab
MME_DEV=1 VARIANTS=70,-1 SHAPES=o_proj timeout -k 10 300 bash tools/pmc_gemm_ab.sh > gpurun_out/r03_v13_pmc_ab_oproj.log 2>&1
rc=$?; tail -30 gpurun_out/r03_v13_pmc_ab_oproj.log
exit $rc
