# Round-6 final measurement set, part A2 (RUN=r06_final2): the PMC / bench / profile half of part A; the
# original header follows.
# GPU tests (production and development libraries), smoke, the PMC
# HBM-traffic passes at the headline bench geometry (first, so the bench line carries this build's traffic),
# the headline bench (+ CPU baseline, parity), its rocprofv3 kernel summary + timing check, and the
# production fc1 GEMM's counters.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r06_final}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
PMC_CONFIG='{"model": "SigLIP-400M", "n_images": 5000, "img_batch": 512, "txt_batch": 8192, "fp8": false}' \
PMC_BUILD="${RUN:-r06_final}" bash tools/pmc_job.sh > ${P}_pmc.log 2>&1 || { tail -5 ${P}_pmc.log; exit 1; }
tail -12 ${P}_pmc.log
cp gpurun_out/hbm_traffic.json profiles/hbm_traffic.json  # this build's traffic on the bench line
timeout -k 10 600 python -u bench.py > ${P}_bench.log 2>&1 || exit $?
tail -1 ${P}_bench.log | cut -c1-200
rm -rf gpurun_out/prof
PROF_TIMEOUT=500 bash tools/profile_bench.sh > ${P}_prof.log 2>&1 || exit $?
S=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$S" ${P}_bench_kernel_stats.csv
python3 tools/check_profile.py ${P}_bench_kernel_stats.csv ${P}_bench.log > ${P}_timing_check.json && cat ${P}_timing_check.json
EPI=gelu SHAPES=fc1 bash tools/pmc_gemm_util.sh > ${P}_pmc_gemm_util.log 2>&1 || { tail -5 ${P}_pmc_gemm_util.log; exit 1; }
tail -20 ${P}_pmc_gemm_util.log
