# Round-6 final measurement set, part B2 (RUN=r06_final2): ColPali, the same-device rank rehearsals and the
# LAION / fp8 kernel summaries of part B below.
# every other BASELINE config on one GPU (fp8 with its whole-job drift,
# gated on decided rows), LAION-CLIP-H's and the fp8 job's PMC traffic at this build (mx11 included),
# the kernel summaries of those two jobs, and the same-device rank rehearsals (2 ranks; 3 uneven shards).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r06_final}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 > ${P}_ColPali-v1.3_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --same-device --n-images 1000 --no-cpu-baseline > ${P}_multirank2.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 3 --backend gloo --same-device --n-images 1001 --no-cpu-baseline > ${P}_multirank3.log 2>&1 || exit $?
for f in ${P}_*bench.log ${P}_multirank*.log; do echo "$f $(tail -1 $f | cut -c1-160)"; done
rm -rf gpurun_out/prof
PROF_TIMEOUT=500 PROF_ARGS="--model LAION-CLIP-H" bash tools/profile_bench.sh > ${P}_LAION-CLIP-H_prof.log 2>&1 || exit $?
S=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$S" ${P}_LAION-CLIP-H_kernel_stats.csv
rm -rf gpurun_out/prof
PROF_TIMEOUT=500 PROF_ARGS="--model Apple-DFN5B-H --fp8" bash tools/profile_bench.sh > ${P}_DFN5B-fp8_prof.log 2>&1 || exit $?
S=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$S" ${P}_Apple-DFN5B-H-fp8_kernel_stats.csv
