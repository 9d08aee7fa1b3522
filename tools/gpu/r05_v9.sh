# Round 5, step 9: in-job A/B of the persistent ViT-H attention (production kind 94 vs form 29 = kind 86
# in the same mix) on LAION-CLIP-H; the DFN5B-H fp8 kernel summary without the post-timed bf16 drift job.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v9
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
for i in 1 2; do
timeout -k 10 600 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline --no-parity > ${P}_laion_prod_$i.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline --no-parity --attn-form 29 > ${P}_laion_f29_$i.log 2>&1 || exit $?
done
for f in ${P}_laion_*_[12].log; do echo "$f $(tail -1 $f | cut -c80-130)"; done
rm -rf gpurun_out/prof
PROF_TIMEOUT=500 PROF_ARGS="--model Apple-DFN5B-H --fp8 --no-parity" bash tools/profile_bench.sh > ${P}_dfn5b_fp8_prof.log 2>&1 || exit $?
S=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$S" ${P}_Apple-DFN5B-H-fp8_kernel_stats.csv
rm -rf gpurun_out/prof
PROF_TIMEOUT=500 PROF_ARGS="--model LAION-CLIP-H --no-parity --attn-form 29" bash tools/profile_bench.sh > ${P}_laion_f29_prof.log 2>&1 || exit $?
S=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$S" ${P}_LAION-CLIP-H_f29_kernel_stats.csv
