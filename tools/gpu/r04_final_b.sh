# Round-4 final measurement set, part B: every other BASELINE config on one GPU (fp8 with its whole-job
# drift), and the 2-rank same-device rehearsal of the sharded path.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_final}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
for m in OpenAI-CLIP-L LAION-CLIP-H Apple-DFN5B-H; do
  timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline > ${P}_${m}_bench.log 2>&1 || exit $?
done
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_Apple-DFN5B-H_fp8_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 > ${P}_ColPali-v1.3_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --same-device --n-images 1000 --no-cpu-baseline > ${P}_multirank2.log 2>&1 || exit $?
for f in ${P}_*bench.log ${P}_multirank2.log; do echo "$f $(tail -1 $f | cut -c1-160)"; done
