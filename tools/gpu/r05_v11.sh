# Round 5, step 11: the verdict's o_proj-in-fp8 trial under the whole-job drift bounds (MME_FP8_OPROJ=1:
# o_proj on mx11 with its input quantised by a separate pass), A/B against the production fp8 mode.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v11
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
for i in 1 2; do
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_fp8_prod_$i.log 2>&1 || exit $?
MME_FP8_OPROJ=1 timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_fp8_oproj_$i.log 2>&1 || exit $?
done
for f in ${P}_fp8_*_[12].log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["fp8_drift"])')"; done
