# Round-3 final measurement set: GPU tests, smoke, the headline bench (+ CPU baseline, parity),
# its rocprofv3 kernel summary, every BASELINE config on one GPU, and the N-rank rehearsal.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r03_final}
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > ${P}_bench.log 2>&1 || exit $?
tail -1 ${P}_bench.log | cut -c1-200
PROF_TIMEOUT=500 bash tools/profile_bench.sh > ${P}_prof.log 2>&1 || exit $?
for m in OpenAI-CLIP-L LAION-CLIP-H Apple-DFN5B-H; do
  timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline > ${P}_${m}_bench.log 2>&1 || exit $?
done
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_Apple-DFN5B-H_fp8_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 > ${P}_ColPali-v1.3_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --same-device --n-images 1000 --no-cpu-baseline > ${P}_multirank2.log 2>&1 || exit $?
for f in ${P}_*bench.log ${P}_multirank2.log; do echo "$f $(tail -1 $f | cut -c1-160)"; done
