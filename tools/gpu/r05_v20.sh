# Round 5, step 20: mx form 15 (mx11 with the bias loaded up front) bit-identity and the DFN5B-H fp8 job
# A/B (production = compiled bf16 epilogues, mx 15); GEMM bit-identity of the compiled epilogues.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v20
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 500 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_mx.py tests/test_gpu_kernels.py -k "mx12_bit_identical or form95 or compiled_epilogues or dispatched_fc1" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for i in 1 2; do
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline --no-parity > ${P}_fp8_prod_$i.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline --no-parity --mx-form 15 > ${P}_fp8_mx15_$i.log 2>&1 || exit $?
done
for f in ${P}_fp8_*_[12].log; do echo "$f $(tail -1 $f | cut -c80-150)"; done
