# Round 5, step 12: mx12 (persistent mx11) bit-identity, shape A/B against mx11 with the fp8 job's
# epilogues at DFN5B-H's execution batch (14 = mx12 without DMA under the epilogue), and the fp8 job A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v12
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_mx.py -k "mx12 or wave_epilogue" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python -u tools/gemm_bench.py --rows 304410 --iters 5 --variants=-1 --mx --mx-variants 11,12,14 --mx-epi job --shapes h_qkv,h_fc1,h_fc2 >> ${P}_gemm.log 2>&1 || exit 1
done
grep mx8 ${P}_gemm.log
for i in 1 2; do
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline --no-parity > ${P}_fp8_mx11_$i.log 2>&1 || exit $?
MME_MX_VARIANT=12 timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline --no-parity > ${P}_fp8_mx12_$i.log 2>&1 || exit $?
done
for f in ${P}_fp8_*_[12].log; do echo "$f $(tail -1 $f | cut -c80-130)"; done
