# Round 5, step 22: mx form 16 (form 15 + the mx8 output's block absmax by DPP quad permutes and
# quick_gelu in packed f32): bit-identity against mx11, fp8 GEMM microbench and job A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v22
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_mx.py -k "mx12_bit_identical or quantize or layernorm_mx" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --rows 304410 --shapes h_qkv,h_fc1,h_fc2 --mx --mx-epi job --mx-variants=-1,16,-1,16 --variants=-1 > ${P}_gemm.log 2>&1 || exit 1
grep -i "mx" ${P}_gemm.log | tail -14
for i in 1 2; do
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline --no-parity > ${P}_fp8_prod_$i.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline --no-parity --mx-form 16 > ${P}_fp8_mx16_$i.log 2>&1 || exit $?
done
for f in ${P}_fp8_*_[12].log; do echo "$f $(tail -1 $f | cut -c80-150)"; done
