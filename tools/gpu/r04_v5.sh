# Round 4 step 5: mx11 (fp8 GEMM on pipe9's whole-line ring, mx_srow scale planes) -- mx tests
# (quantiser / planes bit-exact, every form bit-identical to the round-2 kernel), A/B against mx10
# (form 10) at the DFN5B-H fp8 job's execution batch, the fp8 job bench; then the attention skip
# bit-identity tests (production pairs 65/41, 62/58; dev pair 38/64).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v5}
timeout -k 10 400 python -u -m pytest -q -rs --maxfail=3 --timeout 200 --timeout-method thread -m "gpu and not slow" \
    tests/test_gpu_mx.py > ${P}_mx_pytest.log 2>&1
rc=$?; tail -3 ${P}_mx_pytest.log; [ $rc -ne 0 ] && exit $rc
R=$((417*730))
timeout -k 10 300 python -u tools/gemm_bench.py --rows $R --variants=-1 --epi none --mx \
    --mx-variants=-1,10,-1,10 --mx-epi job --shapes h_qkv,h_fc1,h_fc2 > ${P}_mx11_ab_job.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_bench.py --rows $R --variants=-1 --epi none --mx \
    --mx-variants=-1,10,-1,10 --mx-epi none --shapes h_qkv,h_fc1,h_fc2 > ${P}_mx11_ab_plain.log 2>&1 || exit $?
grep -h "mx8" ${P}_mx11_ab_*.log | cut -c1-120
timeout -k 10 400 python -u bench.py --model Apple-DFN5B-H --fp8 --steps 3 --warmup 1 --no-cpu-baseline \
    > ${P}_dfn5b_fp8_bench.log 2>&1 || exit $?
tail -1 ${P}_dfn5b_fp8_bench.log | cut -c1-400
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -m gpu -k "skip_bit_identical" \
    tests/test_gpu_kernels.py > ${P}_skip_prod.log 2>&1; rc=$?
grep -E "kind |passed|failed" ${P}_skip_prod.log | tail -16
[ $rc -gt 1 ] && exit $rc
MME_DEV=1 timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -m gpu -k "8wave_skip" \
    tests/test_gpu_kernels.py > ${P}_skip_dev.log 2>&1
grep -E "kinds |passed|failed" ${P}_skip_dev.log | tail -10
