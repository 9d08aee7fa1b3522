# Round 4 step 6: the zero-operand MFMA probe (cause of the attention skip's rare differences), the
# matrix / vector ping-pong attention (dev kinds 70-72) against kind 62: bit-identity tests, then
# timing at the SigLIP job's execution batch (417 images x 16 heads, T 729, hd 72).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v6}
timeout -k 10 60 ./tools/mfma_zero_probe > ${P}_mfma_zero_probe.log 2>&1 || { tail -5 ${P}_mfma_zero_probe.log; exit 1; }
cat ${P}_mfma_zero_probe.log
MME_DEV=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu -k "pingpong" \
    tests/test_gpu_kernels.py > ${P}_pp_pytest.log 2>&1; rc=$?
tail -4 ${P}_pp_pytest.log
[ $rc -gt 1 ] && exit $rc
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --batch 417 \
    --variants 92,100,101,102,92,100,101,102 > ${P}_pp_bench.log 2>&1 || exit $?
cat ${P}_pp_bench.log
timeout -k 10 400 python -u bench.py --model Apple-DFN5B-H --fp8 --steps 3 --warmup 1 --no-cpu-baseline \
    > ${P}_dfn5b_fp8_bench.log 2>&1 || exit $?
tail -1 ${P}_dfn5b_fp8_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['fp8_drift'], d['parity']['rows'])"
