# Round 4 step 18: hd-72 attention VALU trims on the staggered kernel (dev kind 80: packed exp arguments +
# 2^8 rescale threshold; 81: packed exp arguments only) against kind 79 and production kind 62; identity /
# fp32-reference tests of the ring forms.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v18}
MME_DEV=1 timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread -m gpu \
    -k "ring_forms or (test_attention_m32 and (78 or 79 or 80 or 81))" tests/test_gpu_kernels.py > ${P}_ring_pytest.log 2>&1; rc=$?
grep -E "kinds 62|passed|failed|Error" ${P}_ring_pytest.log | tail -12
[ $rc -ne 0 ] && exit $rc
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --batch 417 \
    --variants 0,109,110,111,0,109,110,111,0,109,110,111 > ${P}_trim_bench.log 2>&1 || { cat ${P}_trim_bench.log; exit 1; }
cat ${P}_trim_bench.log
