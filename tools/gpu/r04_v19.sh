# Round 4 step 19: the 2^8 rescale threshold alone (dev kinds 82: on the stagger, 83: on kind 62's loop)
# against kind 62 / 80: time at the SigLIP job batch, error vs an fp64 reference, fp32-reference tests.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v19}
MME_DEV=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    -k "test_attention_m32 and (82 or 83)" tests/test_gpu_kernels.py > ${P}_thr_pytest.log 2>&1 || { tail -20 ${P}_thr_pytest.log; exit 1; }
tail -1 ${P}_thr_pytest.log
MME_DEV=1 timeout -k 10 300 python -u tools/attn_err.py --variants 0,110,112,113 > ${P}_thr_err.log 2>&1 || { cat ${P}_thr_err.log; exit 1; }
MME_DEV=1 timeout -k 10 300 python -u tools/attn_err.py --variants 0,113 --scale 4 >> ${P}_thr_err.log 2>&1 || { cat ${P}_thr_err.log; exit 1; }
cat ${P}_thr_err.log
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --batch 417 \
    --variants 0,113,112,110,0,113,112,110,0,113,112,110 > ${P}_thr_bench.log 2>&1 || { cat ${P}_thr_bench.log; exit 1; }
cat ${P}_thr_bench.log
