# Round 4 step 24: ViT-H (hd 80, T 257) attention in smaller blocks (dev kinds 91: 5 waves, 92: 4 waves,
# 93: 5 waves held to 128 VGPRs) against production kind 86 (9 waves, one block per CU), at LAION-CLIP-H's
# 455-image execution batch; fp32-reference tests of the new kinds.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v24}
MME_DEV=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    -k "test_attention_m32 and (91 or 92 or 93)" tests/test_gpu_kernels.py > ${P}_vith_pytest.log 2>&1 || { tail -20 ${P}_vith_pytest.log; exit 1; }
tail -1 ${P}_vith_pytest.log
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --cases vitH_vision --batch 455 \
    --variants 0,121,122,123,0,121,122,123,0,121,122,123 > ${P}_vith_bench.log 2>&1 || { cat ${P}_vith_bench.log; exit 1; }
cat ${P}_vith_bench.log
