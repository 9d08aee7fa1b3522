# Round 6, step 7: attn_m32_kernel with the MFMA bias (kinds 99 / 100 / 101): accuracy against fp64 beside
# the kernels they extend, isolated timing at the jobs' batches (SigLIP 417 x T 729 hd 72 against kind 98,
# DFN5B 500 x T 730 and ViT-H 455 x T 257 hd 80 against kinds 87 / 86), all through mme_attention_qs.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v7
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_kernels.py -k "m32_mfma_bias" > ${P}_pytest.log 2>&1 || exit 1
for r in 1 2 3; do
timeout -k 10 200 python -u tools/attn_bench.py --qs --cases siglip_vision --batch 417 --variants 128,129,113 >> ${P}_attn.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/attn_bench.py --qs --cases dfn5b_vision --batch 500 --variants 117,130 >> ${P}_attn.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/attn_bench.py --qs --cases vitH_vision --batch 455 --variants 116,131 >> ${P}_attn.log 2>&1 || exit 1
done
