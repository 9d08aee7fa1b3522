# Round 6, step 3: (a) the exact-erf GELU as a sigmoid of a degree-6 polynomial (common.h gelu_erf2) against
# round 5's erfc fit (the same source built before the change: mme/libmme_ab_erfc.so, via MME_LIB): accuracy
# tests, fc1 activation cost at LAION's fc1 shape, the LAION-CLIP-H job A/B on one box; (b) attention kind 96
# (kind 83's K / V DMA from fixed per-lane offsets): bit-identity test and A/B at SigLIP's 417-image batch;
# (c) the split grid's cost at SigLIP's N = 256 k + 128 shapes against the neighbouring multiples of 256.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v3
OLD=multimodal-embedding_amd/mme/libmme_ab_erfc.so
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_kernels.py -k "gelu_erf_fp32 or activation_vs_float64 or buffer_dma" > ${P}_pytest.log 2>&1 || exit 1
for r in 1 2 3; do
timeout -k 10 200 python -u tools/attn_bench.py --cases siglip_vision --batch 417 --variants 113,126 >> ${P}_attn.log 2>&1 || exit 1
done
for r in 1 2; do
for e in bias gelu erf; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 116935 --shapes h_fc1 --epi $e --variants=-1 >> ${P}_gemm.log 2>&1 || exit 1
done
MME_LIB=$OLD timeout -k 10 200 python -u tools/gemm_bench.py --rows 116935 --shapes h_fc1 --epi erf --variants=-1 >> ${P}_gemm_old.log 2>&1 || exit 1
done
for s in 1024:1152 1152:1152 1280:1152 1024:4352 1152:4352 1280:4352; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 303993 --shapes $s --epi resstats --variants=-1 >> ${P}_split.log 2>&1 || exit 1
done
for s in 3328:1152 3456:1152 3584:1152; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 303993 --shapes $s --epi bias --variants=-1 >> ${P}_split.log 2>&1 || exit 1
done
for r in 1 2; do
timeout -k 10 400 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > ${P}_laion_new_$r.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 400 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > ${P}_laion_old_$r.log 2>&1 || exit 1
done
for r in 1 2; do
timeout -k 10 400 python -u bench.py --no-cpu-baseline --attn-form 126 > ${P}_siglip_k96_$r.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > ${P}_siglip_k83_$r.log 2>&1 || exit 1
done
grep -h -o '"value": [0-9.]*' ${P}_laion_*.log ${P}_siglip_*.log
