# Round 6, step 3: the exact-erf GELU as a sigmoid of a degree-6 polynomial (common.h gelu_erf2) against
# round 5's erfc fit (the same source built before the change: mme/libmme_ab_erfc.so, via MME_LIB):
# fc1 activation cost at LAION's / SigLIP's fc1 shapes, the LAION-CLIP-H job A/B on one box, and the
# accuracy tests of the new form.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v3
OLD=multimodal-embedding_amd/mme/libmme_ab_erfc.so
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_kernels.py -k "gelu_erf_fp32 or activation_vs_float64" > ${P}_pytest.log 2>&1 || exit 1
for r in 1 2; do
for e in bias gelu erf; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 116935 --shapes h_fc1 --epi $e --variants=-1 >> ${P}_gemm.log 2>&1 || exit 1
done
MME_LIB=$OLD timeout -k 10 200 python -u tools/gemm_bench.py --rows 116935 --shapes h_fc1 --epi erf --variants=-1 >> ${P}_gemm_old.log 2>&1 || exit 1
done
for r in 1 2; do
timeout -k 10 400 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > ${P}_laion_new_$r.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 400 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > ${P}_laion_old_$r.log 2>&1 || exit 1
done
grep TFLOP ${P}_gemm.log ${P}_gemm_old.log
grep -h -o '"value": [0-9.]*' ${P}_laion_*.log
