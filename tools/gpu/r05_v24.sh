# Round 5, step 24: the fc1 activation's share of the GEMM at the ViT-H / LAION-CLIP-H fc1 shape
# (116 935 x 5 120 x 1 280) and SigLIP's (186 624 x 4 352 x 1 152): bias only vs gelu_tanh vs quick_gelu vs exact GELU.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v24
for r in 1 2; do
for e in bias gelu quick erf; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 116935 --shapes h_fc1 --epi $e --variants=-1 >> ${P}_gemm.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/gemm_bench.py --shapes fc1 --epi $e --variants=-1 >> ${P}_gemm.log 2>&1 || exit 1
done
done
grep "TFLOP" ${P}_gemm.log
