set -o pipefail
export PYTHONUNBUFFERED=1
for sh in 1152:1152 1152:4352 4352:1152; do
timeout -k 10 120 python -u tools/gemm_stamps.py --shape $sh --epi res >> gpurun_out/r02_stamps.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/gemm_stamps.py --shape $sh --epi bias >> gpurun_out/r02_stamps.log 2>&1 || exit 1
done
