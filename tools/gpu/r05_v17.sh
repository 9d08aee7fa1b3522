# Round 5, step 17: mx12 (one prologue path per tile, SGPR-read hazard padded in its asm loads) -- which tiles of the persistent walk mx12 / its seam variants get wrong (v, block, k).
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
MX12_FORMS=12,14 timeout -k 10 300 python -u tools/mx12_debug.py 304410 5120 1280 2 > gpurun_out/r05_v17_debug.log 2>&1 || exit 1
MX12_FORMS=12,14 timeout -k 10 300 python -u tools/mx12_debug.py 304410 5120 1280 0 >> gpurun_out/r05_v17_debug.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05_v17_debug.log
