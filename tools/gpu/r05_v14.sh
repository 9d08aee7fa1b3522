# Round 5, step 14: mx12's seam variants (13: + lgkmcnt(0) before the post-epilogue barrier, 14: no DMA
# under the epilogue) against mx11 on the mx8-output epilogue, three runs each.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for act in 0 2; do
MX12_FORMS=12,13,14 timeout -k 10 300 python -u tools/mx12_debug.py 304410 5120 1280 $act >> gpurun_out/r05_v14_debug.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r05_v14_debug.log
