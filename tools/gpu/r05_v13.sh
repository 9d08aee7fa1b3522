# Round 5, step 13: where mx12's mx8-output epilogue differs from mx11's.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/mx12_debug.py 304410 5120 1280 > gpurun_out/r05_v13_debug.log 2>&1
timeout -k 10 200 python -u tools/mx12_debug.py 304410 5120 1280 0 >> gpurun_out/r05_v13_debug.log 2>&1
timeout -k 10 200 python -u tools/mx12_debug.py 8192 5120 1280 >> gpurun_out/r05_v13_debug.log 2>&1
cat gpurun_out/r05_v13_debug.log | grep -v amdgpu.ids
