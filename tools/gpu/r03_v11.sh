set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread -m gpu -k "m32_skip" tests/test_gpu_kernels.py > gpurun_out/r03_v11_pytest.log 2>&1
timeout -k 10 300 python -u tools/attn_bench.py --variants 68,94,68,94,68,94,68,94 --cases dfn5b_vision > gpurun_out/r03_v11_attn_dfn5b.log 2>&1 && \
timeout -k 10 300 python -u tools/attn_bench.py --variants 71,95,71,95,71,95,71,95 --cases vitH_vision > gpurun_out/r03_v11_attn_vith.log 2>&1
rc=$?
grep 'kinds\|passed\|failed' gpurun_out/r03_v11_pytest.log; grep -v amdgpu gpurun_out/r03_v11_attn_dfn5b.log | tail -8; grep -v amdgpu gpurun_out/r03_v11_attn_vith.log | tail -8
exit $rc
