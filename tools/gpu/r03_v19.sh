set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "attention" tests/test_gpu_kernels.py > gpurun_out/r03_v19_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r03_v19_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_bench.py --variants 68,99,68,99,68,99 --cases dfn5b_vision > gpurun_out/r03_v19_attn_dfn5b.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/attn_bench.py --variants 95,100,95,100,95,100 --cases vitH_vision > gpurun_out/r03_v19_attn_vith.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r03_v19_attn_dfn5b.log | grep dfn5b; grep -v amdgpu gpurun_out/r03_v19_attn_vith.log | grep vitH
