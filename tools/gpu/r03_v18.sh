set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "attention" tests/test_gpu_kernels.py > gpurun_out/r03_v18_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r03_v18_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_bench.py --variants 92,96,97,98,92,96,97,98,92,96,97,98 --cases siglip_vision > gpurun_out/r03_v18_attn_ab.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r03_v18_attn_ab.log | grep siglip
