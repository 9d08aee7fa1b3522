set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_mx.py > gpurun_out/r03_v16_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r03_v16_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/ln_mx_bench.py > gpurun_out/r03_v16_ln_mx.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r03_v16_ln_mx.log
timeout -k 10 400 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r03_v16_dfn5b_fp8_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r03_v16_dfn5b_fp8_bench.log | cut -c1-200
