# Round 4 step 12: GEMM / mx / attention kernel tests after the epilogue template change (production
# pipe9 must be unchanged), the dev pipe10 identity test, and one headline bench.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v12}
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
    tests/test_gpu_mx.py > ${P}_kernels_pytest.log 2>&1
rc=$?; tail -2 ${P}_kernels_pytest.log; [ $rc -ne 0 ] && exit $rc
MME_DEV=1 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu -k "pipe10 or pingpong" \
    tests/test_gpu_kernels.py > ${P}_dev_pytest.log 2>&1
rc=$?; tail -2 ${P}_dev_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > ${P}_bench.log 2>&1 || exit $?
tail -1 ${P}_bench.log | cut -c1-200
