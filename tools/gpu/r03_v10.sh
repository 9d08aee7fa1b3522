set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx.py > gpurun_out/r03_v10_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/mx_rows_bench.py > gpurun_out/r03_v10_mx_rows.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r03_v10_dfn5b_fp8_bench.log 2>&1 && \
MME_FP8_OPROJ=1 timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r03_v10_dfn5b_fp8_oproj_bench.log 2>&1 && \
MME_FP8_OPROJ=1 timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread -m gpu -k fp8_dfn5b_full_size tests/test_gpu_mx.py > gpurun_out/r03_v10_oproj_drift.log 2>&1
rc=$?
tail -2 gpurun_out/r03_v10_pytest.log; grep -v amdgpu gpurun_out/r03_v10_mx_rows.log | tail -13
for f in gpurun_out/r03_v10_dfn5b_fp8_bench.log gpurun_out/r03_v10_dfn5b_fp8_oproj_bench.log; do tail -1 $f | cut -c1-200; done
grep -i 'fp8 vs bf16\|passed\|failed' gpurun_out/r03_v10_oproj_drift.log
exit $rc
