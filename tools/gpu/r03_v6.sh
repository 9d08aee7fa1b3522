set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx.py > gpurun_out/r03_v6_mx_pytest.log 2>&1 && \
MME_DEV=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "pipe9 or res_stats or gemm" tests/test_gpu_kernels.py > gpurun_out/r03_v6_gemm_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --rows 186880 --shapes h_qkv,h_fc1,h_fc2 --mx --mx-variants=0,-1,0,-1 > gpurun_out/r03_v6_mx_gemm.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r03_v6_dfn5b_fp8_bench.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --no-cpu-baseline > gpurun_out/r03_v6_dfn5b_bf16_bench.log 2>&1
rc=$?
tail -3 gpurun_out/r03_v6_mx_pytest.log; tail -2 gpurun_out/r03_v6_gemm_pytest.log; cat gpurun_out/r03_v6_mx_gemm.log
exit $rc
