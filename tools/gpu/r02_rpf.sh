set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm" > gpurun_out/r02_rpf_pytest.log 2>&1 && \
( for v in -1 90 -1 90; do timeout -k 10 120 python -u tools/gemm_bench.py --shapes o_proj,fc2 --iters 10 --epi resstats --variants=$v || exit 1; timeout -k 10 120 python -u tools/gemm_bench.py --shapes o_proj,fc2 --iters 10 --epi res --variants=$v || exit 1; done ) > gpurun_out/r02_rpf_bench.log 2>&1
