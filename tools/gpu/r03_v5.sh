set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03_v5_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r03_v5_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_v5_smoke.log 2>&1 && \
MME_DEV=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "pipe9 or attention_m32" tests/test_gpu_kernels.py > gpurun_out/r03_v5_devtests.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03_v5_bench.log 2>&1 && \
PROF_TIMEOUT=500 bash tools/profile_bench.sh > gpurun_out/r03_v5_prof.log 2>&1 && \
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --variants 92,93,92,93,92,93,92,93 --cases siglip_vision > gpurun_out/r03_v5_attn.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 > gpurun_out/r03_v5_colpali_bench.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu -k "fp8_dfn5b_full_size or colpali_full_geometry" tests/ > gpurun_out/r03_v5_fp8_colpali_tests.log 2>&1
