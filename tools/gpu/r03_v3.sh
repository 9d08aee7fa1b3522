set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03_v3_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r03_v3_pytest.log
# a failing test is not a GPU fault: go on unless the run timed out / crashed
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_v3_smoke.log 2>&1 && \
MME_DEV=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "pipe9 or attention_m32" tests/test_gpu_kernels.py > gpurun_out/r03_v3_devtests.log 2>&1 && \
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --variants -1,80,-1,80 --epi gelu --shapes qkv,fc1 > gpurun_out/r03_v3_gemm_gelu.log 2>&1 && \
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --variants -1,80,-1,80 --epi bias --shapes qkv,o_proj,fc1,fc2 > gpurun_out/r03_v3_gemm_bias.log 2>&1 && \
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --variants -1,80,-1,80 --epi res --shapes o_proj,fc2 > gpurun_out/r03_v3_gemm_res.log 2>&1 && \
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --variants 92,93,92,93 --cases siglip_vision > gpurun_out/r03_v3_attn.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 > gpurun_out/r03_v3_colpali_bench.log 2>&1
