set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/pmc gpurun_out/pmc_gemm_util
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r02_s2f_pytest.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_s2f_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r02_s2f_bench.log 2>&1 && \
PROF_TIMEOUT=500 bash tools/profile_bench.sh > gpurun_out/r02_s2f_prof.log 2>&1 && \
PMC_TIMEOUT=400 bash tools/pmc_gemm.sh > gpurun_out/r02_s2f_pmc.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model OpenAI-CLIP-L --no-cpu-baseline > gpurun_out/r02_s2f_clip_l_bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > gpurun_out/r02_s2f_laion_clip_h_bench.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model Apple-DFN5B-H --no-cpu-baseline > gpurun_out/r02_s2f_dfn5b_bf16_bench.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r02_s2f_dfn5b_fp8_bench.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 --no-cpu-baseline > gpurun_out/r02_s2f_colpali_bench.log 2>&1
