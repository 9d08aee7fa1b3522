set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r03_v9_dfn5b_fp8_bench.log 2>&1 && \
PROF_TIMEOUT=500 PROF_ARGS="--model Apple-DFN5B-H --fp8" bash tools/profile_bench.sh > gpurun_out/r03_v9_prof.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --no-cpu-baseline > gpurun_out/r03_v9_dfn5b_bf16_bench.log 2>&1
rc=$?
tail -1 gpurun_out/r03_v9_dfn5b_fp8_bench.log | cut -c1-300; tail -1 gpurun_out/r03_v9_dfn5b_bf16_bench.log | cut -c1-300
exit $rc
