set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 600 python -u bench.py > gpurun_out/r02_s2h_bench.log 2>&1 && \
PROF_TIMEOUT=500 bash tools/profile_bench.sh > gpurun_out/r02_s2h_prof.log 2>&1
