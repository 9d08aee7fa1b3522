set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03_v8_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r03_v8_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_v8_smoke.log 2>&1 && \
timeout -k 10 300 python -u tools/preprocess_bench.py > gpurun_out/r03_v8_preprocess.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03_v8_bench.log 2>&1 && \
PROF_TIMEOUT=500 bash tools/profile_bench.sh > gpurun_out/r03_v8_prof.log 2>&1
rc2=$?
grep -v amdgpu gpurun_out/r03_v8_preprocess.log | tail -8; tail -1 gpurun_out/r03_v8_bench.log | cut -c1-400
exit $rc2
