# Round 4 step 25: pipe10 as production for the non-split gelu_tanh / quick_gelu GEMMs (fc1): GPU suite,
# smoke, the pipe10 identity test, the SigLIP job and the DFN5B-H job (quick_gelu fc1).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v25}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit $?
tail -1 ${P}_smoke.log
MME_DEV=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu -k pipe10 \
    tests/test_gpu_kernels.py > ${P}_pipe10_pytest.log 2>&1 || { tail -20 ${P}_pipe10_pytest.log; exit 1; }
tail -1 ${P}_pipe10_pytest.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > ${P}_bench.log 2>&1 || exit $?
tail -1 ${P}_bench.log | cut -c1-120
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --no-cpu-baseline > ${P}_dfn5b_bench.log 2>&1 || exit $?
tail -1 ${P}_dfn5b_bench.log | cut -c1-120
