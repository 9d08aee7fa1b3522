# Round 6, third session: GPU tests (production and development libraries) and smoke at HEAD.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r06_s3}
timeout -k 10 600 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
MME_DEV=1 timeout -k 10 600 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m "gpu and dev" tests/ > ${P}_dev_pytest.log 2>&1
rc=$?; tail -2 ${P}_dev_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit $?
tail -2 ${P}_smoke.log
