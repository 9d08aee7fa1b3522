# Round 6, second session: the container was re-created, so libmme.so was rebuilt from the same
# sources; re-run the production GPU suite, smoke and the headline bench on the rebuilt library.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_s2
timeout -k 10 600 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > ${P}_bench.log 2>&1 || exit $?
tail -1 ${P}_bench.log | cut -c1-300
