# Round 6, second session, v8: the production GPU suite and smoke once more at HEAD (ops.py / bench.py changed
# after final set 2's part A1: the attention_short2 accounting family; kernels unchanged).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_s2_v8
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit $?
tail -1 ${P}_smoke.log
