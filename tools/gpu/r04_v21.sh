# Round 4 step 21: the whole GPU suite including the development forms (MME_DEV=1: libmme_dev.so).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v21}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
MME_DEV=1 timeout -k 10 1000 python -u -m pytest -q -rs --maxfail=10 --timeout 300 --timeout-method thread -m gpu tests/ \
    > ${P}_dev_pytest.log 2>&1
rc=$?; tail -3 ${P}_dev_pytest.log; exit $rc
