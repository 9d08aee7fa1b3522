#!/bin/bash
# One GPU session: kernel/parity tests, then (only if no crash) a short bench.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
MARK="${MARK:-gpu and not slow}"
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m "$MARK" -q --maxfail=30 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: pytest ended abnormally"; exit $rc; fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  brc=$?
  tail -5 gpurun_out/bench.log
  echo "bench rc=$brc"
  exit $brc
fi
exit $rc
