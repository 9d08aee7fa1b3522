#!/bin/bash
# rocprofv3 kernel-trace summary of one bench step (no PMC in this pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-500} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${PROF_ARGS} > gpurun_out/prof/bench_stdout.log 2>&1
rc=$?
tail -3 gpurun_out/prof/bench_stdout.log
echo "rocprof rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
