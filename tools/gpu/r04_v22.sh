# Round 4 step 22: the rescale-threshold accuracy test (threshold forms vs exact-rescale forms vs fp64)
# and the dev grid test against kind 30, after the round-4 production switch.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v22}
MME_DEV=1 timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu \
    -k "threshold_vs_exact or production_grid" tests/test_gpu_kernels.py > ${P}_thr_pytest.log 2>&1
rc=$?; grep -E "mean err|production grid|passed|failed" ${P}_thr_pytest.log; exit $rc
