# Round 5, step 4: half-wave LayerNorm rows with per-width chunk counts (A/B vs round 4), the fp8 job
# with its whole-job drift_ok, and the whole-job drift test.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v4
OLD=multimodal-embedding_amd/build_exp/libmme_old.so
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_mx.py tests/test_gpu_kernels.py -k "layernorm or mx_quant" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
MME_LIB=$OLD timeout -k 10 120 python -u tools/ln_bench.py >> ${P}_ln_old.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/ln_bench.py >> ${P}_ln_new.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_dfn5b_fp8_bench.log 2>&1 || exit $?
tail -1 ${P}_dfn5b_fp8_bench.log | cut -c1-200
timeout -k 10 600 python -u -m pytest -q -s --timeout 500 --timeout-method thread tests/test_gpu_mx.py -k "whole_job_drift" > ${P}_drift_pytest.log 2>&1
tail -3 ${P}_drift_pytest.log
