# Round 4 step 14: the 5-tap branch-free preprocess (resample_patch_p_kernel<14, 5>): bit-exactness
# tests, its timing per BASELINE geometry, and the headline bench's hbm_kernels line.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v14}
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_preprocess.py \
    tests/test_gpu_encoders.py > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/preprocess_bench.py > ${P}_preprocess_bench.log 2>&1 || exit $?
cat ${P}_preprocess_bench.log | grep -v "^{"
timeout -k 10 600 python -u bench.py --no-cpu-baseline > ${P}_bench.log 2>&1 || exit $?
tail -1 ${P}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['roofline']['hbm_kernels']['preprocess']))"
