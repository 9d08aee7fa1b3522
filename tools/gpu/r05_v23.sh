# Round 5, step 23: ColPali's GeGLU gate / up GEMM with its epilogue compiled (FOLD 2) against the run-time
# form (gemm form 93): bit-identity and the ColPali job A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v23
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_colpali.py -k "geglu or colpali" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 --no-cpu-baseline --no-parity > ${P}_colpali_prod_$i.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 --no-cpu-baseline --no-parity --gemm-form 93 > ${P}_colpali_f93_$i.log 2>&1 || exit $?
done
for f in ${P}_colpali_*_[12].log; do echo "$f $(tail -1 $f | cut -c80-150)"; done
