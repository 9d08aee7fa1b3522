set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "wave_epilogue" tests/test_gpu_mx.py > gpurun_out/r03_v15_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_v15_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_mx.py > gpurun_out/r03_v15_pytest_all.log 2>&1 || exit $?
tail -1 gpurun_out/r03_v15_pytest_all.log
timeout -k 10 300 python -u tools/gemm_bench.py --rows 186880 --shapes h_qkv,h_fc1,h_fc2 --variants=-1 --mx --mx-epi job --mx-variants=-1,10,-1,10 > gpurun_out/r03_v15_mx10_ab.log 2>&1 || exit $?
grep 'mx8' gpurun_out/r03_v15_mx10_ab.log
A="--model Apple-DFN5B-H --fp8 --no-cpu-baseline --no-parity --no-host-inputs"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $A > gpurun_out/r03_v15_fp8_base_$i.log 2>&1 || exit $?
  MME_MX_VARIANT=10 timeout -k 10 400 python -u bench.py $A > gpurun_out/r03_v15_fp8_mx10_$i.log 2>&1 || exit $?
done
for f in gpurun_out/r03_v15_fp8_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"], d["roofline"]["avg_launch_ms"])')"; done
