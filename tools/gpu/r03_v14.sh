set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mx.py > gpurun_out/r03_v14_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r03_v14_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --rows 186880 --shapes h_qkv,h_fc1,h_fc2 --variants=-1 --mx --mx-epi job --mx-variants=-1,2,3,-1,2,3 > gpurun_out/r03_v14_mx_wepi_ab.log 2>&1 || exit $?
grep 'mx8' gpurun_out/r03_v14_mx_wepi_ab.log
A="--model Apple-DFN5B-H --fp8 --no-cpu-baseline --no-parity --no-host-inputs"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $A > gpurun_out/r03_v14_fp8_base_$i.log 2>&1 || exit $?
  MME_MX_VARIANT=2 timeout -k 10 400 python -u bench.py $A > gpurun_out/r03_v14_fp8_wepi_$i.log 2>&1 || exit $?
  MME_MX_VARIANT=3 timeout -k 10 400 python -u bench.py $A > gpurun_out/r03_v14_fp8_wepisc1_$i.log 2>&1 || exit $?
done
for f in gpurun_out/r03_v14_fp8_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"], d["roofline"]["avg_launch_ms"])')"; done
