set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03_v12_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r03_v12_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
A="--no-cpu-baseline --no-parity --no-host-inputs"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $A > gpurun_out/r03_v12_timer_on_$i.log 2>&1 || exit $?
  timeout -k 10 400 python -u bench.py $A --no-kernel-timer > gpurun_out/r03_v12_timer_off_$i.log 2>&1 || exit $?
done
for f in gpurun_out/r03_v12_timer_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --epi bias --variants=-1,81,82,83,-1,81,82,83 > gpurun_out/r03_v12_gemm_prio_bias.log 2>&1 || exit $?
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --epi gelu --shapes fc1 --variants=-1,81,82,83,-1,81,82,83 > gpurun_out/r03_v12_gemm_prio_gelu.log 2>&1 || exit $?
tail -1 gpurun_out/r03_v12_gemm_prio_bias.log; tail -1 gpurun_out/r03_v12_gemm_prio_gelu.log
timeout -k 10 600 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > gpurun_out/r03_v12_laion_bench.log 2>&1 && \
SHAPES=fc1 timeout -k 10 500 bash tools/pmc_gemm_util.sh > gpurun_out/r03_v12_pmc_gemm_util.log 2>&1 && \
PMC_TIMEOUT=400 timeout -k 10 900 bash tools/pmc_gemm.sh > gpurun_out/r03_v12_pmc_traffic.log 2>&1
rc2=$?
tail -1 gpurun_out/r03_v12_laion_bench.log | cut -c1-300; tail -30 gpurun_out/r03_v12_pmc_gemm_util.log; tail -12 gpurun_out/r03_v12_pmc_traffic.log
exit $rc2
