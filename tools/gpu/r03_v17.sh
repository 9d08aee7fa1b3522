# N-rank rehearsals of the two 8-GPU BASELINE configs on one device (gloo, --same-device: everything
# but the RCCL transport), and the kernel summary of the fp8 job with the round-3 mx10 GEMM.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --model LAION-CLIP-H --gpus 2 --backend gloo --same-device --n-images 1000 --no-cpu-baseline > gpurun_out/r03_v17_laion_multirank2.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --gpus 2 --backend gloo --same-device --n-images 1000 --no-cpu-baseline > gpurun_out/r03_v17_dfn5b_fp8_multirank2.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --n-images 1000 --no-cpu-baseline > gpurun_out/r03_v17_dfn5b_fp8_1000.log 2>&1 || exit $?
PROF_TIMEOUT=500 PROF_ARGS="--model Apple-DFN5B-H --fp8" bash tools/profile_bench.sh > gpurun_out/r03_v17_prof.log 2>&1 || exit $?
for f in gpurun_out/r03_v17_*multirank2.log gpurun_out/r03_v17_dfn5b_fp8_1000.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["n_gpus"], d["recall"], (d.get("parity") or {}).get("recall_identical"))')"; done
