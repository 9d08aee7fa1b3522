# Round 5, step 5: pipe10 on every non-split GEMM (form 95: bias, residual + statistics, LayerNorm fold)
# against the production dispatch (pipe10 only for activation fc1), A/B/A/B on the configs whose GEMMs are
# all 256-column multiples (LAION-CLIP-H, DFN5B-H bf16, OpenAI-CLIP-L); forms tested bit-identical first.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v5
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "form95" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for m in LAION-CLIP-H Apple-DFN5B-H OpenAI-CLIP-L; do
for i in 1 2; do
timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline --no-parity > ${P}_${m}_prod_$i.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline --no-parity --gemm-form 95 > ${P}_${m}_f95_$i.log 2>&1 || exit $?
done
done
for f in ${P}_*_*_[12].log; do echo "$f $(tail -1 $f | cut -c80-160)"; done
