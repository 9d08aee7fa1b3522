# Round 6, step 8: Q pre-scaled at hd 80 too (kinds 100 / 101 in production through mme_attention_qs;
# DFN5B fp8 with the factor in its mx8 Q rows): the GPU suite, then job A/B against MME_Q_PRESCALE=0 on one
# box (LAION-CLIP-H: ViT-H kind 101 vs 86; Apple-DFN5B-H bf16 and fp8: kind 100 vs 87).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v8
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for m in LAION-CLIP-H Apple-DFN5B-H; do
timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline > ${P}_${m}_qs_$r.log 2>&1 || exit 1
MME_Q_PRESCALE=0 timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline > ${P}_${m}_plain_$r.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_fp8_qs_$r.log 2>&1 || exit 1
MME_Q_PRESCALE=0 timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_fp8_plain_$r.log 2>&1 || exit 1
done
grep -H -o '"value": [0-9.]*' ${P}_*.log
