# Round 5, step 6: kind 94 (persistent ViT-H attention) bit-identity against kind 86 and microbench A/B
# at the job's execution batch; form 95 (pipe10 on every non-split GEMM) bit-identity and job A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v6
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "form95 or persistent_vith" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
timeout -k 10 200 python -u tools/attn_bench.py --cases vitH_vision --batch 512 --variants 116,124 >> ${P}_attn.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/attn_bench.py --cases vitH_vision --batch 64 --variants 116,124 >> ${P}_attn.log 2>&1 || exit 1
done
cat ${P}_attn.log
for m in LAION-CLIP-H Apple-DFN5B-H OpenAI-CLIP-L; do
for i in 1 2; do
timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline --no-parity > ${P}_${m}_prod_$i.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline --no-parity --gemm-form 95 > ${P}_${m}_f95_$i.log 2>&1 || exit $?
done
done
for f in ${P}_*_*_[12].log; do echo "$f $(tail -1 $f | cut -c80-160)"; done
