# Round 6, second session, v7: the CLIP text attention (kind 102) accounted as its own HBM-bound family
# (`attention_short2`, bench.py HBM_FAMILIES; tools/pmc_summary.py): LAION-CLIP-H's PMC traffic and bench line
# with it, and the default headline bench once more (bench.py changed; kernels unchanged).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_final2
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
PMC_MODEL=LAION-CLIP-H PMC_CONFIG='{"model": "LAION-CLIP-H", "n_images": 5000, "img_batch": 512, "txt_batch": 4096, "fp8": false}' \
PMC_BUILD=r06_final2 bash tools/pmc_job.sh > ${P}_LAION-CLIP-H_pmc.log 2>&1 || { tail -5 ${P}_LAION-CLIP-H_pmc.log; exit 1; }
cp gpurun_out/hbm_traffic.json profiles/hbm_traffic.json
timeout -k 10 600 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > ${P}_LAION-CLIP-H_bench.log 2>&1 || exit $?
tail -1 ${P}_LAION-CLIP-H_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['roofline']['hbm_kernels'].get('attention_short2')))"
timeout -k 10 600 python -u bench.py > gpurun_out/r06_s2_v7_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06_s2_v7_bench.log | cut -c1-200
