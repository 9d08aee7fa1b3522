# Round 4 step 13: PMC HBM traffic of the DFN5B-H fp8 job (configs[4]) at its bench geometry, so the
# --fp8 bench line carries the mx GEMM's traffic too; then that bench line.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v13}
cp profiles/hbm_traffic.json gpurun_out/hbm_traffic.json
PMC_MODEL=Apple-DFN5B-H PMC_ARGS="--fp8" PMC_TAG=dfn5b_fp8 \
PMC_CONFIG='{"model": "Apple-DFN5B-H", "n_images": 5000, "img_batch": 512, "txt_batch": 4096, "fp8": true}' \
PMC_BUILD="${RUN:-r04_v13}" bash tools/pmc_job.sh > ${P}_pmc.log 2>&1 || { tail -5 ${P}_pmc.log; exit 1; }
grep -A4 '"gemm_mx"' ${P}_pmc.log | head -6
cp gpurun_out/hbm_traffic.json profiles/hbm_traffic.json
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_dfn5b_fp8_bench.log 2>&1 || exit $?
tail -1 ${P}_dfn5b_fp8_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['achieved'], r['frac'], r.get('traffic'), r.get('traffic_note'))"
