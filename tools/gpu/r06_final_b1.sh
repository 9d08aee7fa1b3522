# Round-6 final measurement set, part B1 (RUN=r06_final2; part B split in two calls): the PMC passes and the
# bf16 / fp8 bench lines of part B below.
# every other BASELINE config on one GPU (fp8 with its whole-job drift,
# gated on decided rows), LAION-CLIP-H's and the fp8 job's PMC traffic at this build (mx11 included),
# the kernel summaries of those two jobs, and the same-device rank rehearsals (2 ranks; 3 uneven shards).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r06_final}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
PMC_MODEL=LAION-CLIP-H PMC_CONFIG='{"model": "LAION-CLIP-H", "n_images": 5000, "img_batch": 512, "txt_batch": 4096, "fp8": false}' \
PMC_BUILD="${RUN:-r06_final}" bash tools/pmc_job.sh > ${P}_LAION-CLIP-H_pmc.log 2>&1 || { tail -5 ${P}_LAION-CLIP-H_pmc.log; exit 1; }
tail -6 ${P}_LAION-CLIP-H_pmc.log
PMC_MODEL=Apple-DFN5B-H PMC_ARGS=--fp8 PMC_TAG=Apple-DFN5B-H-fp8 \
PMC_CONFIG='{"model": "Apple-DFN5B-H", "n_images": 5000, "img_batch": 512, "txt_batch": 4096, "fp8": true}' \
PMC_BUILD="${RUN:-r06_final}" bash tools/pmc_job.sh > ${P}_Apple-DFN5B-H-fp8_pmc.log 2>&1 || { tail -5 ${P}_Apple-DFN5B-H-fp8_pmc.log; exit 1; }
tail -6 ${P}_Apple-DFN5B-H-fp8_pmc.log
cp gpurun_out/hbm_traffic.json profiles/hbm_traffic.json
for m in OpenAI-CLIP-L LAION-CLIP-H Apple-DFN5B-H; do
  timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline > ${P}_${m}_bench.log 2>&1 || exit $?
done
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_Apple-DFN5B-H_fp8_bench.log 2>&1 || exit $?
for f in ${P}_*bench.log; do echo "$f $(tail -1 $f | cut -c1-160)"; done
