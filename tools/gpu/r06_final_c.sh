# Round-6 final measurement set, part C: after mx form 17 and layernorm_mx's packing (the fp8 path only; the
# bf16 kernels of parts A / B unchanged): both GPU suites and smoke again, the fp8 job's PMC traffic, its bench
# line and its kernel summary at this build (replacing part B's fp8 files).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r06_final}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
MME_DEV=1 timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_dev_pytest.log 2>&1
rc=$?; tail -2 ${P}_dev_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit $?
PMC_MODEL=Apple-DFN5B-H PMC_ARGS=--fp8 PMC_TAG=Apple-DFN5B-H-fp8 \
PMC_CONFIG='{"model": "Apple-DFN5B-H", "n_images": 5000, "img_batch": 512, "txt_batch": 4096, "fp8": true}' \
PMC_BUILD="${RUN:-r06_final}" bash tools/pmc_job.sh > ${P}_Apple-DFN5B-H-fp8_pmc.log 2>&1 || { tail -5 ${P}_Apple-DFN5B-H-fp8_pmc.log; exit 1; }
tail -6 ${P}_Apple-DFN5B-H-fp8_pmc.log
cp gpurun_out/hbm_traffic.json profiles/hbm_traffic.json
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_Apple-DFN5B-H_fp8_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --no-cpu-baseline > ${P}_Apple-DFN5B-H_bench.log 2>&1 || exit $?
for f in ${P}_Apple-DFN5B-H*bench.log; do echo "$f $(tail -1 $f | cut -c1-160)"; done
rm -rf gpurun_out/prof
PROF_TIMEOUT=500 PROF_ARGS="--model Apple-DFN5B-H --fp8" bash tools/profile_bench.sh > ${P}_DFN5B-fp8_prof.log 2>&1 || exit $?
S=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$S" ${P}_Apple-DFN5B-H-fp8_kernel_stats.csv
