# Round 4 step 23 (= step 8 at the rescale-threshold build): rocprof kernel-trace summaries of the LAION-CLIP-H job (BASELINE configs[2]) and of
# the DFN5B-H fp8 job (configs[4]) at HEAD (verdict item 2), each beside its bench line.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v23}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
for M in LAION-CLIP-H Apple-DFN5B-H-fp8; do
  A="--model ${M%-fp8}"; [ "$M" != "${M%-fp8}" ] && A="$A --fp8"
  rm -rf gpurun_out/prof
  PROF_ARGS="$A --no-parity" PROF_TIMEOUT=500 bash tools/profile_bench.sh > ${P}_${M}_prof.log 2>&1 || exit $?
  S=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
  cp "$S" ${P}_${M}_kernel_stats.csv
  cp gpurun_out/prof/bench_stdout.log ${P}_${M}_prof_bench.log
  python3 - "$S" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print(f"{float(r['TotalDurationNs'])/tot*100:6.2f}% {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f}us {r['Name'][:90]}")
PY
done
