# bench.py default caption batches per family: SigLIP 8192 (5 x 5000), LAION-CLIP-H 4096 (7 x 3572).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r03_v30
for m in SigLIP-400M LAION-CLIP-H; do
  timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --steps 2 --warmup 1 > ${P}_${m}.log 2>&1 || exit $?
  echo "$m: $(tail -1 ${P}_${m}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["txt_batch"], d["encode_texts_s"], d["parity"]["recall_identical"], d["parity"]["encoders"]["ok"])')"
done
