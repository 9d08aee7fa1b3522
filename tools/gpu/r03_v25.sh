# Image execution-batch cap 512 vs 640 on the other configs (full job), and DFN5B-H's N = 8 share
# (625 images: 5 x 125 at cap 512, 1 x 625 at 640); interleaved, one box.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r03_v25
for rep in 1 2; do
  for m in OpenAI-CLIP-L LAION-CLIP-H Apple-DFN5B-H; do
    for ib in 512 640; do
      timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --steps 2 --warmup 1 --img-batch $ib > ${P}_${m}_${ib}_${rep}.log 2>&1 || exit $?
      echo "$m 5000 cap $ib rep $rep: $(tail -1 ${P}_${m}_${ib}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["encode_texts_s"], d["parity"]["recall_identical"])')"
    done
  done
  for ib in 512 640; do
    timeout -k 10 300 python -u bench.py --model Apple-DFN5B-H --n-images 625 --no-cpu-baseline --steps 3 --warmup 1 --img-batch $ib > ${P}_dfn625_${ib}_${rep}.log 2>&1 || exit $?
    echo "DFN5B 625 cap $ib rep $rep: $(tail -1 ${P}_dfn625_${ib}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["encode_texts_s"], d["parity"]["recall_identical"])')"
  done
done
