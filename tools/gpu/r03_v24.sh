# Larger image execution batches: the full SigLIP job at caps 512 / 640 / 1024 images, and one
# rank's N = 8 share (625 images) at caps 512 (2 x 313) / 640 (1 x 625); interleaved, one box.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r03_v24
for rep in 1 2; do
  for ib in 512 640 1024; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --img-batch $ib > ${P}_5000_${ib}_${rep}.log 2>&1 || exit $?
    echo "5000 images cap $ib rep $rep: $(tail -1 ${P}_5000_${ib}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["encode_texts_s"], d["parity"]["recall_identical"])')"
  done
  for ib in 512 640; do
    timeout -k 10 300 python -u bench.py --n-images 625 --no-cpu-baseline --steps 3 --warmup 1 --img-batch $ib > ${P}_625_${ib}_${rep}.log 2>&1 || exit $?
    echo "625 images cap $ib rep $rep: $(tail -1 ${P}_625_${ib}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["encode_texts_s"], d["parity"]["recall_identical"])')"
  done
done
