# Execution-batch caps per model: 256 / 2048 (round 2) vs 512 / 4096 (round 3 default) on the
# ViT-H configs and CLIP-L, interleaved A/B/A/B on one box.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r03_v22
for m in LAION-CLIP-H Apple-DFN5B-H OpenAI-CLIP-L; do
  for rep in 1 2; do
    for bb in "256 2048" "512 4096"; do
      set -- $bb
      timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --steps 2 --warmup 1 --img-batch $1 --txt-batch $2 > ${P}_${m}_${1}_${2}_${rep}.log 2>&1 || exit $?
      echo "$m img $1 txt $2 rep $rep: $(tail -1 ${P}_${m}_${1}_${2}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["encode_texts_s"], d["config"]["img_batch"])')"
    done
  done
done
