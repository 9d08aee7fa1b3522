# Execution-batch sweep of the headline job (img / txt batch sizes are internal choices; the
# reference's own batch of 32 only shapes its host-side loop).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--no-cpu-baseline --no-parity --no-host-inputs"
for cfg in "256 2048" "384 2048" "512 2048" "256 4096" "512 4096" "256 2048"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py $A --img-batch $1 --txt-batch $2 > gpurun_out/r03_v20_b$1_t$2.log 2>&1 || exit $?
  echo "img $1 txt $2: $(tail -1 gpurun_out/r03_v20_b$1_t$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["encode_texts_s"], d["roofline"]["achieved"])')"
done
