# Caption execution-batch cap 4096 vs 8192 on the CLIP configs, interleaved on one box.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r03_v29
for rep in 1 2; do
  for m in OpenAI-CLIP-L LAION-CLIP-H; do
    for tb in 4096 8192; do
      timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --steps 2 --warmup 1 --txt-batch $tb > ${P}_${m}_${tb}_${rep}.log 2>&1 || exit $?
      echo "$m txt cap $tb rep $rep: $(tail -1 ${P}_${m}_${tb}_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["encode_texts_s"], d["parity"]["recall_identical"])')"
    done
  done
done
