# One-rank RCCL exchange test on the GPU; one rank's share of the N = 8 job (625 images + 3 125
# captions) on one GPU at the round-3 execution batches.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r03_v23
timeout -k 10 300 python -u -m pytest -q -rs -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rccl.py > ${P}_pytest.log 2>&1
rc=$?; tail -3 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --n-images 625 --no-cpu-baseline --steps 3 --warmup 1 > ${P}_625_${rep}.log 2>&1 || exit $?
  echo "625 images rep $rep: $(tail -1 ${P}_625_${rep}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["encode_texts_s"], d["parity"]["recall_identical"])')"
done
