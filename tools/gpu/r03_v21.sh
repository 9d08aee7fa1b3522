# Last-layer pruning to the pooled rows (models.PRUNE_LAST): encoder / fp8 / config0 parity,
# then a job A/B (MME_PRUNE_LAST=1 vs 0) on SigLIP-400M and OpenAI-CLIP-L.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r03_v21
timeout -k 10 600 python -u -m pytest -q -rs -s --maxfail=3 --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_encoders.py tests/test_gpu_config0.py tests/test_gpu_mx.py > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
grep -E "pruned vs full|bit-identical to the" ${P}_pytest.log
for m in SigLIP-400M OpenAI-CLIP-L; do
  for pr in 1 0 1; do
    MME_PRUNE_LAST=$pr timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --steps 3 --warmup 1 > ${P}_${m}_p${pr}.log 2>&1 || exit $?
    echo "$m prune=$pr $(tail -1 ${P}_${m}_p${pr}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("parity"))')"
  done
done
