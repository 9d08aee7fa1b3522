# SigLIP MAP head with the probe absorbed (mme_map_pool): kernel + encoder parity, then a job
# A/B (MME_MAP_ABSORB=1 / 0 / 1) and a kernel-stats profile of the absorbed job.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r03_v26
timeout -k 10 600 python -u -m pytest -q -rs -s --maxfail=3 --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py::test_map_pool tests/test_gpu_kernels.py::test_probe_attention tests/test_gpu_encoders.py tests/test_gpu_config0.py tests/test_gpu_edge.py > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
grep -E "MAP head absorbed|bit-identical to the|pruned vs full" ${P}_pytest.log
for ab in 1 0 1 0; do
  MME_MAP_ABSORB=$ab timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > ${P}_ab${ab}.log 2>&1 || exit $?
  echo "absorb=$ab $(tail -1 ${P}_ab${ab}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["encode_images_s"], d["parity"]["recall_identical"], d["parity"]["encoders"]["img_cos_min"], d["parity"]["encoders"]["ok"])')"
done
