# Round 6, second session, v6: pipe9's LayerNorm-fold epilogue (QKV) takes the rows' statistics loaded under
# the main loop's last stage instead of at its start. GEMM tests, then A/B against HEAD's build
# (libmme_v6base.so): the LayerNorm-folded QKV / fc1 microbenchmark (checksums), SigLIP-400M and LAION-CLIP-H.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_s2_v6
timeout -k 10 400 python -u -m pytest -q -rs --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for L in libmme.so libmme_v6base.so libmme.so libmme_v6base.so; do
  MME_LIB=$PWD/multimodal-embedding_amd/mme/$L timeout -k 10 120 python -u tools/lnfold_bench.py 2>/dev/null | tail -1 >> ${P}_lnfold.log || exit $?
done
cat ${P}_lnfold.log
for M in SigLIP-400M LAION-CLIP-H; do
for L in libmme.so libmme_v6base.so libmme.so libmme_v6base.so libmme.so libmme_v6base.so; do
  echo "== $M $L" >> ${P}_jobs.log
  MME_LIB=$PWD/multimodal-embedding_amd/mme/$L timeout -k 10 300 python -u bench.py --model $M --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-host-inputs > ${P}_job.tmp 2>&1 || { tail -5 ${P}_job.tmp; exit 1; }
  tail -1 ${P}_job.tmp >> ${P}_jobs.log
  tail -1 ${P}_job.tmp | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$M $L', d['value'], r.get('achieved'), r.get('frac'))"
done
done
