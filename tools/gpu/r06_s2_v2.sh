# Round 6, second session, v2: the GEMM epilogue's bias loaded ahead of the residual rows (FOLD 2 / 3, 8-B
# groups; gemm_epilogue_wave). GPU GEMM tests (bit-identity between forms included), then A/B against the
# v1 build (libmme_v1.so: the same sources with HEAD's gemm.hip): o_proj / fc2 / QKV microbenchmarks with the
# residual, residual + statistics and bias epilogues, then the SigLIP-400M and LAION-CLIP-H jobs, alternating.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r06_s2_v2}
# v2's first run: every selected test green but the fp8 whole-job drift (84 decided I2T rows < 100; the gate
# now counts the decided rows of T2I, I2T and I2T_Sym, mme.mx.job_drift): that test alone, reported
timeout -k 10 400 python -u -m pytest -q -rs -s --timeout 380 --timeout-method thread -m gpu tests/test_gpu_mx.py -k "whole_job_drift or full_size_vs_oracle" > ${P}_drift.log 2>&1
tail -2 ${P}_drift.log; grep -E "fp8 vs bf16|drift" ${P}_drift.log | head -5
for L in libmme.so libmme_v1.so libmme.so libmme_v1.so; do
  for E in res resstats bias; do
    echo "== $L $E" >> ${P}_gemm.log
    MME_LIB=$PWD/multimodal-embedding_amd/mme/$L timeout -k 10 120 python -u tools/gemm_bench.py --rows 303993 --shapes o_proj,fc2,qkv --epi $E >> ${P}_gemm.log 2>&1 || exit $?
  done
done
grep -v "^$\|amdgpu.ids" ${P}_gemm.log | tail -40
for M in SigLIP-400M LAION-CLIP-H; do
for L in libmme.so libmme_v1.so libmme.so libmme_v1.so; do
  echo "== $M $L" >> ${P}_jobs.log
  MME_LIB=$PWD/multimodal-embedding_amd/mme/$L timeout -k 10 300 python -u bench.py --model $M --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-host-inputs > ${P}_job.tmp 2>&1 || { tail -5 ${P}_job.tmp; exit 1; }
  tail -1 ${P}_job.tmp >> ${P}_jobs.log
  tail -1 ${P}_job.tmp | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$M $L', d['value'], r.get('achieved'), r.get('frac'))"
done
done
