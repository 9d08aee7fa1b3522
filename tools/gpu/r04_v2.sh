# Round 4 step 2: GPU suite at HEAD (ABI 8: exact-tie ranking, per-call kernel forms, conflict-free
# epilogue staging), smoke, and the epilogue-staging A/B (dev forms 84 / mx 4 = the round-3 layout).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v2}
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit $?
R=303993  # one SigLIP vision execution batch: 417 images x 729 tokens
for E in res gelu bias; do
  MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --rows $R --variants=-1,84,-1,84 --epi $E \
      --shapes qkv,o_proj,fc1,fc2 > ${P}_gemm_epi_swz_${E}.log 2>&1 || exit $?
done
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --rows $R --variants=-1,84,-1,84 --epi resstats \
    --shapes o_proj,fc2 > ${P}_gemm_epi_swz_resstats.log 2>&1 || exit $?
MME_DEV=1 timeout -k 10 300 python -u tools/gemm_bench.py --rows $((417*730)) --variants=-1 --epi none --mx \
    --mx-variants=-1,4,-1,4 --mx-epi job --shapes h_qkv,h_fc1,h_fc2 > ${P}_mx_epi_swz.log 2>&1 || exit $?
grep -h "TFLOP" ${P}_gemm_epi_swz_*.log ${P}_mx_epi_swz.log | cut -c1-110
