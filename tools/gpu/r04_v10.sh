# Round 4 step 10: pipe10 (persistent pipe9, the next tile's prologue under the epilogue) against
# production pipe9: bit-identity on small / ragged shapes, then A/B at the SigLIP job's batch.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v10}
export MME_DEV=1
for R in 300 1000 5000 70001; do
  timeout -k 10 120 python -u tools/pers_ab.py --a -1 --b 90 --rows $R --check-only --cases fc1,h_fc1,bias_gelu,qkv \
      >> ${P}_pipe10_check.log 2>&1 || { tail -5 ${P}_pipe10_check.log; exit 1; }
done
grep -h bit_identical ${P}_pipe10_check.log | cut -c1-80
timeout -k 10 300 python -u tools/pers_ab.py --a -1 --b 90 --rows 303993 --rounds 5 --iters 5 --cases fc1,h_fc1,bias_gelu \
    > ${P}_pipe10_ab.log 2>&1 || exit $?
grep -v "^{" ${P}_pipe10_ab.log
