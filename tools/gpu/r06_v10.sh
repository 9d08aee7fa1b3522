# Round 6, step 10: layernorm_mx with the mx8 output packed by mx_pack8_fast (bit-exact: its outputs are
# bf16-rounded) against the same build with mx_pack8 (mme/libmme_ab_lnmx.so via MME_LIB): the bit-exactness
# tests, the kernel at the encoder geometries, and the DFN5B-H fp8 job on one box.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v10
OLD=multimodal-embedding_amd/mme/libmme_ab_lnmx.so
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_mx.py -k "layernorm_mx or quant_bit_exact" > ${P}_pytest.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 200 python -u tools/ln_bench.py >> ${P}_ln_new.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 200 python -u tools/ln_bench.py >> ${P}_ln_old.log 2>&1 || exit 1
done
for r in 1 2; do
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_fp8_new_$r.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_fp8_old_$r.log 2>&1 || exit 1
done
grep -h "mx8" ${P}_ln_new.log ${P}_ln_old.log
grep -H -o '"value": [0-9.]*' ${P}_fp8_*.log
