# Round 5, step 3: branch-free erfc GELU (+ pipe10 for gelu_erf fc1) and half-wave LayerNorm rows: GEMM /
# mx tests, LayerNorm timing and the LAION-CLIP-H job, A/B against round 4's library (libm erff, pipe9,
# whole-wave LayerNorm rows), alternating.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v3
OLD=multimodal-embedding_amd/build_exp/libmme_old.so
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_mx.py -k "activation_vs_float64 or dispatched_fc1 or bias_act or lnfold or layernorm or mx_quant" > ${P}_pytest.log 2>&1
rc=$?; tail -3 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
MME_LIB=$OLD timeout -k 10 120 python -u tools/ln_bench.py >> ${P}_ln_old.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/ln_bench.py >> ${P}_ln_new.log 2>&1 || exit 1
done
for i in 1 2; do
MME_LIB=$OLD timeout -k 10 600 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > ${P}_laion_old_$i.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > ${P}_laion_new_$i.log 2>&1 || exit $?
done
for f in ${P}_laion_*.log; do echo "$f $(tail -1 $f | cut -c1-120)"; done
