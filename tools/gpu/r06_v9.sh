# Round 6, step 9: the fp8 fc1 epilogue. (a) Where its cost goes (DFN5B-H fc1 at the job's 500-image batch:
# M 365 000, N 5 120, K 1 280): mx11 with bias only, + quick_gelu (bf16 out), bias to an mx8 output, the job's
# bias + quick_gelu to mx8; (b) mx form 17 (the mx8 output packed without the inactive clamp) against form 16:
# bit-identity tests, fc1 timing, the DFN5B-H fp8 job A/B on one box.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v9
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_mx.py -k "mx12_bit_identical or residual_and_mx_output or vs_dequantised" > ${P}_pytest.log 2>&1 || exit 1
for e in bias quick mx8 job; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 365000 --shapes h_fc1 --mx --mx-epi $e --mx-variants 16,17 --iters 5 >> ${P}_mx_epi.log 2>&1 || exit 1
done
for r in 1 2; do
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > ${P}_fp8_f17_$r.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline --mx-form 16 > ${P}_fp8_f16_$r.log 2>&1 || exit 1
done
grep -h "mx8 v" ${P}_mx_epi.log
grep -H -o '"value": [0-9.]*' ${P}_fp8_*.log
