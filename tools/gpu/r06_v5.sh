# Round 6, step 5: attention kind 97 (kind 83 with the exp2 argument out of the QK^T MFMA): accuracy
# against fp64 beside kind 83, isolated timing at SigLIP's 417-image batch, SigLIP-400M job A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v5
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_kernels.py -k "mfma_bias or qs_entry or threshold_vs_exact or skip_vs_unskipped" > ${P}_pytest.log 2>&1 || exit 1
for r in 1 2 3; do
timeout -k 10 200 python -u tools/attn_bench.py --cases siglip_vision --batch 417 --variants 113,127 >> ${P}_attn.log 2>&1 || exit 1
done
for r in 1 2; do
timeout -k 10 400 python -u bench.py --no-cpu-baseline > ${P}_siglip_k98_$r.log 2>&1 || exit 1
MME_Q_PRESCALE=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline > ${P}_siglip_k83_$r.log 2>&1 || exit 1
done
grep -h -o '"value": [0-9.]*' ${P}_siglip_*.log
