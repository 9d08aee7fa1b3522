# Round 6, step 4: SigLIP's split grid (N = 256 k + 128: o_proj / fc2 / QKV) with its 512 x 128 tiles on
# pipe4_tile (64-deep stages of whole-line DMA pieces) against round 5's pipe6_tile (mme/libmme_ab_split.so,
# the HEAD build before the change, via MME_LIB): bit-identity tests, the split shapes, the SigLIP-400M job.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v4
OLD=multimodal-embedding_amd/mme/libmme_ab_split.so
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_kernels.py -k "form95 or res_stats or pipe8_bit" > ${P}_pytest.log 2>&1 || exit 1
for r in 1 2; do
for s in 1024:1152 1152:1152 1024:4352 1152:4352; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 303993 --shapes $s --epi resstats --variants=-1 >> ${P}_split_new.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 200 python -u tools/gemm_bench.py --rows 303993 --shapes $s --epi resstats --variants=-1 >> ${P}_split_old.log 2>&1 || exit 1
done
for s in 3328:1152 3456:1152; do
timeout -k 10 200 python -u tools/gemm_bench.py --rows 303993 --shapes $s --epi bias --variants=-1 >> ${P}_split_new.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 200 python -u tools/gemm_bench.py --rows 303993 --shapes $s --epi bias --variants=-1 >> ${P}_split_old.log 2>&1 || exit 1
done
done
for r in 1 2; do
timeout -k 10 400 python -u bench.py --no-cpu-baseline > ${P}_siglip_new_$r.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 400 python -u bench.py --no-cpu-baseline > ${P}_siglip_old_$r.log 2>&1 || exit 1
done
grep TFLOP ${P}_split_new.log ${P}_split_old.log
grep -h -o '"value": [0-9.]*' ${P}_siglip_*.log
