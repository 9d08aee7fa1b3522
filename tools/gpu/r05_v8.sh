# Round 5, step 8: 8-wave persistent ViT-H blocks (dev kind 95: one per CU, 2 waves per SIMD) against
# kind 87 (8-wave, two blocks per CU) at T 256, and kind 94 at T 257.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P=gpurun_out/r05_v8
for i in 1 2; do
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --cases vitH_256 --batch 512 --variants 117,124,125 >> ${P}_attn.log 2>&1 || exit 1
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --cases vitH_vision --batch 512 --variants 124 >> ${P}_attn.log 2>&1 || exit 1
done
grep -v amdgpu.ids ${P}_attn.log
