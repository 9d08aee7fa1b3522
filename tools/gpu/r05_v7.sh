# Round 5, step 7: is the 9-wave ViT-H block (3 + 2 + 2 + 2 waves over the SIMDs) imbalance-bound?
# T 257 vs T 256 under kinds 86 (9-wave), 87 (8-wave), 94 (persistent 9-wave).
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P=gpurun_out/r05_v7
for i in 1 2; do
timeout -k 10 200 python -u tools/attn_bench.py --cases vitH_vision,vitH_256 --batch 512 --variants 116,117,124 >> ${P}_attn.log 2>&1 || exit 1
done
grep -v amdgpu.ids ${P}_attn.log
