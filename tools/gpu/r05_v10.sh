# Round 5, step 10: kind 86 vs 94 in isolation at the LAION job's batches (455, 450) and 512.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
P=gpurun_out/r05_v10
for i in 1 2; do
for b in 455 450 512; do
timeout -k 10 200 python -u tools/attn_bench.py --cases vitH_vision --batch $b --variants 116,124 >> ${P}_attn.log 2>&1 || exit 1
done
done
grep -v amdgpu.ids ${P}_attn.log
