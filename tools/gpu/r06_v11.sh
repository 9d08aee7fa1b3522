# Round 6, step 11: attention waves whose queries all lie past T (the eighth wave of the last query block at
# T 729 / 730) and causal waves before a tile's first key skip that tile's arithmetic (kinds 98 / 100 / 101
# and attn_fwd_kernel, kind 89): bit-identity against the same build without the skip (MME_LIB), the kernels
# alone, and the SigLIP-400M / LAION-CLIP-H / OpenAI-CLIP-L / DFN5B-H jobs on one box.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r06_v11
OLD=multimodal-embedding_amd/mme/libmme_ab_noskip.so
timeout -k 10 300 python -u tools/attn_identity.py > ${P}_id_new.txt 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 300 python -u tools/attn_identity.py > ${P}_id_old.txt 2>&1 || exit 1
diff <(grep ^B ${P}_id_new.txt) <(grep ^B ${P}_id_old.txt) > ${P}_id_diff.txt && echo "attention outputs bit-identical" || { echo "DIFFER"; cat ${P}_id_diff.txt; }
for r in 1 2; do
timeout -k 10 200 python -u tools/attn_bench.py --qs --cases siglip_vision,dfn5b_vision,clip_text_causal --batch 417 >> ${P}_attn_new.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 200 python -u tools/attn_bench.py --qs --cases siglip_vision,dfn5b_vision,clip_text_causal --batch 417 >> ${P}_attn_old.log 2>&1 || exit 1
done
for r in 1 2; do
for m in SigLIP-400M LAION-CLIP-H OpenAI-CLIP-L Apple-DFN5B-H; do
timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline > ${P}_${m}_new_$r.log 2>&1 || exit 1
MME_LIB=$OLD timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline > ${P}_${m}_old_$r.log 2>&1 || exit 1
done
done
grep -h "TFLOP" ${P}_attn_new.log ${P}_attn_old.log
grep -H -o '"value": [0-9.]*' ${P}_*_[12].log
