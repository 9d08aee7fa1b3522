set -o pipefail
export PYTHONUNBUFFERED=1
# hd 80: kind 21 (51) vs 21 + priority (65) on ViT-H; kind 23 (53) vs 23 + priority (66) on DFN5B
timeout -k 10 300 python -u tools/attn_bench.py --cases vitH_vision --variants 51,65,51,65,51,65 > gpurun_out/r02_attn_prio80.log 2>&1 && \
timeout -k 10 300 python -u tools/attn_bench.py --cases dfn5b_vision --variants 53,66,53,66,53,66 >> gpurun_out/r02_attn_prio80.log 2>&1
