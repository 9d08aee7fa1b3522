set -o pipefail
export PYTHONUNBUFFERED=1
# kind 27 (57, production hd 72) vs 30 (60, static priority) vs 33 (63, 16-B O stores) vs 34 (64, both)
timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --variants 57,60,63,64,57,60,63,64,57,60,63,64 > gpurun_out/r02_attn_wide.log 2>&1
