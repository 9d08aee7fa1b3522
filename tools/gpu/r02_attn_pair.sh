set -o pipefail
export PYTHONUNBUFFERED=1
# kind 30 (60, production hd 72) vs 37 (67: 4-tile ring, one barrier per pair of key tiles)
timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --variants 60,67,60,67,60,67 > gpurun_out/r02_attn_pair.log 2>&1
