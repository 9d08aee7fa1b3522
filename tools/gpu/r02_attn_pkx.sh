set -o pipefail
export PYTHONUNBUFFERED=1
# kind 27 (production hd 72) vs 29 (packed exp-argument FMAs) vs 30 (static priority) vs 31 (both)
timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --variants 57,59,60,61,57,59,60,61,57,59 > gpurun_out/r02_attn_pkx.log 2>&1
