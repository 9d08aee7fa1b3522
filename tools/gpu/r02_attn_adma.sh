set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --variants 47,57,58,47,57,58 > gpurun_out/r02_attn_adma.log 2>&1
