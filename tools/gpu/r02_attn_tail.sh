set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --variants 57,59,57,59 > gpurun_out/r02_attn_tail.log 2>&1
