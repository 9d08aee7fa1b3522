set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 --no-cpu-baseline > gpurun_out/r02_s2g_colpali_bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model OpenAI-CLIP-L --no-cpu-baseline > gpurun_out/r02_s2g_clip_l_bench.log 2>&1
