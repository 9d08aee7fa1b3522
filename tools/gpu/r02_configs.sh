set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --model OpenAI-CLIP-L --no-cpu-baseline > gpurun_out/r02_v2_clip_l_bench.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline > gpurun_out/r02_v2_laion_clip_h_bench.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model Apple-DFN5B-H --no-cpu-baseline > gpurun_out/r02_v2_dfn5b_bf16_bench.log 2>&1 && \
timeout -k 10 500 python -u bench.py --model Apple-DFN5B-H --fp8 --no-cpu-baseline > gpurun_out/r02_v2_dfn5b_fp8_bench.log 2>&1 && \
timeout -k 10 600 python -u bench.py --model ColPali-v1.3 --no-cpu-baseline > gpurun_out/r02_v2_colpali_bench.log 2>&1
