set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
# N-rank path rehearsed on one GPU (gloo, every rank on cuda:0) with the round-2 kernels,
# SigLIP (hd 72) and DFN5B (hd 80: the 32x32x16 attention) at 1 000 images
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --same-device --steps 1 --warmup 1 --n-images 1000 --no-cpu-baseline > gpurun_out/r02_s2_multirank.log 2>&1 && \
timeout -k 10 400 python -u bench.py --gpus 4 --backend gloo --same-device --steps 1 --warmup 1 --n-images 1000 --no-cpu-baseline >> gpurun_out/r02_s2_multirank.log 2>&1 && \
timeout -k 10 400 python -u bench.py --gpus 1 --steps 1 --warmup 1 --n-images 1000 --no-cpu-baseline >> gpurun_out/r02_s2_multirank.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model Apple-DFN5B-H --gpus 2 --backend gloo --same-device --steps 1 --warmup 1 --n-images 1000 --no-cpu-baseline >> gpurun_out/r02_s2_multirank.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model Apple-DFN5B-H --gpus 1 --steps 1 --warmup 1 --n-images 1000 --no-cpu-baseline >> gpurun_out/r02_s2_multirank.log 2>&1
