set -o pipefail
export PYTHONUNBUFFERED=1
# N = 2 and 4 ranks on the one GPU of this box: bench.py's own launcher, gloo process group,
# every rank on cuda:0 (the RCCL path needs one GPU per rank; this rehearses everything else)
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --same-device --steps 1 --warmup 1 --n-images 1000 --no-cpu-baseline > gpurun_out/r02_multirank.log 2>&1 && \
timeout -k 10 400 python -u bench.py --gpus 4 --backend gloo --same-device --steps 1 --warmup 1 --n-images 1000 --no-cpu-baseline >> gpurun_out/r02_multirank.log 2>&1 && \
timeout -k 10 400 python -u bench.py --gpus 1 --steps 1 --warmup 1 --n-images 1000 --no-cpu-baseline >> gpurun_out/r02_multirank.log 2>&1
