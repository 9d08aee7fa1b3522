set -o pipefail
export PYTHONUNBUFFERED=1
# pipe8 row-band height: 70 = 4 (production, no split), 68 = 2, 69 = 8; fc1 (N % 256 == 0) and the text-tower rows
timeout -k 10 300 python -u tools/gemm_bench.py --epi bias --shapes fc1,h_fc1 --variants=70,68,69,70,68,69 > gpurun_out/r02_pipe8_group.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_bench.py --rows 100032 --epi bias --shapes fc1,qkv,fc2 --variants=-1,70,68,69 >> gpurun_out/r02_pipe8_group.log 2>&1
