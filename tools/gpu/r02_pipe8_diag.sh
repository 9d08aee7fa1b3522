set -o pipefail
export PYTHONUNBUFFERED=1
# pipe8 (-1) and its diagnostic builds: 65 no epilogue, 66 no loop DMA, 67 no MFMA; pipe6: 39 no epilogue, 33 no DMA, 34 no MFMA
timeout -k 10 300 python -u tools/gemm_bench.py --epi bias --shapes fc1,fc2 --variants=-1,65,66,67,39,33,34 > gpurun_out/r02_pipe8_diag.log 2>&1 && \
timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --variants 57,62,60,57,62,60 >> gpurun_out/r02_pipe8_diag.log 2>&1
