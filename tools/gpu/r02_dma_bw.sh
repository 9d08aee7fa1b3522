set -o pipefail
timeout -k 10 120 tools/probes/dma_bw > gpurun_out/r02_dma_bw.log 2>&1
