set -o pipefail
timeout -k 10 120 tools/probes/mfma_rate > gpurun_out/r02_mfma_rate.log 2>&1
