set -o pipefail
timeout -k 10 120 tools/probes/store_bw > gpurun_out/r02_storebw.log 2>&1
