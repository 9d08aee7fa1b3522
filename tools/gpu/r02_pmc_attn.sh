set -o pipefail; bash tools/pmc_attn.sh > gpurun_out/r02_pmc_attn.log 2>&1
