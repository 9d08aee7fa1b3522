set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_attn
CASES=siglip_vision VARIANTS=0,68 bash tools/pmc_attn.sh > gpurun_out/r02_pmc_attn_m32.log 2>&1
