# Dev kind 66 (attn_short_pf_kernel: persistent, next pair's loads in flight) vs the production
# short kernel (kind 16) on the SigLIP text shapes: time and max difference (0 = bit-identical).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  MME_DEV=1 timeout -k 10 200 python -u tools/attn_bench.py --variants 0,96,0,96 --cases siglip_text,siglip_text_pad,siglip_text_2500 || exit $?
done
