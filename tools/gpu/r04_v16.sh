# Round 4 step 16: hd-72 attention on a three-slot K / V ring with the DMA from inline asm (dev kind 78:
# no hipcc vmcnt(0) before the V^T reads, tile t + 2's DMA in flight) against production kind 62, at the
# SigLIP job's execution batch; bit identity printed by attn_bench ("identical").
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v16}
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision,dfn5b_vision --batch 417 \
    --variants 0,108,0,108,0,108 > ${P}_ring3_bench.log 2>&1 || { cat ${P}_ring3_bench.log; exit 1; }
cat ${P}_ring3_bench.log
