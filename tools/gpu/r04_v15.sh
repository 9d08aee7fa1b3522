# Round 4 step 15: SQ counters of the production hd-72 attention (kind 62) at the SigLIP job's execution
# batch (417 images x 16 heads, T 729): clock, MFMA / VALU busy, LDS and wait cycles, two PMC passes.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v15}
A="tools/attn_bench.py --cases siglip_vision --batch 417"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU \
    SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT \
    --output-format csv -d ${P}_pmc1 -o run -- python3 $A > ${P}_pmc1.log 2>&1 || { tail -5 ${P}_pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d ${P}_pmc2 -o run -- python3 $A > ${P}_pmc2.log 2>&1 || { tail -5 ${P}_pmc2.log; exit 1; }
tail -2 ${P}_pmc1.log
python3 tools/pmc_kernel_sum.py attn_hyb ${P}_pmc1 ${P}_pmc2 > ${P}_attn_pmc.json && cat ${P}_attn_pmc.json
