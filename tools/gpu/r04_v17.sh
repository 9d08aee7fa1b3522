# Round 4 step 17: staggered hd-72 attention (dev kind 79: the late wave row runs PV one tile behind on a
# four-slot ring, asm DMA) and the three-slot ring (kind 78) against production kind 62, SigLIP job batch.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v17}
MME_DEV=1 timeout -k 10 300 python -u tools/attn_bench.py --cases siglip_vision --batch 417 \
    --variants 0,109,108,0,109,108,0,109,108 > ${P}_stagger_bench.log 2>&1 || { cat ${P}_stagger_bench.log; exit 1; }
cat ${P}_stagger_bench.log
MME_DEV=1 timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread -m gpu \
    -k "ring_forms" tests/test_gpu_kernels.py > ${P}_ring_pytest.log 2>&1; rc=$?
grep -E "kinds 62|passed|failed" ${P}_ring_pytest.log | tail -30
exit $rc
