# Round 4 step 20: kind 83 (hd 72 with the 2^8 rescale threshold) as production: GPU suite, the SigLIP job;
# hd-80 threshold kinds 86 / 87 against production kinds 65 / 38 (ViT-H T 257, DFN5B T 730); hd 64
# attn_fwd_kernel with the threshold (kind 89) against kind 0 (CLIP-L vision, CLIP causal text).
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/${RUN:-r04_v20}
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/attn_bench.py --cases vitH_vision,dfn5b_vision --batch 417 \
    --variants 0,116,117,0,116,117,0,116,117 > ${P}_hd80_thr_bench.log 2>&1 || { cat ${P}_hd80_thr_bench.log; exit 1; }
cat ${P}_hd80_thr_bench.log
timeout -k 10 300 python -u tools/attn_bench.py --cases clipL_vision,clip_text_causal \
    --variants 0,119,0,119,0,119 > ${P}_fwd_thr_bench.log 2>&1 || { cat ${P}_fwd_thr_bench.log; exit 1; }
cat ${P}_fwd_thr_bench.log
timeout -k 10 300 python -u tools/attn_err.py --variants 0,113 > ${P}_thr_err.log 2>&1 || { cat ${P}_thr_err.log; exit 1; }
cat ${P}_thr_err.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > ${P}_bench.log 2>&1 || exit $?
tail -1 ${P}_bench.log | cut -c1-200
