# Round 5, step 19: form 99 (every pipe9 / pipe10 epilogue compiled for its operand set, gemm_epilogue_wave
# FOLD 1 / 2 / 3): bit-identity against pipe6, per-shape microbench, job A/B on four models.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v19
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 240 python -u tools/resstats_forms_debug.py > ${P}_resstats_debug.log 2>&1 || exit 1
cat ${P}_resstats_debug.log
timeout -k 10 500 python -u -m pytest -q -s --timeout 400 --timeout-method thread tests/test_gpu_kernels.py -k "seams or form95" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc  # 1 = a bit-identity assertion: timing still informative
for e in gelu res none; do
V=-1,99,-1,99; [ $e = gelu ] && V=-1,99,96,-1,99,96
timeout -k 10 200 python -u tools/gemm_bench.py --shapes qkv,o_proj,fc1,fc2 --epi $e --variants=$V >> ${P}_gemm.log 2>&1 || exit 1
done
cat ${P}_gemm.log
for i in 1 2; do
for m in SigLIP-400M LAION-CLIP-H; do
for f in -1 99; do
timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline --no-parity $( [ $f != -1 ] && echo --gemm-form $f ) > ${P}_${m}_f${f}_$i.log 2>&1 || exit $?
done
done
done
for m in OpenAI-CLIP-L Apple-DFN5B-H; do
for f in -1 99; do
timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline --no-parity $( [ $f != -1 ] && echo --gemm-form $f ) > ${P}_${m}_f${f}_1.log 2>&1 || exit $?
done
done
for f in ${P}_*_f*_[12].log; do echo "$f $(tail -1 $f | cut -c80-150)"; done
