# Round 5, step 21: form 95 (pipe10 on every non-split GEMM) with the compiled epilogues (residual = FOLD 3)
# against the production dispatch (pipe9 for the non-fc1 GEMMs): bit-identity and job A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v21
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "form95" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/gemm_bench.py --shapes h_qkv,h_fc2,1280:1280 --rows 116935 --epi res --variants=-1,95,-1,95 > ${P}_gemm.log 2>&1 || exit 1
cat ${P}_gemm.log
for i in 1 2; do
for m in LAION-CLIP-H Apple-DFN5B-H OpenAI-CLIP-L; do
for f in -1 95; do
timeout -k 10 600 python -u bench.py --model $m --no-cpu-baseline --no-parity $( [ $f != -1 ] && echo --gemm-form $f ) > ${P}_${m}_f${f}_$i.log 2>&1 || exit $?
done
done
done
for f in ${P}_*_f*_[12].log; do echo "$f $(tail -1 $f | cut -c80-150)"; done
