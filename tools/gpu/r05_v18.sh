# Round 5, step 18: pipe10 seam forms (96: SEAM 1 constants before the next tile's DMA + stores in flight
# across the seam; 98: SEAM 2 DMA between the staging passes; 99: fc1 epilogue compiled per operand set): bit-identity, fc1 microbench, job A/B.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v18
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "seams or form95" > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 200 python -u tools/gemm_bench.py --shapes fc1,h_fc1 --epi gelu --variants -1,96,98,99,-1,96,98,99 >> ${P}_gemm.log 2>&1 || exit 1
done
cat ${P}_gemm.log
for i in 1 2; do
for f in -1 99 96; do
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-parity $( [ $f != -1 ] && echo --gemm-form $f ) > ${P}_siglip_f${f}_$i.log 2>&1 || exit $?
done
done
for i in 1 2; do
for f in -1 99; do
timeout -k 10 600 python -u bench.py --model LAION-CLIP-H --no-cpu-baseline --no-parity $( [ $f != -1 ] && echo --gemm-form $f ) > ${P}_laion_f${f}_$i.log 2>&1 || exit $?
done
done
for f in ${P}_*_f*_[12].log; do echo "$f $(tail -1 $f | cut -c80-150)"; done
