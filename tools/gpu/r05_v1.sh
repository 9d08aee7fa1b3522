# Round 5, step 1: fp-contract experiment on the flash loops (verdict item 8) + a baseline bench on this box.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v1
NC=multimodal-embedding_amd/build_exp/libmme_nc.so
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "skip_vs_unskipped or threshold_vs_exact" > ${P}_skip_contract_on.log 2>&1; echo "contract on rc=$?"
MME_LIB=$NC timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "skip_vs_unskipped or threshold_vs_exact" > ${P}_skip_contract_off.log 2>&1; echo "contract off rc=$?"
for i in 1 2; do
timeout -k 10 200 python -u tools/attn_bench.py --cases siglip_vision,dfn5b_vision,vitH_vision,clipL_vision --batch 417 >> ${P}_attn_on.log 2>&1 || exit 1
MME_LIB=$NC timeout -k 10 200 python -u tools/attn_bench.py --cases siglip_vision,dfn5b_vision,vitH_vision,clipL_vision --batch 417 >> ${P}_attn_off.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py > ${P}_bench.log 2>&1 || exit $?
tail -1 ${P}_bench.log | cut -c1-300
