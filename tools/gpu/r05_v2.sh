# Round 5, step 2: explicit-FMA attention under -ffp-contract=off (bit-identical skip pairs), A/B against
# round 4's attention object (contraction on); the GPU suite at this build.
set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/r05_v2
OLD=multimodal-embedding_amd/build_exp/libmme_old.so
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest -q -rs --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > ${P}_pytest.log 2>&1
rc=$?; tail -2 ${P}_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
MME_LIB=$OLD timeout -k 10 200 python -u tools/attn_bench.py --cases siglip_vision,dfn5b_vision,vitH_vision,clipL_vision,siglip_text_2500 --batch 417 >> ${P}_attn_old.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/attn_bench.py --cases siglip_vision,dfn5b_vision,vitH_vision,clipL_vision,siglip_text_2500 --batch 417 >> ${P}_attn_new.log 2>&1 || exit 1
done
