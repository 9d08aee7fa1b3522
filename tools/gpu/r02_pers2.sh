set -o pipefail
export PYTHONUNBUFFERED=1
for v in 49 61 62 38 39; do
timeout -k 10 200 python -u tools/pers_ab.py --rows 174231 --cases fc1,h_o,h_fc2 --b $v --rounds 3 >> gpurun_out/r02_pers_ab2.log 2>&1 || exit 1
done
