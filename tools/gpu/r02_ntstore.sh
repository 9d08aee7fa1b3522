set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/pers_ab.py --rows 174231 --cases fc1,h_qkv,h_fc1,h_o,h_fc2,bias_gelu --a 30 --b 44 --rounds 5 > gpurun_out/r02_ntstore.log 2>&1
