set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/pers_ab.py --rows 174231 > gpurun_out/r02_pers_ab.log 2>&1 && \
timeout -k 10 200 python -u tools/pers_ab.py --rows 3000 --check-only >> gpurun_out/r02_pers_ab.log 2>&1
