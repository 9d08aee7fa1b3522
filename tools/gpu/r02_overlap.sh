set -o pipefail
export PYTHONUNBUFFERED=1
# A/B/A/B: text tower on a second stream beside the vision tower vs serial
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > gpurun_out/r02_overlap_serial_$i.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --overlap-towers > gpurun_out/r02_overlap_on_$i.log 2>&1 || exit 1
done
