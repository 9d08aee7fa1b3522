set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py \
  tests/test_gpu_encoders.py::test_fused_statistics_at_production_geometry tests/test_gpu_colpali.py::test_colpali_recall_vs_reference_scores > gpurun_out/r02_t2.log 2>&1
