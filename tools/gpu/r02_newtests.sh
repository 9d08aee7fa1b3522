set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_config0.py tests/test_gpu_colpali.py::test_colpali_recall_vs_reference_scores \
  tests/test_gpu_encoders.py tests/test_gpu_mx.py::test_fp8_dfn5b_full_size_vs_oracle > gpurun_out/r02_newtests.log 2>&1
