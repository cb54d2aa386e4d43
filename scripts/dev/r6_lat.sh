#!/bin/bash
# round 6: latency IPM (refinement, square root) GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ipm_latency.py tests/test_gpu_ipm.py tests/test_gpu_lq.py tests/test_hpipm_cpp.py > gpurun_out/r6_lat_tests.log 2>&1
