#!/bin/bash
# round 6: the resident server tests, the latency IPM with refinement, the call pattern
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_riccati.py > gpurun_out/r6_server_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ipm_latency.py tests/test_gpu_ipm.py tests/test_hpipm_cpp.py > gpurun_out/r6_lat_tests.log 2>&1 || exit $?
timeout -k 10 120 ./build/call_pattern_bench > gpurun_out/r6_call_pattern.log 2>&1
