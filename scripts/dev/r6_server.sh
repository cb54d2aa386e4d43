#!/bin/bash
# round 6: the resident server -- queue-sharing probe, relaunch-after-post and other-stream tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_riccati.py > gpurun_out/r6_server_tests.log 2>&1 || exit $?
timeout -k 10 120 ./build/call_pattern_bench > gpurun_out/r6_call_pattern.log 2>&1
