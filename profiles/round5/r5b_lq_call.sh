#!/bin/bash
# round 5: lq_fact on the GPU -- the new tests first (verbose), then the whole GPU suite
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lq.py -x -v --timeout 120 --timeout-method thread > $O/pytest_lq.log 2>&1; rc=$?
tail -25 $O/pytest_lq.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log
exit $rc
