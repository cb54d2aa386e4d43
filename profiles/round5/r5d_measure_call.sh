#!/bin/bash
# round 5: lq_fact 1 as two instantiations -- the lq tests, the whole suite, the mode costs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_lq.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lq.log 2>&1; rc=$?; tail -3 $O/pytest_lq.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/ipm_modes.py 65536 3 box_u > $O/modes_box_u.json 2> $O/modes_box_u.log || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo done
