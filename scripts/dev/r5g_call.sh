#!/bin/bash
# round 5: latency IPM with fused-DPP factorization pieces: parity tests, batch-1 breakdown, timing
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm_latency.py tests/test_gpu_ipm.py -q --timeout 120 --timeout-method thread > gpurun_out/lat_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lat_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u scripts/dev/degen_counts.py > gpurun_out/degen_counts.log 2>&1 || exit $?
cat gpurun_out/degen_counts.log
SRBD_QP_LIB=build/variants/tstamp/libsrbd_qp.so timeout -k 10 120 python -u scripts/dev/lat_ipm_breakdown.py box_u > gpurun_out/lat_breakdown.json 2>&1 || exit $?
timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 > gpurun_out/small_lat.json 2>/dev/null || exit $?
cat gpurun_out/small_lat.json
exit $rc
