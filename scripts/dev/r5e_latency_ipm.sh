#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm_latency.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lat_tests.log 2>&1
rc=$?; tail -25 gpurun_out/lat_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 > gpurun_out/small_lat.json 2>gpurun_out/small_lat.err || exit $?
cat gpurun_out/small_lat.json
timeout -k 10 200 python -u scripts/ipm_small_batch.py 10 cone > gpurun_out/small_lat_cone.json 2>>gpurun_out/small_lat.err || exit $?
cat gpurun_out/small_lat_cone.json
SRBD_IPM_LATENCY_MAX=0 timeout -k 10 200 python -u scripts/ipm_small_batch.py 10 > gpurun_out/small_bat.json 2>>gpurun_out/small_lat.err || exit $?
cat gpurun_out/small_bat.json
exit $rc
