#!/bin/bash
# round 5: latency IPM, symmetrized F - Y'Y (product) against F + K'H (pkh variant)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in product pkh; do
  if [ $v = product ]; then unset SRBD_QP_LIB; else export SRBD_QP_LIB=build/variants/$v/libsrbd_qp.so; fi
  echo "== $v"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm_latency.py -q --timeout 120 --timeout-method thread > gpurun_out/lat_tests_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/lat_tests_$v.log; [ $rc -le 1 ] || exit $rc
  timeout -k 10 120 python -u scripts/dev/degen_counts.py 2>&1 | grep conv || exit 1
  timeout -k 10 120 python -u scripts/dev/lat_debug.py 2>&1 | grep status || exit 1
  timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 2>/dev/null | cut -c1-200 || exit 1
done
