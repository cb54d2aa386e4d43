#!/bin/bash
# Dev aid: a latency-IPM variant build (build/variants/$1): its latency-IPM GPU tests and
# batch-1..1024 timings of the square root beside the product library's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
V=build/variants/$1/libsrbd_qp.so
O=gpurun_out/var_$1
mkdir -p $O
SRBD_QP_LIB=$V timeout -k 10 300 python -u -m pytest --timeout 300 --timeout-method thread tests/test_gpu_ipm_latency.py -q > $O/tests.log 2>&1; echo "rc $?" >> $O/tests.log
for m in "box_u Speed 1" "cone Speed 1" "box_u Balance 1"; do
  n=$(echo $m | tr ' ' _)
  timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 $m > $O/small_prod_$n.json || exit 1
  SRBD_QP_LIB=$V timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 $m > $O/small_var_$n.json || exit 1
done
