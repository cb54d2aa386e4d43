#!/bin/bash
# Dev aid: the latency IPM unit built with -fno-pointer-tbaa (build/variants/npt_prod; with the
# square root on C rows too: sqrtc_npt): the C = 0 / C = None probe, the GPU tests and batch-1
# timings beside the product library's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/npt
mkdir -p $O
SRBD_QP_LIB=build/variants/sqrtc_npt/libsrbd_qp.so timeout -k 10 200 python -u scripts/dev/sqrt_c_first.py > $O/first_npt.log 2>&1 || exit 1
P="python -u -m pytest --timeout 300 --timeout-method thread"
T="tests/test_gpu_ipm_latency.py tests/test_gpu_ipm.py tests/test_gpu_lq.py tests/test_gpu_mixed.py"
SRBD_QP_LIB=build/variants/npt_prod/libsrbd_qp.so timeout -k 10 400 $P $T -q > $O/tests_prod.log 2>&1; echo "rc $?" >> $O/tests_prod.log
for m in "box_u Speed 0" "cone Speed 1"; do
  n=$(echo $m | tr ' ' _)
  timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 $m > $O/small_prod_$n.json || exit 1
  SRBD_QP_LIB=build/variants/npt_prod/libsrbd_qp.so timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 $m > $O/small_npt_$n.json || exit 1
done
