#!/bin/bash
# round 6: Balance / Robust small-batch solves on the latency IPM (with refinement) against the
# batched kernels, and a kernel trace of the reference test's compareResults (Balance, ric_alg 0)
set -o pipefail
mkdir -p gpurun_out/r6m
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in Balance Robust Speed; do
  timeout -k 10 240 python -u scripts/ipm_small_batch.py 20 box_u $m > gpurun_out/r6m/small_${m}_lat.json || exit $?
  SRBD_IPM_LATENCY_MAX=0 timeout -k 10 240 python -u scripts/ipm_small_batch.py 20 box_u $m > gpurun_out/r6m/small_${m}_batched.json || exit $?
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r6m/cmp -o cmp -- ./build/hpipm_cpp_test --golden tests/golden compareResults > gpurun_out/r6m/cmp.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r6m/con -o con -- ./build/hpipm_cpp_test --golden tests/golden constrained > gpurun_out/r6m/con.log 2>&1
