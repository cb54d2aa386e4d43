#!/bin/bash
# round 5: GPU suite with the latency IPM, degenerate-family counts per path, small-batch timing
# (latency IPM vs batched kernels), headline A/B of non-temporal data loads
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r5f.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r5f.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u scripts/dev/degen_counts.py > gpurun_out/degen_counts.log 2>&1 || exit $?
cat gpurun_out/degen_counts.log
timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 > gpurun_out/small_lat.json 2>/dev/null || exit $?
timeout -k 10 200 python -u scripts/ipm_small_batch.py 10 cone > gpurun_out/small_lat_cone.json 2>/dev/null || exit $?
SRBD_IPM_LATENCY_MAX=0 timeout -k 10 200 python -u scripts/ipm_small_batch.py 10 cone > gpurun_out/small_bat_cone.json 2>/dev/null || exit $?
cat gpurun_out/small_lat.json gpurun_out/small_lat_cone.json gpurun_out/small_bat_cone.json
timeout -k 10 400 python -u scripts/dev/ab_variants.py product,nt1,nt2 --no-pipeline --no-host-path --no-secondary --steps 30 --warmup 3 > gpurun_out/ab_nt.log 2>&1 || exit $?
tail -4 gpurun_out/ab_nt.log
exit $rc
