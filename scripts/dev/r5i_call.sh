#!/bin/bash
# round 5: P_{k+1} b~ from RB for B2 (record slot kRecPb) and the latency IPM's fused stage
# pass: GPU suite, same-box A/B on configs 3 and 5 against the previous library
# (build/variants/base), small-batch timing
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r5i.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r5i.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/ipm_small_batch.py 20 > gpurun_out/small_lat.json 2>/dev/null || exit $?
cat gpurun_out/small_lat.json
timeout -k 10 500 python -u scripts/dev/ab_variants.py product,base --workload box_u_n20 --no-pipeline --no-host-path --no-secondary --steps 3 --warmup 1 > gpurun_out/ab_pb_box.log 2>&1 || exit $?
tail -2 gpurun_out/ab_pb_box.log
timeout -k 10 500 python -u scripts/dev/ab_variants.py product,base --workload cone_n40_f32 --no-pipeline --no-host-path --no-secondary --steps 2 --warmup 1 > gpurun_out/ab_pb_cone.log 2>&1 || exit $?
tail -2 gpurun_out/ab_pb_cone.log
exit $rc
