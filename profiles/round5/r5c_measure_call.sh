#!/bin/bash
# round 5: the fp32 LQ test; IPM cost by mode / lq_fact on box-u and cone (65536 QPs, N = 20);
# batch-1 box-u kernel trace (launch structure of a small solve)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_lq.py -x -q --timeout 120 --timeout-method thread -k fp32 > $O/pytest_lq_fp32.log 2>&1; rc=$?; tail -5 $O/pytest_lq_fp32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/ipm_modes.py 65536 3 box_u > $O/modes_box_u.json 2> $O/modes_box_u.log || exit 1
timeout -k 10 400 python scripts/ipm_modes.py 65536 2 cone > $O/modes_cone.json 2> $O/modes_cone.log || exit 1
timeout -k 10 120 python scripts/ipm_small_batch.py 20 > $O/small_batch.json 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_small -o small -- python3 scripts/ipm_small_batch.py 5 > $O/prof_small.log 2>&1 || exit 1
echo done
