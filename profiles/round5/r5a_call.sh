#!/bin/bash
# round 5, first GPU call: suite with the HPIPM-form oracle, same-box A/B of round-3 HEAD
# (bc8d3ff, build/r03tree) against HEAD on configs 3 and 5, endgame counts, and one re-run of
# round 4's faulting diagnostic build (build/variants/co_symavg_r4), last.
set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for r in 1 2; do
  for W in box_u_n20 cone_n40_f32; do
    timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > $O/ab_head_${W}_$r.json 2>/dev/null || exit 1
    (cd build/r03tree && timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --no-secondary --steps 3 --warmup 1) > $O/ab_r03_${W}_$r.json 2>/dev/null || exit 1
  done
  timeout -k 10 200 python bench.py --workload box_u_n20 --mode Balance --no-cpu-baseline --no-secondary --steps 3 --warmup 1 > $O/ab_head_box_bal_$r.json 2>/dev/null || exit 1
  (cd build/r03tree && timeout -k 10 200 python bench.py --workload box_u_n20 --mode Balance --no-cpu-baseline --no-secondary --steps 3 --warmup 1) > $O/ab_r03_box_bal_$r.json 2>/dev/null || exit 1
done
timeout -k 10 120 python scripts/dev/endgame_counts.py 0,1 Speed x > $O/endgame_counts.log 2>&1
echo counts rc=$?
SRBD_QP_LIB=$PWD/build/variants/co_symavg_r4/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_linres.py $O/endgame_co_symavg.json 64 > $O/endgame_co_symavg.log 2>&1
echo co_symavg rc=$?
