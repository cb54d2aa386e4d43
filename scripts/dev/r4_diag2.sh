set -o pipefail
mkdir -p gpurun_out/r4
V=$PWD/build/variants
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/pytest_gpu2.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r4/pytest_gpu2.log; exit 1; }
for n in checkonly co_symavg co_div co_both; do
  SRBD_QP_LIB=$V/$n/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_linres.py gpurun_out/r4/endgame_$n.json 64 > gpurun_out/r4/endgame_$n.log 2>&1 || exit 1
done
SRBD_QP_LIB=$V/tstamp/libsrbd_qp.so timeout -k 10 120 python scripts/dev/latency_breakdown.py > gpurun_out/r4/lat_breakdown.json 2>&1 || exit 1
timeout -k 10 120 bash scripts/dev/r4_cp_prof.sh > gpurun_out/r4/cp_prof.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_new2.json 2>&1
LD_LIBRARY_PATH=$V/block SRBD_QP_LIB=$V/block/libsrbd_qp.so timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_block.json 2>&1
