# final evidence (scripts/dev/r4_final.sh), then the round-4 diagnostics of r4_diag2.sh without
# its pytest pass, on one box
set -o pipefail
bash scripts/dev/r4_final.sh || exit 1
mkdir -p gpurun_out/r4
V=$PWD/build/variants
for n in checkonly co_symavg co_div co_both; do
  SRBD_QP_LIB=$V/$n/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_linres.py gpurun_out/r4/endgame_$n.json 64 > gpurun_out/r4/endgame_$n.log 2>&1 || exit 1
done
SRBD_QP_LIB=$V/tstamp/libsrbd_qp.so timeout -k 10 120 python scripts/dev/latency_breakdown.py > gpurun_out/r4/lat_breakdown.json 2>&1 || exit 1
timeout -k 10 120 bash scripts/dev/r4_cp_prof.sh > gpurun_out/r4/cp_prof.txt 2>&1 || exit 1
LD_LIBRARY_PATH=$V/block SRBD_QP_LIB=$V/block/libsrbd_qp.so timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_block.json 2>&1
