# endgame variants (check-only builds: Speed's iterates with the unrefined step's linear
# residual in the stat table); co_hk ric_alg 0 only (its SYM_AVG touches ric_alg 0's RB only)
set -o pipefail
mkdir -p gpurun_out/r4
V=$PWD/build/variants
run() { SRBD_QP_LIB=$V/$1/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_linres.py gpurun_out/r4/endgame_$1.json 64 $2 > gpurun_out/r4/endgame_$1.log 2>&1; }
run co_hk 0 && run co_hk1 0,1 && run co_div 0,1
SRBD_QP_LIB=$V/tstamp/libsrbd_qp.so timeout -k 10 120 python scripts/dev/latency_breakdown.py > gpurun_out/r4/lat_breakdown.json 2>&1 || exit 1
timeout -k 10 120 bash scripts/dev/r4_cp_prof.sh > gpurun_out/r4/cp_prof.txt 2>&1 || exit 1
LD_LIBRARY_PATH=$V/block SRBD_QP_LIB=$V/block/libsrbd_qp.so timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_block.json 2>&1
