# call pattern: latency-kernel phase stamps (tstamp build), kernel + HIP API trace of the
# shim's construct-solve-destruct loop, and the plain call-pattern numbers
set -o pipefail
mkdir -p gpurun_out/r4
V=$PWD/build/variants
SRBD_QP_LIB=$V/tstamp/libsrbd_qp.so timeout -k 10 120 python scripts/dev/latency_breakdown.py > gpurun_out/r4/lat_breakdown.json 2>&1 || exit 1
timeout -k 10 120 bash scripts/dev/r4_cp_prof.sh > gpurun_out/r4/cp_prof.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_new2.json 2>&1
