set -o pipefail
mkdir -p gpurun_out/r4
V=$PWD/build/variants
SRBD_QP_LIB=$V/dump2/libsrbd_qp.so timeout -k 10 60 python scripts/dev/scan_debug.py 2 > gpurun_out/r4/scan_dbg2.log 2>&1
SRBD_QP_LIB=$V/dump1/libsrbd_qp.so timeout -k 10 60 python scripts/dev/scan_debug.py 1 > gpurun_out/r4/scan_dbg1.log 2>&1
timeout -k 10 60 python scripts/dev/scan_debug.py 0 > gpurun_out/r4/scan_dbg0.log 2>&1
cat gpurun_out/r4/scan_dbg2.log gpurun_out/r4/scan_dbg1.log gpurun_out/r4/scan_dbg0.log
