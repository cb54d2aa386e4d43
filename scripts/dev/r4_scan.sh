# round 4: the parallel-in-time single-QP kernel -- its tests first, then the whole GPU suite,
# then the reference call pattern against the serial matrix-core kernel (-DSRBD_SCAN=0)
set -o pipefail
mkdir -p gpurun_out/r4
V=$PWD/build/variants
SRBD_QP_LIB=$V/dump1/libsrbd_qp.so timeout -k 10 60 python scripts/dev/scan_debug.py 1 > gpurun_out/r4/scan_dbg1.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_riccati.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4/pytest_scan.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r4/pytest_scan.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/pytest_scan_all.log 2>&1 || { echo PYTEST_ALL_FAIL; tail -40 gpurun_out/r4/pytest_scan_all.log; exit 1; }
timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/cp_scan.json 2>&1 || exit 1
LD_LIBRARY_PATH=$V/noscan SRBD_QP_LIB=$V/noscan/libsrbd_qp.so timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/cp_noscan.json 2>&1 || exit 1
timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/cp_scan2.json 2>&1
