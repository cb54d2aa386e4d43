# latency kernel: one Newton step on v_rcp_f64 (-DSRBD_LAT_NEWTON=1) against two, same box:
# the reference call pattern, alternating builds; then the riccati GPU tests on the variant
set -o pipefail
mkdir -p gpurun_out/newton
for r in 1 2; do
  timeout -k 10 120 python3 scripts/dev/call_pattern.py > gpurun_out/newton/prod_$r.json 2>/dev/null || exit 1
  LD_LIBRARY_PATH=$PWD/build/variants/n1 timeout -k 10 120 python3 scripts/dev/call_pattern.py > gpurun_out/newton/n1_$r.json 2>/dev/null || exit 1
done
SRBD_QP_LIB=build/variants/n1/libsrbd_qp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_riccati.py -q --timeout 120 --timeout-method thread > gpurun_out/newton/pytest_n1.log 2>&1
