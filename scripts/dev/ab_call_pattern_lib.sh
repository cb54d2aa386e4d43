mkdir -p gpurun_out/r6aug
SRBD_QP_LIB=$PWD/build/variants/aug/libsrbd_qp.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_riccati.py > gpurun_out/r6aug/tests.log 2>&1 || exit $?
for r in 1 2 3; do
  timeout -k 10 120 python -u scripts/dev/call_pattern.py >> gpurun_out/r6aug/cp_product.log 2>&1 || exit $?
  LD_LIBRARY_PATH=$PWD/build/variants/aug SRBD_QP_LIB=$PWD/build/variants/aug/libsrbd_qp.so timeout -k 10 120 python -u scripts/dev/call_pattern.py >> gpurun_out/r6aug/cp_aug.log 2>&1 || exit $?
done
