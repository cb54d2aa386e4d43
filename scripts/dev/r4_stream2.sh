# (record only: the SRBD_LAT_STREAM=2 code this measured was removed after it ran, see stream_call_pattern.log)
# single-QP latency kernel, SRBD_LAT_STREAM=2 (asm LDS-DMA two stages ahead, raw barrier in the
# sweep) against the product (copy first), same box: GPU tests on the variant, then the call
# pattern alternating
set -o pipefail
mkdir -p gpurun_out/stream2
V=$PWD/build/variants/s2
SRBD_QP_LIB=$V/libsrbd_qp.so LD_LIBRARY_PATH=$V timeout -k 10 300 python3 -u -m pytest tests/test_gpu_riccati.py tests/test_hpipm_cpp.py -q --timeout 120 --timeout-method thread > gpurun_out/stream2/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python3 scripts/dev/call_pattern.py > gpurun_out/stream2/prod_$r.json 2>/dev/null || exit 1
  LD_LIBRARY_PATH=$V timeout -k 10 120 python3 scripts/dev/call_pattern.py > gpurun_out/stream2/s2_$r.json 2>/dev/null || exit 1
done
