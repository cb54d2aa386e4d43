# single-QP latency kernel: the QP's stages streamed into LDS during the backward sweep
# (product, SRBD_LAT_STREAM=1) against the whole copy first (-DSRBD_LAT_STREAM=0), same box:
# riccati GPU tests on the product, then the call pattern alternating the two builds
set -o pipefail
mkdir -p gpurun_out/stream
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_riccati.py tests/test_hpipm_cpp.py -q --timeout 120 --timeout-method thread > gpurun_out/stream/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python3 scripts/dev/call_pattern.py > gpurun_out/stream/prod_$r.json 2>/dev/null || exit 1
  LD_LIBRARY_PATH=$PWD/build/variants/nostream timeout -k 10 120 python3 scripts/dev/call_pattern.py > gpurun_out/stream/nostream_$r.json 2>/dev/null || exit 1
done
