# round-4 check: latency kernel first (riccati tests), then the GPU suite + smoke, call
# pattern (product / no-MFMA / round-3 head), IPM async A/B, small-batch IPM, endgame diag
set -o pipefail
mkdir -p gpurun_out/r4
V=$PWD/build/variants
timeout -k 10 240 python -u -m pytest tests/test_gpu_riccati.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/pytest_riccati.log 2>&1 || { echo RICCATI_FAIL; tail -40 gpurun_out/r4/pytest_riccati.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r4/pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 || exit 1
timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_new.json 2>&1 || exit 1
LD_LIBRARY_PATH=$V/nolat SRBD_QP_LIB=$V/nolat/libsrbd_qp.so timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_nolat.json 2>&1 || exit 1
LD_LIBRARY_PATH=$V/head SRBD_QP_LIB=$V/head/libsrbd_qp.so timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_head.json 2>&1 || exit 1
timeout -k 10 300 python scripts/dev/ab_variants.py head,product --workload box_u_n20 --steps 3 --warmup 1 --no-secondary --no-host-path --no-pipeline > gpurun_out/r4/ab_async_box.log 2>&1 || exit 1
timeout -k 10 300 python scripts/dev/ab_variants.py head,product --workload cone_n40_f32 --steps 3 --warmup 1 --no-secondary --no-host-path --no-pipeline > gpurun_out/r4/ab_async_cone.log 2>&1 || exit 1
SRBD_QP_LIB=$V/head/libsrbd_qp.so timeout -k 10 120 python scripts/ipm_small_batch.py > gpurun_out/r4/small_head.json 2>&1 || exit 1
timeout -k 10 120 python scripts/ipm_small_batch.py > gpurun_out/r4/small_async.json 2>&1 || exit 1
SRBD_QP_LIB=$V/checkonly/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_linres.py gpurun_out/r4/endgame_linres.json 64 > gpurun_out/r4/endgame_linres.log 2>&1
