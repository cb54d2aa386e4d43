# round-4 check: GPU suite + smoke, async A/B (IPM), small-batch IPM latency, call pattern A/B,
# endgame linear-residual diagnostic
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r4/pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 || exit 1
timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_new.json 2>&1 || exit 1
LD_LIBRARY_PATH=$PWD/build/variants/head SRBD_QP_LIB=$PWD/build/variants/head/libsrbd_qp.so timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/r4/call_pattern_head.json 2>&1 || exit 1
timeout -k 10 300 python scripts/dev/ab_variants.py head,product --workload box_u_n20 --steps 3 --warmup 1 --no-secondary --no-host-path --no-pipeline > gpurun_out/r4/ab_async_box.log 2>&1 || exit 1
timeout -k 10 300 python scripts/dev/ab_variants.py head,product --workload cone_n40_f32 --steps 3 --warmup 1 --no-secondary --no-host-path --no-pipeline > gpurun_out/r4/ab_async_cone.log 2>&1 || exit 1
SRBD_QP_LIB=$PWD/build/variants/head/libsrbd_qp.so timeout -k 10 120 python scripts/ipm_small_batch.py > gpurun_out/r4/small_head.json 2>&1 || exit 1
timeout -k 10 120 python scripts/ipm_small_batch.py > gpurun_out/r4/small_async.json 2>&1 || exit 1
SRBD_QP_LIB=$PWD/build/variants/checkonly/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_linres.py gpurun_out/r4/endgame_linres.json 64 > gpurun_out/r4/endgame_linres.log 2>&1
