# round 4: the IPM's classical RB with P_k = F + K'H symmetrized (riccati.h SYMP) -- endgame
# counts in Speed, the GPU suite, and a same-box A/B of config 3 / 5 against the previous HEAD
# (build/variants/r4base); last, the square-root variant (e_sq: SRBD_SQRT_SYMP=1), ric_alg 1
set -o pipefail
mkdir -p gpurun_out/r4
V=$PWD/build/variants
timeout -k 10 120 python scripts/dev/endgame_counts.py 0,1 Speed > gpurun_out/r4/counts_product.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/pytest_sym.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r4/pytest_sym.log; exit 1; }
timeout -k 10 400 python scripts/dev/ab_variants.py product,r4base --workload box_u_n20 > gpurun_out/r4/ab_sym_box.log 2>&1 || exit 1
timeout -k 10 500 python scripts/dev/ab_variants.py product,r4base --workload cone_n40_f32 > gpurun_out/r4/ab_sym_cone.log 2>&1 || exit 1
SRBD_QP_LIB=$V/e_sq/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_counts.py 1 Speed > gpurun_out/r4/counts_e_sq.log 2>&1
