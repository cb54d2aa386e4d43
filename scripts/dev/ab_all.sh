# A/B of library variants on all three benchmarked kernels + GPU parity of the last variant
cd $GRAFT_REPO_ROOT
LAST=${VARIANTS##*,}
SRBD_QP_LIB=$PWD/build/variants/$LAST/libsrbd_qp.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_variant.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_variant.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python scripts/dev/ab_variants.py ${VARIANTS} --steps 10 --warmup 2 --no-pipeline --no-host-path --no-secondary > gpurun_out/ab_all.log 2>&1 || exit $?
timeout -k 10 600 python scripts/dev/ab_variants.py ${VARIANTS} --workload box_u_n20 --steps 5 --warmup 1 --no-pipeline --no-host-path --no-secondary >> gpurun_out/ab_all.log 2>&1 || exit $?
timeout -k 10 600 python scripts/dev/ab_variants.py ${VARIANTS} --workload cone_n40_f32 --steps 3 --warmup 1 --no-pipeline --no-host-path --no-secondary >> gpurun_out/ab_all.log 2>&1
grep -v " [01] (" gpurun_out/ab_all.log
