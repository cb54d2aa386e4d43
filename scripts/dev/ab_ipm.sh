# A/B of IPM library variants (build/variants/*) on box-u N=20 and cone N=40 fp32
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py tests/test_gpu_fp32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ipm.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ipm.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python scripts/dev/ab_variants.py ${VARIANTS:-product} --workload box_u_n20 --steps 5 --warmup 1 --no-pipeline --no-host-path --no-secondary > gpurun_out/ab_ipm.log 2>&1 || exit $?
timeout -k 10 600 python scripts/dev/ab_variants.py ${VARIANTS:-product} --workload cone_n40_f32 --steps 3 --warmup 1 --no-pipeline --no-host-path --no-secondary >> gpurun_out/ab_ipm.log 2>&1
grep -v " [01] (" gpurun_out/ab_ipm.log
