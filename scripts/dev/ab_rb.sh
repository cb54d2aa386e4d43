cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python scripts/dev/ab_variants.py product,base --workload box_u_n20 --steps 5 --warmup 1 --no-pipeline --no-host-path > gpurun_out/ab_rb.log 2>&1 || exit $?
timeout -k 10 600 python scripts/dev/ab_variants.py product,base --workload cone_n40_f32 --steps 3 --warmup 1 --no-pipeline --no-host-path >> gpurun_out/ab_rb.log 2>&1
grep -v "^product [01]\|^base [01]" gpurun_out/ab_rb.log
