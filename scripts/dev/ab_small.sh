# A/B of unconstrained-kernel variants on the small-batch configuration (BASELINE config 2)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python scripts/dev/ab_variants.py ${VARIANTS} --workload unconstr_n10_b4096 --steps 50 --warmup 5 --no-pipeline --no-host-path --no-secondary > gpurun_out/ab_small.log 2>&1 || exit $?
timeout -k 10 600 python scripts/dev/ab_variants.py ${VARIANTS} --workload unconstr_n10_b4096 --batch 1024 --steps 50 --warmup 5 --no-pipeline --no-host-path --no-secondary >> gpurun_out/ab_small.log 2>&1 || exit $?
grep -v " [01] (" gpurun_out/ab_small.log
