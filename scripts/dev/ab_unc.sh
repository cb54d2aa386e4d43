cd $GRAFT_REPO_ROOT
timeout -k 10 700 python scripts/dev/ab_variants.py ${VARIANTS:-product} --steps 10 --warmup 2 --no-pipeline --no-host-path --no-secondary > gpurun_out/ab_unc.log 2>&1
rc=$?; grep -v " [01] (" gpurun_out/ab_unc.log; exit $rc
