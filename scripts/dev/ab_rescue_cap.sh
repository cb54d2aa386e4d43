cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32.py -x -q -k rescue --timeout 200 --timeout-method thread > gpurun_out/fp32.log 2>&1 || exit $?
for c in 0 30 14 12 10 8; do
timeout -k 10 300 python bench.py --workload cone_n40_f32 --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-pipeline --f64-rescue $c > gpurun_out/cap$c.json 2> gpurun_out/cap$c.log || exit $?
done
