# fp64 friction-cone config (N = 40, 65536 QPs): fp64 IPM vs the mixed-precision IPM (f32_iters)
cd $GRAFT_REPO_ROOT
for n in 0 6 8 9; do
timeout -k 10 300 python bench.py --workload cone_n40_f64 --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-pipeline --f32-iters $n > gpurun_out/mc$n.json 2> gpurun_out/mc$n.log || exit $?
done
