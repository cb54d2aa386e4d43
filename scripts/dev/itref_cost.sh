BA="--steps 2 --warmup 1 --no-cpu-baseline --no-pipeline --no-host-path --no-secondary"
for m in Speed Balance Robust; do
  timeout -k 10 300 python3 bench.py --workload box_u_n20 --mode $m $BA > gpurun_out/mode_box_$m.json 2> gpurun_out/mode_box_$m.log || exit $?
done
for m in Speed Balance; do
  timeout -k 10 300 python3 bench.py --workload cone_n40_f32 --mode $m $BA > gpurun_out/mode_cone_$m.json 2> gpurun_out/mode_cone_$m.log || exit $?
done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/mode_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d['roofline']['kernel_avg_ms'],2), d['success_rate'], d['iters_mean'])
"
