#!/bin/bash
# One gpurun call: the bench line of every workload (default first, full line).
# Usage: bench_all.sh TAG [extra bench args for the secondary workloads]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-dev}; shift
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-secondary > gpurun_out/bench_${TAG}_unconstr_n20.json 2> gpurun_out/bench_${TAG}_unconstr_n20.log || exit $?
for W in box_u_n20 cone_n40_f32 unconstr_n10_b4096; do
  timeout -k 10 300 python bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-pipeline --no-host-path "$@" \
    > gpurun_out/bench_${TAG}_${W}.json 2> gpurun_out/bench_${TAG}_${W}.log || exit $?
done
for f in gpurun_out/bench_${TAG}_*.json; do
  python -c "import json,sys; d=json.load(open('$f')); r=d['roofline']; print('$f', d['config']['workload'], '%.4g QP/s'%d['value'], 'kernel %.3f ms'%r['kernel_avg_ms'], 'frac %.3f'%r['frac'], 'ok %.3f'%d['success_rate'], 'it %.2f'%d['iters_mean'])"
done
