# run-to-run spread of the headline on one box: the default workload 5 times, no secondaries
set -o pipefail
mkdir -p gpurun_out/variance
for i in 1 2 3 4 5; do
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-secondary --no-host-path --no-pipeline > gpurun_out/variance/run_$i.json 2> gpurun_out/variance/run_$i.err || exit 1
done
