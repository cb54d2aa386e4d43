#!/bin/bash
# Dev aid: per-dispatch durations and HBM bytes of the IPM phase kernels (one solve).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/phtr; mkdir -p $O
BA="--workload ${W:-box_u_n20} --batch ${B:-16384} --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py $BA > $O/t.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d $O/p -o run -- python3 bench.py $BA > $O/p.log 2>&1 || exit $?
ls -R $O | head
