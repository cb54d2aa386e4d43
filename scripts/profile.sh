#!/bin/bash
# rocprofv3 kernel stats + HBM PMC counters (separate --pmc passes, per the
# MI355X guide) for one bench workload.  Usage: profile.sh TAG WORKLOAD [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=$1; W=$2; shift 2
OUT=gpurun_out/prof_${TAG}_${W}
mkdir -p $OUT
BA="--workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-pipeline --no-host-path --no-secondary $*"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $BA > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $BA > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $BA > $OUT/write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -20
