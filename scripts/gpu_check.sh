#!/bin/bash
# One gpurun call: GPU parity tests -> smoke -> short bench -> rocprofv3 kernel stats.
# Stops at the first step that faults / times out (exit codes >= 124 or pytest > 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2"}
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json; tail -3 gpurun_out/bench_${TAG}.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$NO_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $PROF_ARGS > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  find gpurun_out/prof_${TAG} -name "*stats*" | head
fi
exit 0
