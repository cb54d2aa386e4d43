# round-4 final evidence on ONE box: the GPU suite and smoke at this tree's HEAD, then the
# round's profiles (kernel trace + FETCH/WRITE passes of the three workloads) and the
# default bench line (scripts/profile_round.sh), all under gpurun_out/round4/
set -o pipefail
mkdir -p gpurun_out/round4
HEAD=$(cat .head 2>/dev/null || echo unknown)
echo "HEAD $HEAD" > gpurun_out/round4/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread >> gpurun_out/round4/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/round4/pytest_gpu.log; exit 1; }
echo "HEAD $HEAD" > gpurun_out/round4/smoke.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/round4/smoke.log 2>&1 || exit 1
timeout -k 10 120 python scripts/dev/call_pattern.py > gpurun_out/round4/call_pattern.json 2>&1 || exit 1
bash scripts/profile_round.sh round4
