# the GPU suite and smoke once more at .head (after the last test was added)
set -o pipefail
mkdir -p gpurun_out/round4_suite
HEAD=$(cat .head 2>/dev/null || echo unknown)
echo "HEAD $HEAD" > gpurun_out/round4_suite/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread >> gpurun_out/round4_suite/pytest_gpu.log 2>&1 || exit 1
echo "HEAD $HEAD" > gpurun_out/round4_suite/smoke.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/round4_suite/smoke.log 2>&1
