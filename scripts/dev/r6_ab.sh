#!/bin/bash
# round 6: same-box A/B of the product library against build/variants/$1 on workload $2,
# after the GPU tests that exercise the changed kernels ($3: pytest -k expression, optional)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r6ab
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "$3" \
    > gpurun_out/r6ab/tests_$1.log 2>&1 || exit $?
fi
timeout -k 10 900 python -u scripts/dev/ab_variants.py product,$1 --workload $2 --steps 5 --warmup 2 \
  --no-pipeline --no-host-path --no-secondary > gpurun_out/r6ab/ab_$1_$2.log 2>&1
