#!/bin/bash
# Dev aid: scripts/dev/sqrt_c_first.py on each build/variants/sc_* (the square root with C rows,
# built with one optimization switch changed), one log per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/scflags
for d in build/variants/sc_*; do
  n=$(basename $d)
  SRBD_QP_LIB=$d/libsrbd_qp.so timeout -k 10 200 python -u scripts/dev/sqrt_c_first.py > gpurun_out/scflags/$n.log 2>&1 || exit 1
done
