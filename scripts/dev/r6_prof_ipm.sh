#!/bin/bash
# round 6: per-dispatch traffic of the IPM workloads (config 5 cone_n40_f32, config 3 box_u_n20)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for w in cone_n40_f32 box_u_n20; do
  ./scripts/profile.sh round6 $w || exit $?
done
