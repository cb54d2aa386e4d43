set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 150 python scripts/dev/endgame_variant.py
timeout -k 10 400 python scripts/dev/ab_variants.py product,prev --workload box_u_n20 --steps 3 --warmup 1 --no-host-path --no-secondary --no-pipeline --no-gather
timeout -k 10 400 python scripts/dev/ab_variants.py product,prev --workload cone_n40_f32 --steps 3 --warmup 1 --no-host-path --no-secondary --no-pipeline --no-gather
