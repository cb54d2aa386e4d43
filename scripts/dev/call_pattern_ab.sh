# Dev aid (GPU): the reference call pattern with the resident server (SRBD_LAT_SERVER=1) and
# with a launch per call (=0), alternating, one line each: construct-solve-destruct median us
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for i in 1 2 3 4; do
  for s in 1 0; do
    r=$(SRBD_LAT_SERVER=$s timeout -k 10 120 python -u scripts/dev/call_pattern_profile.py 2>&1 | head -1) || exit 1
    echo "server=$s $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["construct_solve_destruct_us"]["median"], d["persistent_solver_us"]["median"], d["nmpc_step_15_solves_us"]["median"])')"
  done
done
