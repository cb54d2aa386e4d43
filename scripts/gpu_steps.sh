#!/bin/bash
# One parameterised GPU call (replaces the per-experiment r5*/r6* launch scripts): runs the
# named steps in order on the box, each under its own time limit, and stops at the first step
# that fails (no retries: a GPU step that faults or times out ends the call).
#
#   gpurun -- ./scripts/gpu_steps.sh [-o OUTDIR] STEP [STEP ...]
#
# STEP                          what it runs (outputs under OUTDIR, default gpurun_out/steps)
#   suite                       the whole GPU suite (pytest -m gpu)
#   tests:EXPR                  pytest -m gpu -k EXPR, verbose
#   file:PATH                   pytest PATH, verbose (a test file, GPU tests included)
#   small:MODE:CONS[:RIC]       scripts/ipm_small_batch.py (batches 1..1024, N = 20) in HPIPM mode
#                               MODE on SRBD QPs CONS (box_u / cone), latency IPM and batched;
#                               RIC: ric_alg (0 classical, the default; 1 square root)
#   ab:VARIANT:WORKLOAD         scripts/dev/ab_variants.py: product vs build/variants/VARIANT
#   modes:CONS                  scripts/ipm_modes.py: IPM cost by mode / lq_fact, 65536 QPs
#   degen                       scripts/dev/degen_counts.py: degenerate-family counts per path
#   profile:WORKLOAD            scripts/profile.sh (kernel trace + FETCH / WRITE passes)
#   refcase:CASE                rocprofv3 kernel trace of build/hpipm_cpp_test CASE
#   callpattern[:TREE]          bench.py's reference_call_pattern line (the reference's one-QP
#                               call pattern, build/call_pattern_bench) 3 times; with TREE (a
#                               built worktree, e.g. build/r05tree) alternating with that tree
#   bench                       the default bench.py line
#   smoke                       __graft_entry__.smoke()
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/steps
if [ "$1" = "-o" ]; then O=$2; shift 2; fi
mkdir -p "$O"
PYT="python -u -m pytest --timeout 300 --timeout-method thread"
for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  echo "== $step" >&2
  case $kind in
    suite) timeout -k 10 900 $PYT tests -m gpu -q > "$O/suite.log" 2>&1 ;;
    tests) timeout -k 10 600 $PYT tests -m gpu -v -k "$a" > "$O/tests_${a//[^A-Za-z0-9_]/_}.log" 2>&1 ;;
    file) timeout -k 10 600 $PYT "$a" -v > "$O/file_$(basename "$a" .py).log" 2>&1 ;;
    small)
      timeout -k 10 300 python -u scripts/ipm_small_batch.py 20 "$b" "$a" ${c:-0} > "$O/small_${a}_${b}${c:+_ric$c}_lat.json" &&
        SRBD_IPM_LATENCY_MAX=0 timeout -k 10 300 python -u scripts/ipm_small_batch.py 20 "$b" "$a" ${c:-0} \
          > "$O/small_${a}_${b}${c:+_ric$c}_batched.json" ;;
    ab) timeout -k 10 900 python -u scripts/dev/ab_variants.py "product,$a" --workload "$b" --steps 5 --warmup 2 \
          --no-pipeline --no-host-path --no-secondary > "$O/ab_${a}_${b}.log" 2>&1 ;;
    modes) timeout -k 10 600 python scripts/ipm_modes.py 65536 3 "$a" > "$O/modes_$a.json" 2> "$O/modes_$a.log" ;;
    degen) timeout -k 10 300 python -u scripts/dev/degen_counts.py > "$O/degen_counts.log" 2>&1 ;;
    profile) timeout -k 10 900 ./scripts/profile.sh steps "$a" > "$O/profile_$a.log" 2>&1 ;;
    refcase) timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/ref_$a" -o "$a" -- \
               ./build/hpipm_cpp_test --golden tests/golden "$a" > "$O/ref_$a.log" 2>&1 ;;
    callpattern)
      for r in 1 2 3; do
        timeout -k 10 120 python -u scripts/dev/call_pattern.py >> "$O/call_pattern.log" 2>&1 || exit $?
        if [ -n "$a" ]; then
          (cd "$a" && timeout -k 10 120 python -u scripts/dev/call_pattern.py) >> "$O/call_pattern_$(basename "$a").log" 2>&1 || exit $?
        fi
      done ;;
    bench) timeout -k 10 600 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.log" ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then echo "step $step failed (rc $rc)" >&2; exit $rc; fi
done
echo done >&2
