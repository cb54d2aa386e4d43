#!/bin/bash
# One gpurun call that backs a round's numbers on ONE box: rocprofv3 kernel trace and the
# separate FETCH_SIZE / WRITE_SIZE passes of the default workload and the two IPM configs,
# summarised (scripts/pmc_summary.py -> profiles/TAG/ and profiles/pmc_traffic.json on the
# box), then the default bench line itself, which reads that fresh traffic summary.
# Everything is written under gpurun_out/TAG/ (merged back); scripts/collect_round.sh TAG then
# copies it into profiles/TAG/ and profiles/pmc_traffic.json.
# Usage: profile_round.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for W in unconstr_n20 box_u_n20 cone_n40_f32; do
  STEPS=20; [ $W != unconstr_n20 ] && STEPS=2
  timeout -k 10 300 ./scripts/profile.sh $TAG $W --steps $STEPS > $OUT/profile_$W.log 2>&1 || exit $?
  SOLVES=$((STEPS + 1))
  timeout -k 10 120 python3 scripts/pmc_summary.py $TAG $W 65536 $SOLVES > $OUT/summary_$W.json 2>&1 || exit $?
  cp profiles/$TAG/${W}_* $OUT/ || exit $?
done
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.log || exit $?
echo done
