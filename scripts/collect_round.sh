#!/bin/bash
# After `gpurun -- ./scripts/profile_round.sh TAG` has merged gpurun_out/TAG back: copy the
# round's rocprofv3 summaries into profiles/TAG/ and its fresh traffic table over
# profiles/pmc_traffic.json (the file bench.py's roofline.traffic reads), so the committed
# headline numbers and the committed profiles are the same run's.  Usage: collect_round.sh TAG
cd "$(dirname "$0")/.." || exit 1
TAG=${1:?usage: collect_round.sh TAG}
SRC=gpurun_out/$TAG
[ -f $SRC/pmc_traffic.json ] && [ -f $SRC/bench_default.json ] || { echo "no complete $SRC"; exit 1; }
mkdir -p profiles/$TAG
for f in $SRC/*_kernel_stats.csv $SRC/*_summary.json $SRC/summary_*.json $SRC/bench_default.json \
         $SRC/bench_default.log; do
  [ -f "$f" ] && cp "$f" profiles/$TAG/
done
# summary_W.json is pmc_summary.py's stdout (the same object as W_summary.json): keep one
rm -f profiles/$TAG/summary_*.json
cp $SRC/pmc_traffic.json profiles/pmc_traffic.json
python3 - "$TAG" <<'EOF'
import json, sys
t = json.load(open("profiles/pmc_traffic.json"))
for w, e in t.items():
    print(f"{w:14s} {e['profile']:45s} kernel avg {e['avg_ns'] / 1e6:8.3f} ms  "
          f"{e['hbm_bytes_per_qp']:10.0f} B/QP/launch  {e['achieved_hbm_tbs']:.2f} TB/s")
print(open(f"profiles/{sys.argv[1]}/bench_default.json").read().strip()[:400])
EOF
