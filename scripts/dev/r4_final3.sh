# round 4 final evidence at .head: endgame counts, then r4_final.sh (suite, smoke, call
# pattern, profiles, bench line)
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 120 python scripts/dev/endgame_counts.py 0,1 Speed > gpurun_out/r4/counts_final.log 2>&1 || exit 1
bash scripts/dev/r4_final.sh
