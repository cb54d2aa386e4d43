# round 4, after the symmetrized-textbook P_k change: endgame counts, a same-box A/B of config 3
# against the previous HEAD (build/variants/r4base), then the final evidence (r4_final.sh)
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 120 python scripts/dev/endgame_counts.py 0,1 Speed > gpurun_out/r4/counts_final.log 2>&1 || exit 1
timeout -k 10 400 python scripts/dev/ab_variants.py product,r4base --workload box_u_n20 > gpurun_out/r4/ab_final_box.log 2>&1 || exit 1
SRBD_QP_LIB=$PWD/build/variants/e_xp/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_counts.py 1 Speed > gpurun_out/r4/counts_e_xp.log 2>&1 || exit 1
bash scripts/dev/r4_final.sh
