set -o pipefail
mkdir -p gpurun_out/r4x
cd /root/repo
timeout -k 10 240 python3 -u scripts/dev/endgame_counts.py 1 Speed d > gpurun_out/r4x/prod.log 2>&1 &&
SRBD_QP_LIB=build/variants/e_xp0/libsrbd_qp.so timeout -k 10 180 python3 -u scripts/dev/endgame_counts.py 1 Speed d > gpurun_out/r4x/xp0.log 2>&1 &&
SRBD_QP_LIB=build/variants/e_sq/libsrbd_qp.so timeout -k 10 180 python3 -u scripts/dev/endgame_counts.py 1 Speed d > gpurun_out/r4x/sq.log 2>&1
