# ric_alg 1 with the oracle's P_k sequence (-DSRBD_SQRT_RECON=1, with / without the symmetrized
# textbook P_k and explicit-P records): Speed counts on the degenerate family, oracle distances
set -o pipefail
mkdir -p gpurun_out/recon
for v in rc rc_sym rc_sym_xp; do
  SRBD_QP_LIB=build/variants/$v/libsrbd_qp.so timeout -k 10 180 python3 -u scripts/dev/endgame_counts.py 1 Speed d > gpurun_out/recon/$v.log 2>&1 || exit 1
done
