# Speed-mode endgame: unrefined-step linear residual per variant (checkonly builds)
set -o pipefail
mkdir -p gpurun_out/r4
V=$PWD/build/variants
for n in checkonly co_symavg co_div co_both; do
  SRBD_QP_LIB=$V/$n/libsrbd_qp.so timeout -k 10 120 python scripts/dev/endgame_linres.py gpurun_out/r4/endgame_$n.json 64 > gpurun_out/r4/endgame_$n.log 2>&1 || exit 1
done
