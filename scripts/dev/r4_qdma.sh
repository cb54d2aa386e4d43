# Q_k by LDS-DMA in the fp64 box RB: GPU suite, then same-box A/B against the register-load build
set -o pipefail
mkdir -p gpurun_out/qdma
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qdma/pytest.log 2>&1 &&
timeout -k 10 400 python3 -u scripts/dev/ab_variants.py product,noqdma --workload box_u_n20 --steps 2 > gpurun_out/qdma/ab_box_u.log 2>&1
