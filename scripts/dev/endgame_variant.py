"""Dev aid: stall counts of the degenerate general-row family with a variant library
(SRBD_QP_LIB=build/variants/NAME/libsrbd_qp.so)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
print("lib", pkg.capi.lib()._name)
for dims in [(8, 12, 12, 40), (12, 12, 4, 14)]:
    N, nx, nu, ng = dims
    for ric in (0, 1):
        bad = 0
        for seed in range(200, 205):
            qp, x0 = helpers.random_constrained(100, N, nx, nu, ng, seed, pkg.OcpQpBatch)
            out = pkg.capi.solve(qp, x0, dict(iter_max=50, mode="Balance", ric_alg=ric))
            bad += int((out["status"] != 0).sum())
        print(dims, "ric_alg", ric, "unsolved", bad, "/ 500", flush=True)
