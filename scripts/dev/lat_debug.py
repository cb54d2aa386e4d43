"""Dev aid: per-iteration statistics of one QP on the latency IPM and the batched kernels."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import helpers  # noqa: E402

pkg = helpers.load_package()
oracle = helpers.load_oracle()
nx, nu, ng = 12, 12, 14
qp, x0 = helpers.random_constrained(12, 15, nx, nu, ng, 41 + nx + ng, pkg.OcpQpBatch)
st = dict(mode="Speed", iter_max=40, ric_alg=0, split_step=1, pred_corr=1, warm_start=0,
          reg_prim=1e-12, tol_stat=1e-8, tol_eq=1e-8, tol_ineq=1e-8, tol_comp=1e-8)
np.set_printoptions(linewidth=200, precision=3)
for on in ("512", "0"):
    os.environ["SRBD_IPM_LATENCY_MAX"] = on
    out = pkg.capi.solve(qp, x0, st, stats=True)
    print("latency" if on != "0" else "batched", "status", out["status"], "iter", out["iter"])
    for i in (4, 0):
        print(" qp", i)
        for r in range(int(out["iter"][i]) + 1):
            print("  ", r, out["stat"][i, r, :11])
ref = oracle.solve(qp, st, x0=x0)
print("oracle status", ref["status"], "iter", ref["iter"])
