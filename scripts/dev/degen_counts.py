"""Dev aid: converged copies of the degenerate endgame family (tests/test_gpu_ipm.py) per IPM path."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import helpers  # noqa: E402

pkg = helpers.load_package()
qp, x0 = helpers.random_constrained(20, 12, 12, 4, 14, 200, pkg.OcpQpBatch)
M = 64
rng = np.random.default_rng(7)
fields = {}
for name in ("Q", "R", "S", "A", "B", "q", "r", "b", "C", "D", "lg", "ug", "lbu", "ubu", "lbx", "ubx",
             "lg_mask", "ug_mask", "lbu_mask", "ubu_mask", "lbx_mask", "ubx_mask"):
    a = getattr(qp, name, None)
    if a is None:
        continue
    a = np.repeat(np.asarray(a)[12:13], M, axis=0)
    if name in ("Q", "R", "S", "A", "B", "q", "r", "b"):
        a = a * (1 + 1e-15 * rng.standard_normal(a.shape))
    fields[name] = a
fam = pkg.OcpQpBatch(N=qp.N, nx=qp.nx, nu=qp.nu, ng=qp.ng, **fields)
xb = np.repeat(np.asarray(x0)[12:13], M, axis=0)
for path, env in (("batched", "0"), ("latency", "512")):
    os.environ["SRBD_IPM_LATENCY_MAX"] = env
    out = pkg.capi.solve(fam, xb, dict(iter_max=50, mode="Speed", ric_alg=0))
    print(path, "converged", int((out["status"] == 0).sum()), "of", M, flush=True)
