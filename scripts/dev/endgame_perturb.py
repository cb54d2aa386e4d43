"""Dev aid (GPU): how robustly the near-degenerate general-row QP of
tests/test_gpu_ipm.py::test_general_constraints_vs_oracle[(12, 4, 14, 200)] (#12) converges:
64 copies with its data perturbed at 1e-15 relative (rounding level), solved by the GPU
(SRBD_QP_LIB selects the build) and by the oracle; prints the status counts per ric_alg."""
import copy
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
import helpers  # noqa: E402

pkg = helpers.load_package()
oracle = helpers.load_oracle()
qp, x0 = helpers.random_constrained(20, 12, 12, 4, 14, 200, pkg.OcpQpBatch)
M = 64
rng = np.random.default_rng(7)
big = copy.deepcopy(qp)
for name in ("Q", "R", "S", "A", "B", "q", "r", "b", "C", "D", "lg", "ug", "lbu", "ubu", "lbx", "ubx",
             "lg_mask", "ug_mask", "lbu_mask", "ubu_mask", "lbx_mask", "ubx_mask"):
    a = getattr(qp, name, None)
    if a is None:
        continue
    a = np.repeat(np.asarray(a)[12:13], M, axis=0)
    if name in ("Q", "R", "S", "A", "B", "q", "r", "b"):
        a = a * (1 + 1e-15 * rng.standard_normal(a.shape))
        a[0] = np.asarray(getattr(qp, name))[12]
    setattr(big, name, a)
xb = np.repeat(np.asarray(x0)[12:13], M, axis=0)
out = {}
for ric in (0, 1):
    st = dict(iter_max=50, mode="Balance", ric_alg=ric)
    g = pkg.capi.solve(big, xb, st)
    o = oracle.solve(big, st, x0=xb)
    bad = np.nonzero(g["status"] != 0)[0]
    rel = lambda a, b: float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))
    fails = [{"copy": int(i), "iter": int(g["iter"][i]), "res": g["res"][i].tolist(),
              "u_rel_vs_oracle": rel(g["u"][i], o["u"][i]), "x_rel_vs_oracle": rel(g["x"][i], o["x"][i])}
             for i in bad[:6]]
    out[f"ric_alg {ric} failures"] = fails
    out[f"ric_alg {ric}"] = {"gpu_status_counts": {int(s): int(n) for s, n in zip(*np.unique(g["status"], return_counts=True))},
                             "oracle_status_counts": {int(s): int(n) for s, n in zip(*np.unique(o["status"], return_counts=True))},
                             "gpu_unperturbed_status": int(g["status"][0])}
print(json.dumps(out))
