"""Dev aid: accuracy of the scan kernel's solution against the serial kernels' on SRBD QPs --
KKT residuals in extended precision (numpy longdouble) and the distance to the oracle."""
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402
import helpers  # noqa: E402

pkg = g._import_pkg()
oracle = helpers.load_oracle()
qp, x0 = pkg.srbd_model.generate_batch(16, N=20, seed=1003, constraints="none")
out = pkg.capi.solve(qp, x0, dict(ric_alg=0), riccati=True)
ref = oracle.solve(qp, dict(ric_alg=0), x0=x0)
L = np.longdouble


def kkt(i, s):
    N = qp.N
    x, u, pi = (np.asarray(s[k][i], dtype=L) for k in ("x", "u", "pi"))
    f = lambda n: np.asarray(getattr(qp, n)[i], dtype=L)
    Q, S, R, q, r, A, B, b = (f(n) for n in ("Q", "S", "R", "q", "r", "A", "B", "b"))
    gs = 0.0
    for k in range(N):
        ru = R[k] @ u[k] + S[k] @ x[k] + r[k] + B[k].T @ pi[k + 1]
        gs = max(gs, float(np.abs(ru).max()))
        if k > 0:
            rx = Q[k] @ x[k] + S[k].T @ u[k] + q[k] + A[k].T @ pi[k + 1] - pi[k]
            gs = max(gs, float(np.abs(rx).max()))
    rxN = Q[N] @ x[N] + q[N] - pi[N]
    gs = max(gs, float(np.abs(rxN).max()))
    eq = max(float(np.abs(A[k] @ x[k] + B[k] @ u[k] + b[k] - x[k + 1]).max()) for k in range(N))
    return gs, eq


for i in range(4):
    g_o, e_o = kkt(i, out)
    g_r, e_r = kkt(i, ref)
    dx = np.linalg.norm(out["x"][i] - ref["x"][i]) / np.linalg.norm(ref["x"][i])
    du = np.linalg.norm(out["u"][i] - ref["u"][i]) / np.linalg.norm(ref["u"][i])
    print(f"{os.environ.get('TAG','?')} qp {i}: gpu res_stat {g_o:.2e} res_eq {e_o:.2e} | oracle {g_r:.2e} {e_r:.2e} | dx {dx:.1e} du {du:.1e}")
