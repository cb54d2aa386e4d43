"""Dev aid: the scan kernel's diagnostic builds (-DSRBD_SCAN_DUMP=1/2: P, p outputs = the
scan's J, zeta after all rounds / after none) against numpy on one SRBD QP."""
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO))
import __graft_entry__ as g  # noqa: E402

mode = int(sys.argv[1])
pkg = g._import_pkg()
qp, x0 = pkg.srbd_model.generate_batch(1, N=20, seed=1003, constraints="none")
N = 20
f = lambda n: np.asarray(getattr(qp, n)[0])
Q, S, R, q, r, A, B, b = (f(n) for n in ("Q", "S", "R", "q", "r", "A", "B", "b"))
out = pkg.capi.solve(qp, x0, dict(ric_alg=0), riccati=True)
if mode == 2:
    for k in range(N):
        Ri = np.linalg.inv(R[k])
        J = Q[k] - S[k].T @ Ri @ S[k]
        z = q[k] - S[k].T @ Ri @ r[k]
        Ab = A[k] - B[k] @ Ri @ S[k]
        eJ = np.abs(out["P"][0, k] - J).max() / np.abs(J).max()
        ez = np.abs(out["p"][0, k] - z).max() / np.abs(z).max()
        eA = np.abs(out["K"][0, k].T - Ab).max() / np.abs(Ab).max()
        eAn = np.abs(out["K"][0, k] - Ab).max() / np.abs(Ab).max()
        print(k, "J %.2e zeta %.2e A(as K^T) %.2e A(as K) %.2e" % (eJ, ez, eA, eAn))
        if eAn > 0:
            Kk = out["K"][0, k]
            cands = {"Q": Q[k], "Q'": Q[k].T, "A'": Ab.T, "B": B[k], "R": R[k], "S": S[k], "0": 0 * Q[k],
                     "Qk+1": Q[k + 1], "Ak+1": A[k + 1] if k + 1 < N else 0 * Q[k], "Ak-1": A[k - 1]}
            best = min(cands, key=lambda c: np.abs(Kk - cands[c]).max())
            print("   K closest to", best, "%.2e" % np.abs(Kk - cands[best]).max(),
                  "col-diff", [float("%.1e" % np.abs(Kk[:, j] - Ab[:, j]).max()) for j in range(12)])
        if ez > 0:
            print("   p", np.round(out["p"][0, k], 4), "q", np.round(z, 4), "b", np.round(b[k], 4))
else:
    P = Q[N].copy(); p = q[N].copy(); Ps = {N: P}; ps = {N: p}
    for k in range(N - 1, -1, -1):
        G = R[k] + B[k].T @ P @ B[k]; H = S[k] + B[k].T @ P @ A[k]; F = Q[k] + A[k].T @ P @ A[k]
        w = P @ b[k] + p; gg = r[k] + B[k].T @ w; ff = q[k] + A[k].T @ w
        K = -np.linalg.solve(G, H); kk = -np.linalg.solve(G, gg)
        P = F + H.T @ K; P = 0.5 * (P + P.T); p = ff + K.T @ gg; Ps[k] = P; ps[k] = p
    Ks = {}
    P = Q[N].copy()
    for k in range(N - 1, -1, -1):
        G = R[k] + B[k].T @ Ps[k + 1] @ B[k]; H = S[k] + B[k].T @ Ps[k + 1] @ A[k]
        Ks[k] = -np.linalg.solve(G, H)
    for k in range(N + 1):
        eP = np.abs(out["P"][0, k] - Ps[k]).max() / np.abs(Ps[k]).max()
        ep = np.abs(out["p"][0, k] - ps[k]).max() / np.abs(ps[k]).max()
        eK = np.abs(out["K"][0, k] - Ks[k]).max() / np.abs(Ks[k]).max() if k < N else 0.0
        print(k, "P %.2e p %.2e K %.2e" % (eP, ep, eK))
    if mode == 0:
        ref = __import__("oracle").solve(qp, dict(ric_alg=0), x0=x0) if False else None
