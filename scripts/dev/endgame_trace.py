"""Dev aid: GPU vs oracle iterates after k IPM iterations (iter_max = k) for the QPs the
GPU leaves unsolved at tol 1e-8 while the oracle solves them (degenerate general rows)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "."); sys.path.insert(0, "oracle")
import numpy as np
import helpers
pkg = helpers.load_package()
import oracle
np.set_printoptions(linewidth=220, precision=3)
ric = int(sys.argv[1]) if len(sys.argv) > 1 else 0
N, nx, nu, ng, seed = 8, 12, 12, 40, 200
qp, x0 = helpers.random_constrained(100, N, nx, nu, ng, seed, pkg.OcpQpBatch)
st = dict(iter_max=50, mode="Balance", ric_alg=ric)
g = pkg.capi.solve(qp, x0, st, stats=True)
o = oracle.solve(qp, st, x0=x0, riccati=False)
sel = np.nonzero((g["status"] != 0) & (o["status"] == 0))[0][:3]
print("gpu-only failures", np.nonzero((g["status"] != 0) & (o["status"] == 0))[0])
sub = qp.subset(sel)
xs = x0[sel]
for k in range(1, 16):
    stk = dict(st, iter_max=k)
    gk = pkg.capi.solve(sub, xs, stk)
    ok = oracle.solve(sub, stk, x0=xs, riccati=False)
    line = []
    for key in ("x", "u", "pi"):
        d = np.abs(gk[key] - ok[key]).reshape(len(sel), -1).max(1) / np.abs(ok[key]).reshape(len(sel), -1).max(1)
        line.append(f"{key} {d}")
    print(k, " | ".join(line), "res_stat g", gk["res"][:, 0], "o", ok["res"][:, 0])
