"""Dev aid: the IPM step of iteration k (iterate after k+1 minus after k iterations), GPU vs
oracle, per stage, for one QP of the (8,12,12,40) family (seed 200)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "."); sys.path.insert(0, "oracle")
import numpy as np
import helpers
pkg = helpers.load_package()
import oracle
np.set_printoptions(linewidth=220, precision=3)
ric, i, k = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
qp, x0 = helpers.random_constrained(100, 8, 12, 12, 40, 200, pkg.OcpQpBatch)
sub = qp.subset(slice(i, i + 1)); xs = x0[i:i + 1]
st = dict(mode="Balance", ric_alg=ric, tol_stat=1e-30, tol_eq=1e-30, tol_ineq=1e-30, tol_comp=1e-30)
G = [pkg.capi.solve(sub, xs, dict(st, iter_max=j)) for j in (k, k + 1)]
O = [oracle.solve(sub, dict(st, iter_max=j), x0=xs, riccati=False) for j in (k, k + 1)]
for key in ("x", "u", "pi"):
    dg = G[1][key][0] - G[0][key][0]
    do = O[1][key][0] - O[0][key][0]
    print(key, "iterate diff at k:", np.abs(G[0][key][0] - O[0][key][0]).max())
    print("  |step| per stage  ", np.abs(do).max(1))
    print("  |step err| p.stage", np.abs(dg - do).max(1))
print("res g", G[1]["res"][0], "o", O[1]["res"][0])
