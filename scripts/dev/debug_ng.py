"""Dev aid: per-iteration stats of one QP of the (12,4,14) general-constraint
test batch on the GPU next to the oracle's result.  Usage: debug_ng.py [ric_alg] [qp]"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
sys.path.insert(0, "oracle")
import oracle
np.set_printoptions(linewidth=200, precision=4)
ric = int(sys.argv[1]) if len(sys.argv) > 1 else 1
show = int(sys.argv[2]) if len(sys.argv) > 2 else 12
qp, x0 = helpers.random_constrained(20, 12, 12, 4, 14, 200, pkg.OcpQpBatch)
st = dict(iter_max=50, mode="Balance", ric_alg=ric)
out = pkg.capi.solve(qp, x0, st, stats=True)
ref = oracle.solve(qp, st, x0=x0)
print("ric_alg", ric, "gpu status", out["status"], "\niter", out["iter"], "\noracle iter", ref["iter"])
for i in sorted(set(np.nonzero(out["status"] != 0)[0]) | {show}):
    it = min(int(out["iter"][i]), 20)
    print("QP", i, "res", out["res"][i], "oracle res", ref["res"][i])
    print(" it  alpha_aff mu_aff sigma alpha_p alpha_d mu res_stat res_eq res_ineq res_comp")
    for r in range(it + 1):
        print(r, out["stat"][i, r, :10])
