"""Dev aid: per-iteration stats of one QP of the (12,4,14) general-constraint
test batch on the GPU next to the oracle's result."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
sys.path.insert(0, "oracle")
import oracle
np.set_printoptions(linewidth=200, precision=4)
qp, x0 = helpers.random_constrained(20, 12, 12, 4, 14, 200, pkg.OcpQpBatch)
st = dict(iter_max=50, mode="Balance")
out = pkg.capi.solve(qp, x0, st, stats=True)
ref = oracle.solve(qp, st, x0=x0)
print("gpu status", out["status"], "\niter", out["iter"], "\noracle iter", ref["iter"])
for i in np.nonzero(out["status"] != 0)[0]:
    it = out["iter"][i]
    print("QP", i, "res", out["res"][i], "oracle res", ref["res"][i])
    print(out["stat"][i, :it + 2, :11])
