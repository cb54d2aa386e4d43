"""Dev aid: GPU stat rows of one QP (8,12,12,40 family, seed 200) next to nothing else;
compare with the oracle's ORACLE_DEBUG trace printed on the host."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
np.set_printoptions(linewidth=220, precision=6)
ric = int(sys.argv[1]); i = int(sys.argv[2])
qp, x0 = helpers.random_constrained(100, 8, 12, 12, 40, 200, pkg.OcpQpBatch)
sub = qp.subset(slice(i, i + 1))
g = pkg.capi.solve(sub, x0[i:i + 1], dict(iter_max=14, mode="Balance", ric_alg=ric), stats=True)
print("it alpha_aff mu_aff sigma alpha_p alpha_d mu res_stat res_eq res_ineq res_comp")
for r in range(15):
    print(r, g["stat"][0, r, :10])
