"""Dev aid: per-iteration trace of the mixed-precision IPM (f32_iters) against fp64."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import helpers
import bench
pkg = helpers.load_package()
np.set_printoptions(linewidth=200, precision=2)
qp, x0 = pkg.srbd_model.generate_batch(256, N=20, seed=5, constraints="box_u")
NMPC = dict(bench.NMPC_SETTINGS)
k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
o64 = pkg.capi.solve(qp, x0, NMPC, stats=True)
f32 = pkg.capi.solve(qp, x0, dict(NMPC, iter_max=k, tol_stat=1e-30, tol_eq=1e-30, tol_ineq=1e-30,
                                  tol_comp=1e-30), stats=True, dtype=np.float32)
mix = pkg.capi.solve(qp, x0, dict(NMPC, f32_iters=k), stats=True)
print("iters fp64", np.bincount(o64["iter"]), "mixed", np.bincount(mix["iter"]))
for i in range(3):
    for name, o in (("fp64", o64), ("fp32", f32), ("mixed", mix)):
        s = o["stat"][i]
        n = o["iter"][i] + 1
        print(name, i, "alpha_p", s[1:n, 3], "\n   mu", s[:n, 5], "\n   res_st", s[:n, 6], "\n   res_eq", s[:n, 7],
              "\n   res_co", s[:n, 9])
