"""Dev aid: fp32 vs fp64 IPM on the friction-cone problem (status, iters, stats)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
np.set_printoptions(linewidth=220, precision=3)
NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)
F32 = dict(iter_max=30, tol_stat=1e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1)
for N in (20, 40):
    qp, x0 = pkg.srbd_model.generate_batch(32, N=N, seed=93, constraints="cone")
    for dt in (np.float64, np.float32):
        o = pkg.capi.solve(qp, x0, NMPC if dt is np.float64 else F32, dtype=dt, stats=True)
        print(N, dt.__name__, "status", o["status"][:12], "iters", o["iter"][:12])
        if dt is np.float32:
            print("res max", o["res"].max(0), "success", (o["status"] == 0).mean())
            qp2, x02 = pkg.srbd_model.generate_batch(2048, N=N, seed=5, constraints="cone")
            o2 = pkg.capi.solve(qp2, x02, F32, dtype=dt)
            print("2048 QPs: success", (o2["status"] == 0).mean(), "status counts", np.bincount(o2["status"]))
