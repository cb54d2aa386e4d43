"""Dev aid: fp32 cone N=40 success rate vs reg_prim / tolerances."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
qp, x0 = pkg.srbd_model.generate_batch(2048, N=40, seed=5, constraints="cone")
for reg in (1e-12, 1e-8, 1e-6, 1e-4):
    for ts in (1e-2, 3e-2):
        st = dict(iter_max=30, tol_stat=ts, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1, reg_prim=reg)
        o = pkg.capi.solve(qp, x0, st, dtype=np.float32)
        print(f"reg {reg:g} tol_stat {ts:g}: success {(o['status'] == 0).mean():.3f} counts {np.bincount(o['status'], minlength=4)} iters mean {o['iter'].mean():.1f}")
o = pkg.capi.solve(qp, x0, dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1))
print("fp64 NMPC tol: success", (o['status'] == 0).mean(), "iters", o['iter'].mean())
