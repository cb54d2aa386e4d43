"""Dev aid: which fp32 friction-cone QPs end with status 3 (NaN), and their IPM trace."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
np.set_printoptions(linewidth=250, precision=3)
F32 = dict(iter_max=30, tol_stat=3e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1)
qp, x0 = pkg.srbd_model.generate_batch(256, N=40, seed=93, constraints="cone")
o = pkg.capi.solve(qp, x0, F32, dtype=np.float32, stats=True)
print("status counts", np.bincount(o["status"]))
for i in np.nonzero(o["status"] == 3)[0][:3]:
    print("QP", i, "iter", o["iter"][i])
    st = o["stat"][i]
    for r in range(min(len(st), o["iter"][i] + 2)):
        print(r, st[r][:11])
