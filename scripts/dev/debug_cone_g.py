"""Dev aid: fp32 friction cone (config 5 settings) with the fp64 stage factorization --
status / iteration histograms of the plain fp32 solve and of the f64 rescue, and the
trajectories of QPs the rescue leaves unsolved."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
np.set_printoptions(linewidth=220, precision=3)
F32 = dict(iter_max=30, tol_stat=3e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1)
NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
qp, x0 = pkg.srbd_model.generate_batch(B, N=40, seed=1005, constraints="cone")
o = pkg.capi.solve(qp, x0, F32, dtype=np.float32, stats=True)
print("fp32 status", np.bincount(o["status"], minlength=4), "iters", np.bincount(o["iter"]))
r = pkg.capi.solve(qp, x0, dict(F32, f64_rescue=30), dtype=np.float32, stats=True)
bad = np.nonzero(o["status"] != 0)[0]
print("rescue status", np.bincount(r["status"], minlength=4), "rescued iters", r["iter"][bad])
o64 = pkg.capi.solve(qp, x0, NMPC, stats=True)
print("fp64 status", np.bincount(o64["status"], minlength=4))
for i in np.nonzero(r["status"] != 0)[0][:3]:
    s = o["stat"][i]
    n = o["iter"][i] + 1
    print("QP", i, "fp32 status", o["status"][i], "it", o["iter"][i], "| rescue status", r["status"][i],
          "it", r["iter"][i], "res", r["res"][i], "| fp64 it", o64["iter"][i])
    print("  fp32 alpha_p", s[1:n, 3])
    print("  fp32 mu     ", s[:n, 5])
    print("  fp32 res_st ", s[:n, 6])
    print("  fp32 res_co ", s[:n, 9])
    s = r["stat"][i]
    n = r["iter"][i] + 1
    print("  f64c alpha_p", s[1:n, 3])
    print("  f64c mu     ", s[:n, 5])
    print("  f64c res_st ", s[:n, 6])
    print("  f64c res_eq ", s[:n, 7])
    print("  f64c res_co ", s[:n, 9])
