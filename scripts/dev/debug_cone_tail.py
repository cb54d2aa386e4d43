"""Dev aid: which fp32 friction-cone QPs (config 5) fail, and why (status, residual
trajectory, magnitudes), against fp64 on the same QPs."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
np.set_printoptions(linewidth=220, precision=3)
F32 = dict(iter_max=30, tol_stat=3e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1,
           ric_alg=int(sys.argv[1]) if len(sys.argv) > 1 else 0)
N = 40
qp, x0 = pkg.srbd_model.generate_batch(2048, N=N, seed=1005, constraints="cone")
o = pkg.capi.solve(qp, x0, F32, dtype=np.float32, stats=True)
st = o["status"]
print("fp32 status counts", np.bincount(st, minlength=4), "iters hist", np.bincount(o["iter"]))
o64 = pkg.capi.solve(qp, x0, F32, dtype=np.float64, stats=True)
print("fp64 status counts", np.bincount(o64["status"], minlength=4), "iters hist", np.bincount(o64["iter"]))
bad = np.nonzero(st != 0)[0]
good = np.nonzero(st == 0)[0]
print("fail res (stat, eq, ineq, comp) median", np.median(o["res"][bad], 0), "max", o["res"][bad].max(0))
print("ok   res median", np.median(o["res"][good], 0))
u = o64["u"]
umax = np.abs(u).reshape(len(u), -1).max(1)
Rmax = np.abs(qp.R).reshape(qp.batch, -1).max(1)
print("|u|max  fail median %.3g ok median %.3g" % (np.median(umax[bad]), np.median(umax[good])))
print("|R|max  fail median %.3g ok median %.3g" % (np.median(Rmax[bad]), np.median(Rmax[good])))
print("|R||u|  fail median %.3g ok median %.3g" % (np.median((Rmax * umax)[bad]), np.median((Rmax * umax)[good])))
for i in bad[:4]:
    s = o["stat"][i]
    n = o["iter"][i] + 1
    print("QP", i, "status", st[i], "iters", o["iter"][i], "fp64 iters", o64["iter"][i], "status64", o64["status"][i])
    print("  alpha_p", s[1:n, 3])
    print("  alpha_d", s[1:n, 4])
    print("  mu     ", s[:n, 5])
    print("  res_st ", s[:n, 6])
    print("  res_eq ", s[:n, 7])
    print("  res_in ", s[:n, 8])
    print("  res_co ", s[:n, 9])
    s6 = o64["stat"][i]
    n6 = o64["iter"][i] + 1
    print("  f64 res_st ", s6[:n6, 6])
    print("  f64 mu     ", s6[:n6, 5])
    du = np.abs(o["u"][i] - o64["u"][i]).max()
    print("  |u32-u64|max %.3g  |u64|max %.3g" % (du, np.abs(o64["u"][i]).max()))
