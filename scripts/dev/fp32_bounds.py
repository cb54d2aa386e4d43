"""Dev aid: success rate and distance to the fp64 solution of the fp32 IPM on the cases of
tests/test_gpu_fp32.py (to state their bounds at what is achieved)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import helpers
pkg = helpers.load_package()
NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)
F32 = dict(iter_max=30, tol_stat=1e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1)
for (B, N, seed, tol, cons) in [(64, 20, 93, 1e-2, "cone"), (256, 40, 93, 3e-2, "cone"),
                                (512, 40, 1005, 3e-2, "cone"), (4096, 40, 7, 3e-2, "cone"),
                                (64, 20, 92, 1e-4, "box_u")]:
    qp, x0 = pkg.srbd_model.generate_batch(B, N=N, seed=seed, constraints=cons)
    st = dict(F32, tol_stat=tol) if cons == "cone" else NMPC
    o32 = pkg.capi.solve(qp, x0, st, dtype=np.float32)
    o64 = pkg.capi.solve(qp, x0, NMPC)
    ok = o32["status"] == 0
    ru = np.array([np.linalg.norm(o32["u"][i] - o64["u"][i]) / np.linalg.norm(o64["u"][i])
                   for i in np.nonzero(ok)[0]])
    rx = np.array([np.linalg.norm(o32["x"][i] - o64["x"][i]) / np.linalg.norm(o64["x"][i])
                   for i in np.nonzero(ok)[0]])
    print(f"{cons} B={B} N={N} seed={seed}: success {ok.mean():.4f} status {np.bincount(o32['status'])} "
          f"iters mean {o32['iter'].mean():.2f} | ru median {np.median(ru):.2e} p99 {np.quantile(ru, .99):.2e} "
          f"max {ru.max():.2e} | rx median {np.median(rx):.2e} max {rx.max():.2e}", flush=True)
