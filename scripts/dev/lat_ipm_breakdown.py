"""Dev aid (GPU, -DSRBD_TSTAMP=1 build of ipm_latency.hip via SRBD_QP_LIB): where a batch-1 solve
of the latency IPM goes, per phase (cycle-counter stamps of lane 0 of workgroup 0 after each
phase's barrier), summed over the iterations.
  SRBD_QP_LIB=build/variants/tstamp/libsrbd_qp.so python scripts/dev/lat_ipm_breakdown.py [box_u|cone]"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import helpers  # noqa: E402

cons = sys.argv[1] if len(sys.argv) > 1 else "box_u"
pkg = helpers.load_package()
L = pkg.capi.lib()
L.srbd_qp_diag_tstamps_lat.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
L.srbd_qp_diag_tstamps_lat.restype = C.c_int
qp, x0 = pkg.srbd_model.generate_batch(1, N=20, seed=11, constraints=cons)
st = dict(mode="Speed", iter_max=30, ric_alg=0, split_step=1, tol_stat=1e-4, tol_eq=1e-4,
          tol_ineq=1e-4, tol_comp=1e-4)
buf = (C.c_ulonglong * 8192)()
names = {63: "start", 64: "init", 50: "iter top", 51: "stage pass (step, residuals, predictor blocks)",
         53: "factorize", 54: "forward (pred)", 55: "step pass (pred)", 56: "corrector gradient",
         57: "corr rhs stages", 58: "corr rhs chain", 59: "corr k stages", 60: "forward (corr)",
         61: "step pass (corr)", 65: "after loop", 66: "outputs",
         70: "fact: barrier / stage top", 71: "fact: operands, G = R~ + B'PB, G to columns",
         72: "fact: chol(G) (+ W, H, F MFMAs)", 73: "fact: Y = L^-1 [H | g]",
         75: "fact: P = F - Y'Y, symmetrize"}
tot = {}
for rep in range(3):
    L.srbd_qp_diag_tstamps_lat(buf, 4096)
    out = pkg.capi.solve(qp, x0, st)
    n = L.srbd_qp_diag_tstamps_lat(buf, 4096)
    a = np.array(buf[:2 * n], dtype=np.uint64).reshape(-1, 2)
    if rep == 0:
        continue
    for (i0, t0), (i1, t1) in zip(a[:-1], a[1:]):
        tot.setdefault(names.get(int(i1), str(i1)), []).append(int(t1) - int(t0))
total = sum(sum(v) for v in tot.values()) / 2
print(json.dumps({"iters": int(out["iter"][0]), "total_cycles": total,
                  "phases": {k: {"cycles_per_solve": sum(v) / 2, "share": sum(v) / 2 / total}
                             for k, v in sorted(tot.items(), key=lambda kv: -sum(kv[1]))}}, indent=1))
