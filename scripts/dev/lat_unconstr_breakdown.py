"""Dev aid (GPU, -DSRBD_TSTAMP=1 build via SRBD_QP_LIB): where the one-QP unconstrained solve
(the reference's call pattern: N = 20, residuals fused) goes, per phase (cycle-counter stamps
of lane 0 of workgroup 0), on device buffers.
  make variant NAME=tstamp VFLAGS=-DSRBD_TSTAMP=1
  SRBD_QP_LIB=build/variants/tstamp/libsrbd_qp.so python scripts/dev/lat_unconstr_breakdown.py"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import helpers  # noqa: E402

pkg = helpers.load_package()
L = pkg.capi.lib()
L.srbd_qp_diag_tstamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
L.srbd_qp_diag_tstamps.restype = C.c_int
qp, x0 = pkg.srbd_model.generate_batch(1, N=20, seed=1003, constraints="none")
buf = (C.c_ulonglong * 8192)()
names = {16: "entry", 14: "copy issued", 15: "copy landed", 0: "stage top (barrier, record of k+1)",
         1: "operands, WB = P B, G = R + B'WB", 3: "G to columns, chol(G) (+ W, H, F MFMAs)",
         7: "H to columns, Y = L^-1 [H | g]", 9: "hand-over, P = F - Y'Y", 12: "last stage -> sweep done",
         13: "forward sweep", 17: "u, pi (every stage)", 18: "residual pass"}
tot = {}
reps = 5
for rep in range(reps + 1):
    L.srbd_qp_diag_tstamps(buf, 4096)
    out = pkg.capi.solve(qp, x0, dict(ric_alg=0), riccati=True, stats=True)
    n = L.srbd_qp_diag_tstamps(buf, 4096)
    a = np.array(buf[:2 * n], dtype=np.uint64).reshape(-1, 2)
    if rep == 0:
        continue
    for (i0, t0), (i1, t1) in zip(a[:-1], a[1:]):
        key = names.get(int(i1), str(int(i1)))
        if int(i1) == 0 and int(i0) == 15:
            key = "first stage top"
        tot.setdefault(key, []).append(int(t1) - int(t0))
total = sum(sum(v) for v in tot.values()) / reps
print(json.dumps({"total_cycles": total, "phases": {k: {"cycles": sum(v) / reps, "n": len(v) // reps}
                                                    for k, v in tot.items()}}, indent=1))
