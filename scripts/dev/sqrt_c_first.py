"""Dev aid: per QP, the first stat row where the square-root latency IPM with C = 0 leaves the
same QP with C = None (a -DSRBD_LAT_SQRT_C=1 build, SRBD_QP_LIB)."""
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests"))
import helpers  # noqa: E402

pkg = helpers.load_package()
np.set_printoptions(linewidth=220, precision=6)
qp0, x0 = helpers.random_constrained(12, 15, 12, 12, 14, 167, pkg.OcpQpBatch)
qz = qp0.subset(np.arange(12)); qz.C = np.zeros_like(np.asarray(qz.C))
qn = qp0.subset(np.arange(12)); qn.C = None
os.environ["SRBD_IPM_LATENCY_MAX"] = "512"
st = dict(iter_max=40, mode="Speed", ric_alg=1)
rz = pkg.capi.solve(qz, x0, st, stats=True)
rn = pkg.capi.solve(qn, x0, st, stats=True)
for i in range(12):
    a, b = rz["stat"][i], rn["stat"][i]
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    rows = np.nonzero(rel[:, :11].max(axis=1) > 1e-12)[0]
    if len(rows) == 0:
        print(f"QP {i}: identical stat, iter {rz['iter'][i]}")
        continue
    r = rows[0]
    print(f"QP {i}: first differing row {r} cols {np.nonzero(rel[r, :11] > 1e-12)[0].tolist()} iter {rz['iter'][i]} vs {rn['iter'][i]}")
    print(f"   Czero {a[r, :11]}\n   Cnone {b[r, :11]}")
    if r > 0:
        print(f"   prev  {a[r - 1, :11]}")
