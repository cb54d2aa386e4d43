"""Dev aid: C = 0 against C = None (the same QP) on both IPM paths, square-root Riccati: which
path's C instantiation leaves the C-free one (first-iteration stat rows)."""
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests"))
import helpers  # noqa: E402

pkg = helpers.load_package()
oracle = helpers.load_oracle()
np.set_printoptions(linewidth=220, precision=4)
qp0, x0 = helpers.random_constrained(12, 15, 12, 12, 14, 167, pkg.OcpQpBatch)
qz = qp0.subset(np.arange(12)); qz.C = np.zeros_like(np.asarray(qz.C))
qn = qp0.subset(np.arange(12)); qn.C = None
for ric in (1, 0):
    st = dict(iter_max=40, mode="Speed", ric_alg=ric)
    out = {}
    for path, mx in (("lat", "512"), ("bat", "0")):
        os.environ["SRBD_IPM_LATENCY_MAX"] = mx
        for cname, q in (("Czero", qz), ("Cnone", qn)):
            out[path, cname] = pkg.capi.solve(q, x0, st, stats=True)
    ref_z = oracle.solve(qz, st, x0=x0)
    ref_n = oracle.solve(qn, st, x0=x0)
    print(f"ric_alg {ric}: oracle iter Czero {ref_z['iter']} Cnone {ref_n['iter']}")
    for k, r in out.items():
        print(f"  {k}: iter {r['iter']}")
    for a, b in ((("lat", "Czero"), ("lat", "Cnone")), (("bat", "Czero"), ("bat", "Cnone")),
                 (("lat", "Cnone"), ("bat", "Cnone"))):
        x, y = out[a]["stat"][:, 1, :10], out[b]["stat"][:, 1, :10]
        rel = np.abs(x - y) / np.maximum(np.abs(y), 1e-300)
        print(f"  it1 {a} vs {b}: max rel per column {rel.max(axis=0)}")
