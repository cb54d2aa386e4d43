"""Dev aid (GPU): the measured values behind the loose parity bounds VERDICT r02 named,
so the tests can be tightened to them.  Prints one JSON object."""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "oracle"))
import helpers  # noqa: E402

pkg = helpers.load_package()
oracle = helpers.load_oracle()
NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)
F32 = dict(iter_max=30, tol_stat=1e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1)
out = {}


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


# test_box_u_fp32_vs_fp64
qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=92, constraints="box_u")
o32 = pkg.capi.solve(qp, x0, NMPC, dtype=np.float32)
o64 = pkg.capi.solve(qp, x0, NMPC)
ok = o32["status"] == 0
out["box_u_fp32"] = {"success": int(ok.sum()), "of": len(ok),
                     "u_max": max(rel(o32["u"][i].astype(float), o64["u"][i]) for i in np.nonzero(ok)[0]),
                     "x_max": max(rel(o32["x"][i].astype(float), o64["x"][i]) for i in np.nonzero(ok)[0])}
# test_friction_cone_fp32_vs_oracle
qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=93, constraints="cone")
o32 = pkg.capi.solve(qp, x0, F32, dtype=np.float32)
ok = o32["status"] == 0
out["cone_fp32_n20"] = {"success": int(ok.sum()), "of": len(ok), "status": np.bincount(o32["status"]).tolist()}
# test_f64_rescue_cone_n40
for cap, batch in ((30, 512), (12, 512), (12, 2500)):
    qp, x0 = pkg.srbd_model.generate_batch(batch, N=40, seed=1005, constraints="cone")
    st = dict(F32, tol_stat=3e-2)
    plain = pkg.capi.solve(qp, x0, dict(st, iter_max=cap), dtype=np.float32)
    resc = pkg.capi.solve(qp, x0, dict(st, f64_rescue=cap), dtype=np.float32)
    o64 = pkg.capi.solve(qp, x0, NMPC)
    bad = plain["status"] != 0
    ru = [rel(resc["u"][i].astype(float), o64["u"][i]) for i in np.nonzero(bad)[0]]
    out[f"rescue_cap{cap}_b{batch}"] = {"rescued": int(bad.sum()), "ru_median": float(np.median(ru)),
                                        "ru_p90": float(np.quantile(ru, 0.9)), "ru_max": float(np.max(ru)),
                                        "resc_status": np.bincount(resc["status"]).tolist()}
# test_constrained_vs_oracle: pi0 in stationarity form, GPU vs the oracle's own solution
for ric_alg in (0, 1):
    for nx, nu in ((5, 3), (12, 12), (12, 4)):
        qp, x0 = helpers.random_constrained(24, 15, nx, nu, 0, 17 + nx, pkg.OcpQpBatch)
        st = dict(iter_max=40, mode="Balance", ric_alg=ric_alg)
        o = pkg.capi.solve(qp, x0, st, riccati=True)
        r = oracle.solve(qp, st, x0=x0)
        e0, e1, el = [], [], []
        for i in range(qp.batch):
            def pi0(s):
                A0, B0, b0 = qp.A[i, 0], qp.B[i, 0], qp.b[i, 0]
                rb0 = A0 @ x0[i] + B0 @ s["u"][i, 0] + b0 - s["x"][i, 1]
                return (qp.Q[i, 0] @ x0[i] + qp.S[i, 0].T @ s["u"][i, 0] + qp.q[i, 0]
                        + A0.T @ (s["pi"][i, 1] + s["P"][i, 1] @ rb0))
            e0.append(rel(pi0(o), pi0(r)))
            el.append(rel(o["pi"][i, 0], r["pi"][i, 0]))
            e1.append(rel(o["pi"][i, 1:], r["pi"][i, 1:]))
        out[f"pi0_ric{ric_alg}_{nx}x{nu}"] = {"stat_form_max": max(e0), "literal_max": max(el),
                                              "pi_rest_max": max(e1), "has_P": "P" in r}
print(json.dumps(out, indent=1))
