"""Dev aid: the Speed-mode endgame of the degenerate family (tests/test_gpu_ipm.py
test_degenerate_endgame_family) with the linear residual of every unrefined step.
Run with SRBD_QP_LIB=build/variants/checkonly/libsrbd_qp.so (-DSRBD_ITREF_CHECK_ONLY=1):
mode Balance then checks each step (stat columns 14 / 15) and never corrects, i.e. the
iterates are Speed's.  Writes one JSON: per QP status, iter and per-iteration rows
(alpha_p, alpha_d, mu, res_stat, res_eq, lin_res_stat, lin_res_eq)."""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO))
import helpers  # noqa: E402
import __graft_entry__ as g  # noqa: E402

pkg = g._import_pkg()
qp, x0 = helpers.random_constrained(20, 12, 12, 4, 14, 200, pkg.OcpQpBatch)
M = int(sys.argv[2]) if len(sys.argv) > 2 else 64
rng = np.random.default_rng(7)
fields = {}
for name in ("Q", "R", "S", "A", "B", "q", "r", "b", "C", "D", "lg", "ug", "lbu", "ubu", "lbx", "ubx",
             "lg_mask", "ug_mask", "lbu_mask", "ubu_mask", "lbx_mask", "ubx_mask"):
    a = getattr(qp, name, None)
    if a is None:
        continue
    a = np.repeat(np.asarray(a)[12:13], M, axis=0)
    if name in ("Q", "R", "S", "A", "B", "q", "r", "b"):
        a = a * (1 + 1e-15 * rng.standard_normal(a.shape))
    fields[name] = a
fam = pkg.OcpQpBatch(N=qp.N, nx=qp.nx, nu=qp.nu, ng=qp.ng, **fields)
xb = np.repeat(np.asarray(x0)[12:13], M, axis=0)
res = {}
ras = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1]
for ra in ras:
    out = pkg.capi.solve(fam, xb, dict(iter_max=50, mode="Balance", ric_alg=ra), stats=True)
    rows = []
    for i in range(M):
        it = int(out["iter"][i])
        S = out["stat"][i]
        rows.append({"status": int(out["status"][i]), "iter": it,
                     "trace": S[1:it + 1][:, [3, 4, 5, 6, 7, 14, 15]].tolist()})
    res[f"ric_alg{ra}"] = rows
    print(f"ric_alg {ra}: converged {(out['status'] == 0).sum()}/{M}", flush=True)
Path(sys.argv[1]).write_text(json.dumps(res))
