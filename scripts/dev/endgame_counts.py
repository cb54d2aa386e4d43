"""Dev aid: Speed-mode convergence counts on the degenerate endgame family
(tests/test_gpu_ipm.py test_degenerate_endgame_family) for the library in SRBD_QP_LIB (or the
product).  Usage: endgame_counts.py RIC_ALGS [MODE]   e.g. endgame_counts.py 0,1 Speed"""
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
M = 64
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
mode = sys.argv[2] if len(sys.argv) > 2 else "Speed"
for ra in [int(v) for v in sys.argv[1].split(",")]:
    out = pkg.capi.solve(fam, xb, dict(iter_max=50, mode=mode, ric_alg=ra))
    st = out["status"]
    worst = 0.0
    if len(sys.argv) > 3:  # distance of every copy to the oracle's solution (converged copies)
        sys.path.insert(0, str(REPO / "oracle"))
        ref = helpers.load_oracle().solve(fam, dict(iter_max=50, mode=mode, ric_alg=ra), x0=xb)
        for i in range(M):
            if ref["status"][i] == 0:
                for key in ("x", "u"):
                    d = np.linalg.norm(out[key][i] - ref[key][i]) / np.linalg.norm(ref[key][i])
                    worst = max(worst, d)
    print(f"{mode} ric_alg {ra}: converged {(st == 0).sum()}/{M}, statuses {np.bincount(st, minlength=4).tolist()}, "
          f"iters {np.bincount(out['iter'][st == 0]).nonzero()[0].tolist()}, worst rel dist to oracle {worst:.1e}", flush=True)
