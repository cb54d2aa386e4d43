"""Dev aid: which C-free QP families make HPIPM's lq_fact 1 check switch to the LQ
factorization (ric_alg 1), on the batched kernels and on the latency IPM."""
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
import helpers  # noqa: E402

pkg = helpers.load_package()


def perturbed(qp, x0, i, M, seed=7, drop_c=False):
    rng = np.random.default_rng(seed)
    fields = {}
    for name in ("Q", "R", "S", "A", "B", "q", "r", "b", "C", "D", "lg", "ug", "lbu", "ubu", "lbx",
                 "ubx", "lg_mask", "ug_mask", "lbu_mask", "ubu_mask", "lbx_mask", "ubx_mask"):
        a = getattr(qp, name, None)
        if a is None or (drop_c and name == "C"):
            continue
        a = np.repeat(np.asarray(a)[i:i + 1], M, axis=0)
        if name in ("Q", "R", "S", "A", "B", "q", "r", "b"):
            a = a * (1 + 1e-15 * rng.standard_normal(a.shape))
        fields[name] = a
    fam = pkg.OcpQpBatch(N=qp.N, nx=qp.nx, nu=qp.nu, ng=qp.ng, **fields)
    return fam, np.repeat(np.asarray(x0)[i:i + 1], M, axis=0)


def run(name, qp, x0, st):
    out = {"name": name}
    for path, mx in (("lat", "512"), ("bat", "0")):
        os.environ["SRBD_IPM_LATENCY_MAX"] = mx
        r = pkg.capi.solve(qp, x0, st, stats=True)
        out[path] = {"switched": int(np.any(r["stat"][:, :, 11] == 1.0, axis=1).sum()),
                     "status": np.bincount(r["status"], minlength=5).tolist(),
                     "iter_mean": float(r["iter"].mean())}
    print(json.dumps(out), flush=True)


for mode in ("Speed", "Balance"):
    st = dict(iter_max=50, mode=mode, ric_alg=1, lq_fact=1)
    qp, x0 = helpers.random_constrained(20, 12, 12, 4, 14, 200, pkg.OcpQpBatch)
    run(f"{mode} endgame family, C dropped", *perturbed(qp, x0, 12, 64, drop_c=True), st)
    for ng in (0, 14):
        for dims in ((12, 12), (12, 4), (5, 3)):
            for seed in (200, 31, 141):
                qp, x0 = helpers.random_constrained(64, 15, dims[0], dims[1], ng, seed + dims[0] + ng,
                                                    pkg.OcpQpBatch)
                if ng:
                    qp.C = None
                run(f"{mode} random ng={ng} dims={dims} seed={seed}", qp, x0, st)
    for cons in ("box_u", "cone"):
        for seed in (3, 11, 23):
            qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=seed, constraints=cons)
            run(f"{mode} srbd {cons} seed={seed}", qp, x0, st)
