"""Dev aid: how often does the IPM endgame stall above tol 1e-8 on the degenerate
general-row family of test_gpu_ipm.py (nu = 4, ng = 14: more rows than inputs)?
GPU and oracle, both Riccati variants.  Usage: endgame_stats.py [gpu|oracle]"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "."); sys.path.insert(0, "oracle")
import numpy as np
import helpers
pkg = helpers.load_package()
import oracle
which = sys.argv[1] if len(sys.argv) > 1 else "gpu"
for dims in [(12, 12, 4, 14), (12, 6, 3, 24), (8, 12, 12, 40)]:
    N, nx, nu, ng = dims
    for ric in (0, 1):
        bad = 0; tot = 0; its = []
        for seed in range(200, 205):
            qp, x0 = helpers.random_constrained(100, N, nx, nu, ng, seed, pkg.OcpQpBatch)
            st = dict(iter_max=50, mode="Balance", ric_alg=ric)
            out = pkg.capi.solve(qp, x0, st) if which == "gpu" else oracle.solve(qp, st, x0=x0, riccati=False)
            bad += int((out["status"] != 0).sum()); tot += qp.batch
            its.append(out["iter"].mean())
        print(which, dims, "ric_alg", ric, "unsolved", bad, "/", tot, "mean iter %.2f" % np.mean(its), flush=True)
