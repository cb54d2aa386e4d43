"""The reference's NMPC step (NMPCSolver::controlLoop's SQP loop, NMPC_solver.cpp:
362-372 -- BASELINE config 1) for a batch of robots on the device
(srbd_qp_srbd_nmpc_f64: linearise -> QP solve -> filter line search, until the line
search reports convergence or sqp_max_loop iterations), against the same loop run
on the host (numpy model -> C oracle QP -> numpy line search, oracle/nmpc_linesearch.py)."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import nmpc_linesearch as LS  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu

# NMPC_solver.cpp:70-82 (the reference QP is unconstrained: one Riccati solve)
NMPC = dict(mode="Speed", iter_max=30, alpha_min=1e-8, mu0=1e2, tol_stat=1e-4, tol_eq=1e-4,
            tol_ineq=1e-4, tol_comp=1e-4, reg_prim=1e-12, warm_start=0, pred_corr=1, ric_alg=0,
            split_step=1)
SQP_MAX_LOOP = 15  # config/mpc_option.yaml sqp_max_loop


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def reference_start(N):
    """NMPCSolver::initialize / setupReference (NMPC_solver.cpp:56-64, 341-350):
    x_nmpc = 0, u_nmpc = 100, x0 = (0, .., 0, z = 1.0, 0, 0, 0), alpha_ = 1."""
    xs = np.zeros((N + 1, 12))
    us = np.full((N, 12), 100.0)
    x0 = np.zeros(12)
    x0[8] = 1.0
    return xs, us, x0, 1.0


def run_both(pkg, oracle, xs, us, x0, alpha, constraints="none"):
    B, N = us.shape[0], us.shape[1]
    p = pkg.srbd_model.SrbdParams()
    ng = 24 if constraints == "cone" else 0
    h = pkg.capi.Handle(N, 12, 12, ng, constraints == "box_u", False, capacity=B)
    xs_t, us_t, x0_t, al_t = _dev(xs), _dev(us), _dev(x0), _dev(alpha)
    it_t, cv_t = pkg.capi.srbd_nmpc(h, xs_t, us_t, x0_t, al_t, constraints, NMPC, SQP_MAX_LOOP)
    dev = dict(xs=xs_t.cpu().numpy(), us=us_t.cpu().numpy(), alpha=al_t.cpu().numpy(),
               it=it_t.cpu().numpy(), conv=cv_t.cpu().numpy())
    host = [LS.sqp_loop(pkg.srbd_model, oracle, p, xs[i], us[i], x0[i], float(alpha[i]), NMPC,
                        SQP_MAX_LOOP, constraints) for i in range(B)]
    return dev, host


def check(dev, host):
    for i, (hx, hu, ha, hit, hcv) in enumerate(host):
        assert dev["it"][i] == hit, (i, dev["it"][i], hit)
        assert bool(dev["conv"][i]) == hcv, i
        assert dev["alpha"][i] == ha, (i, dev["alpha"][i], ha)
        np.testing.assert_allclose(dev["xs"][i], hx, rtol=1e-7, atol=1e-9, err_msg=str(i))
        np.testing.assert_allclose(dev["us"][i], hu, rtol=1e-7, atol=1e-6, err_msg=str(i))


def test_reference_nmpc_step(pkg, oracle):
    """Config 1 exactly as the reference runs it (one robot from its own start)."""
    N = 20
    xs, us, x0, a0 = reference_start(N)
    dev, host = run_both(pkg, oracle, xs[None], us[None], x0[None], np.array([a0]))
    check(dev, host)
    assert dev["it"][0] >= 2  # the cold start needs several SQP iterations


def test_batched_nmpc_steps(pkg, oracle):
    """A batch of robots from perturbed starts (different SQP iteration counts, some
    hitting sqp_max_loop): every robot stops where its own loop stops."""
    B, N = 24, 20
    p = pkg.srbd_model.SrbdParams()
    xs, us, dx0 = pkg.srbd_model.sample_trajectories(B, N, 4711, p)
    x0 = xs[:, 0] + dx0
    ref = reference_start(N)
    xs[:4], us[:4], x0[:4] = ref[0], ref[1], ref[2]  # the reference's own start too
    alpha = np.where(np.arange(B) % 4 == 1, 0.5, 1.0)
    dev, host = run_both(pkg, oracle, xs, us, x0, alpha)
    check(dev, host)
    assert len(set(int(v) for v in dev["it"])) > 1
