"""Device filter line search (srbd_qp_srbd_linesearch_f64) against the numpy
restatement of NMPCSolver::linearSearch (oracle/nmpc_linesearch.py), and a
batched on-device SQP iteration (linearise -> QP solve -> line search, the body
of NMPCSolver::controlLoop, NMPC_solver.cpp:353-372) against the same iteration
run on the host with the oracle."""
import sys
from pathlib import Path

import numpy as np
import pytest

import helpers

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import nmpc_linesearch as LS  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_linesearch_matches_oracle(pkg):
    import torch
    B, N, seed = 24, 20, 515
    p = pkg.srbd_model.SrbdParams()
    xs, us, x0 = pkg.srbd_model.sample_trajectories(B, N, seed, p)
    rng = np.random.default_rng(3)
    dx = rng.normal(size=xs.shape) * 0.05
    du = rng.normal(size=us.shape) * 2.0
    alpha0 = np.where(np.arange(B) % 3 == 0, 0.25, 1.0)  # persistent alpha_ (NMPC_solver.h:104)
    h = pkg.capi.Handle(N, 12, 12, 0, False, False, capacity=B)
    xs_t, us_t, dx_t, du_t, al_t = _dev(xs), _dev(us), _dev(dx), _dev(du), _dev(alpha0)
    merit, conv = pkg.capi.srbd_linesearch(h, xs_t, us_t, dx_t, du_t, al_t)
    h.synchronize()
    for i in range(B):
        xn, un, an, phi, theta, dphi, cv = LS.line_search(pkg.srbd_model, p, xs[i], us[i], dx[i],
                                                          du[i], float(alpha0[i]))
        m = merit[i].cpu().numpy()
        np.testing.assert_allclose(m, [phi, theta, dphi], rtol=1e-9, atol=1e-12, err_msg=str(i))
        assert al_t[i].item() == an, (i, al_t[i].item(), an)
        assert bool(conv[i].item()) == cv
        np.testing.assert_allclose(xs_t[i].cpu().numpy(), xn, rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(us_t[i].cpu().numpy(), un, rtol=1e-13, atol=1e-13)


def test_device_sqp_iteration_matches_host(pkg, oracle):
    """Two SQP iterations of the reference's loop for a batch of robots, all on
    the device, against the host chain (numpy model -> C oracle QP -> numpy
    line search)."""
    import torch
    B, N, seed = 16, 20, 808
    p = pkg.srbd_model.SrbdParams()
    xs, us, x0s = pkg.srbd_model.sample_trajectories(B, N, seed, p)
    st = dict(iter_max=30, tol_stat=1e-10, tol_eq=1e-10, tol_ineq=1e-10, tol_comp=1e-10)
    # host chain
    hx, hu, ha = xs.copy(), us.copy(), np.ones(B)
    for it in range(2):
        qp, _ = pkg.srbd_model.build_qp(hx, hu, p, constraints="box_u")
        ref = oracle.solve(qp, st, x0=x0s - hx[:, 0])
        for i in range(B):
            hx[i], hu[i], ha[i], *_ = LS.line_search(pkg.srbd_model, p, hx[i], hu[i], ref["x"][i],
                                                     ref["u"][i], ha[i])
    # device chain
    h = pkg.capi.Handle(N, 12, 12, 0, True, False, capacity=B)
    xs_t, us_t, al_t = _dev(xs), _dev(us), _dev(np.ones(B))
    x0_t = _dev(x0s)
    f64 = dict(dtype=torch.float64, device="cuda")
    sol = {"x": torch.zeros(B, N + 1, 12, **f64), "u": torch.zeros(B, N, 12, **f64),
           "pi": torch.zeros(B, N + 1, 12, **f64)}
    S = pkg.capi.Solution(**{k: (sol[k].data_ptr() if k in sol else None) for k in pkg.capi.SOL_FIELDS})
    s = pkg.capi.settings_struct(st)
    for it in range(2):
        t, data = pkg.capi.srbd_linearize(h, xs_t, us_t, "box_u")
        dx0 = (x0_t - xs_t[:, 0]).contiguous()  # x0 - x_nmpc(:,0) (NMPC_solver.cpp:320)
        data.x0 = dx0.data_ptr()
        h.solve_device(B, s, data, S)
        pkg.capi.srbd_linesearch(h, xs_t, us_t, sol["x"], sol["u"], al_t)
        h.synchronize()
    np.testing.assert_allclose(xs_t.cpu().numpy(), hx, rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(us_t.cpu().numpy(), hu, rtol=1e-7, atol=1e-7)
    np.testing.assert_allclose(al_t.cpu().numpy(), ha)
