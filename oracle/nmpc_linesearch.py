"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's filter line
search, the step after the QP solve in every SQP iteration:
NMPCSolver::linearSearch (NMPC_solver.cpp:149-274, constants NMPC_solver.h:97-104).

Used by tests/test_gpu_linesearch.py as the parity reference of
srbd_qp_srbd_linesearch_f64; never imported by the product path.  Per QP:

  merit at the current iterate (alpha = 0):
    theta = sum_k 0.5 |f_k|^2          (shooting defect, GetShootingDynamic)
    phi   = sum_k 0.5 (x-xr)'Q(x-xr) + sum_c b(f_c(u)) + 0.5 u'R u  (+ terminal Qf)
    dphi  = sum_k dx'Jphi_x + du'Jphi_u,  Jphi_x = Q(x-xr), Jphi_u = Ac'db + R u
  trials alpha, beta alpha, ... while alpha > alpha_min, accept on
    theta_a > theta_max:            theta_a < (1 - beta_theta) theta
    max(theta_a, theta) < theta_min and dphi < 0: Armijo phi_a < phi + eta alpha dphi
    otherwise:                      phi_a < phi - beta_phi theta  or  theta_a < (1 - beta_theta) theta
  converged: dphi > -1e-3 and theta < 1e-6.
alpha is NOT reset between calls, exactly as the reference keeps alpha_ (a member)."""
from __future__ import annotations

import math

import numpy as np

LS_DEFAULTS = dict(theta_max=1e-6, theta_min=5e-10, eta=1e-4, beta_phi=1e-6, beta_theta=1e-6,
                   beta_alpha=0.5, alpha_min=1e-4)


def _barrier_value(v, mu, th):
    if v > th:
        return -mu * math.log(v), -mu / v
    z = (v - 2.0 * th) / th
    return 0.5 * mu * (z * z - 1.0) - mu * math.log(th), mu * (v - 2.0 * th) / (th * th)


def _merit(srbd_model, p, xs, us, N, Ac, bc, with_grad):
    """(phi, theta, Jphi_x, Jphi_u) of one QP's trajectory (NMPC_solver.cpp:163-198)."""
    Qd = np.array(p.Q, dtype=np.float64)
    Qf = float(N) * np.array(p.Qf, dtype=np.float64)
    xr = np.array(p.x_ref, dtype=np.float64)
    phi = 0.0
    theta = 0.0
    Jx = np.zeros((N + 1, 12))
    Ju = np.zeros((N, 12))
    _, _, b = srbd_model.shooting_dynamics(xs[:N], xs[1:], us, p)  # b = -f per stage
    for k in range(N + 1):
        e = xs[k] - xr
        if k == N:
            phi += 0.5 * e @ (Qf * e)
            Jx[k] = Qf * e
            continue
        f = -b[k]
        theta += 0.5 * f @ f
        phi += 0.5 * e @ (Qd * e)
        Jx[k] = Qd * e
        fc = Ac @ us[k] + bc
        bsum, db = 0.0, np.zeros(24)
        for c in range(24):
            bv, db[c] = _barrier_value(fc[c], p.mu_b, p.theta_b)
            bsum += bv
        phi += bsum + 0.5 * p.R * (us[k] @ us[k])
        Ju[k] = Ac.T @ db + p.R * us[k]
    return phi, theta, Jx, Ju


def line_search(srbd_model, p, xs, us, dx, du, alpha, ls=None):
    """One QP.  Returns (xs_new, us_new, alpha_new, phi, theta, dphi, converged)."""
    ls = dict(LS_DEFAULTS, **(ls or {}))
    N = us.shape[0]
    Ac, bc = srbd_model.friction_cone(p)
    phi, theta, Jx, Ju = _merit(srbd_model, p, xs, us, N, Ac, bc, True)
    dphi = float(np.sum(dx * Jx) + np.sum(du * Ju))
    xs_new, us_new = xs, us
    while alpha > ls["alpha_min"]:
        xa = xs + alpha * dx
        ua = us + alpha * du
        phi_a, theta_a, _, _ = _merit(srbd_model, p, xa, ua, N, Ac, bc, False)
        if theta_a > ls["theta_max"]:
            if theta_a < (1.0 - ls["beta_theta"]) * theta:
                xs_new, us_new = xa, ua
                break
        elif max(theta_a, theta) < ls["theta_min"] and dphi < 0.0:
            if phi_a < phi + ls["eta"] * alpha * dphi:
                xs_new, us_new = xa, ua
                break
        else:
            if phi_a < phi - ls["beta_phi"] * theta or theta_a < (1.0 - ls["beta_theta"]) * theta:
                xs_new, us_new = xa, ua
                break
        alpha = ls["beta_alpha"] * alpha
    converged = dphi > -1e-3 and theta < 1e-6
    return xs_new, us_new, alpha, phi, theta, dphi, converged


def sqp_loop(srbd_model, oracle, p, xs, us, x0, alpha, settings, sqp_max_loop, constraints="none"):
    """One robot through the SQP loop of NMPCSolver::controlLoop (NMPC_solver.cpp:362-372):
    prepareQpStructures (srbd_model.build_qp), solveQpProblems (the C oracle with
    x0 - x_nmpc(:, 0), NMPC_solver.cpp:316-330), `if (checkConvergence()) break;`
    (line_search above).  Returns (xs, us, alpha, sqp_iterations, converged)."""
    xs, us = xs.copy(), us.copy()
    it, conv = 0, False
    for it in range(1, sqp_max_loop + 1):
        qp, _ = srbd_model.build_qp(xs[None], us[None], p, constraints)
        sol = oracle.solve(qp, settings, x0=(x0 - xs[0])[None])
        xs, us, alpha, _, _, _, conv = line_search(srbd_model, p, xs, us, sol["x"][0], sol["u"][0],
                                                   alpha)
        if conv:
            break
    return xs, us, alpha, it, conv
