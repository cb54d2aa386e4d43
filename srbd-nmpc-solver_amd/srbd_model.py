"""Batched SRBD QP-data generator (numpy): the producer of the hot path's inputs.

Restates, vectorised over (batch, stage), how the reference builds the QP the
solver receives:

* dynamics ``SRBDModel::GetContinuousDynamic`` / ``GetShootingDynamic``
  (dynamics/SRBD_model.cpp:75-235): RK4 defect with *Euler* Jacobians
  (:179-181), A = j_x, B = j_u, b = -f;
* SO(3) helpers expm / jl / jlt / djl / djlt (dynamics/orientation_tool.h:76-227);
* friction cone ``GetConstrain`` (SRBD_model.cpp:237-260) and the relaxed
  log-barrier ``Barrier`` (:262-295);
* QP assembly ``NMPCSolver::prepareQpStructures`` (NMPC_solver.cpp:276-314):
  Q, q = Q (x - x_ref), S = 0, R = R_ + Ac' diag(ddb) Ac, r = R_ u + Ac' db,
  terminal Qf, qf;
* parameters: config/mpc_option.yaml:2-18, setupDynamics (NMPC_solver.cpp:332-339),
  setupReference (:341-351), SRBDModel() defaults (SRBD_model.cpp:5-24).

Inputs are drawn per QP from a counter-based seed (``seed + qp_index``), as
SURVEY.md section 8(d) prescribes, so any shard of a batch can be generated
independently.  The generator is the workload, not the product path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np

from .qp import OcpQpBatch

__all__ = ["SrbdParams", "generate_batch", "build_qp", "sample_trajectories", "shooting_dynamics", "friction_cone", "barrier"]


@dataclass(frozen=True)
class SrbdParams:
    # config/mpc_option.yaml:2-18
    Q: Tuple[float, ...] = (0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 10)
    Qf: Tuple[float, ...] = (0.5, 0.5, 0.5, 0.01, 0.01, 0.01, 100, 100, 100, 0.0, 0.0, 100.0)
    R: float = 0.0001
    dt: float = 0.015
    N: int = 20
    Lbody: Tuple[float, float, float] = (0.541667, 0.516667, 1.0416667)
    mu_b: float = 0.1
    theta_b: float = 5.0
    # NMPC_solver.cpp:332-339 / SRBD_model.cpp:5-24
    mass: float = 15.0
    foot_r: Tuple[float, float, float] = (0.0, -0.1, 0.0)
    foot_l: Tuple[float, float, float] = (0.0, 0.1, 0.0)
    mu: float = 0.5
    Lfx: float = 0.05
    Lfz: float = 0.05
    fmax: float = 1000.0
    fmin: float = 0.0
    # NMPC_solver.cpp:344-345
    x_ref: Tuple[float, ...] = (0, 0, 0.2, 0, 0, 0, 0.5, 0, 1.0, 0, 0, 0)


def load_mpc_option(source) -> Tuple["SrbdParams", Dict]:
    """The reference's config file (config/mpc_option.yaml), read with the keys of
    NMPCSolver::readYaml (NMPC_solver.cpp:22-46): MPC.{Q, Qf, R, dt_MPC, horizon_MPC,
    sqp_max_loop}, Physical.Lbody, mu_b, theta_b, N_rep.  `source` is a path or the
    YAML text.  Returns (SrbdParams, {"sqp_max_loop", "N_rep"}); a missing key raises
    KeyError like yaml-cpp's as<>() on an absent node throws."""
    import os
    import yaml
    text = source
    if isinstance(source, (str, os.PathLike)) and os.path.exists(source):
        with open(source) as f:
            text = f.read()
    cfg = yaml.safe_load(text)
    mpc, phys = cfg["MPC"], cfg["Physical"]
    def vec(v, n, name):
        if len(v) != n:
            raise ValueError(f"{name} needs {n} values, got {len(v)}")
        return tuple(float(x) for x in v)

    p = SrbdParams(Q=vec(mpc["Q"], 12, "MPC.Q"), Qf=vec(mpc["Qf"], 12, "MPC.Qf"), R=float(mpc["R"]),
                   dt=float(mpc["dt_MPC"]), N=int(mpc["horizon_MPC"]),
                   Lbody=vec(phys["Lbody"], 3, "Physical.Lbody"), mu_b=float(cfg["mu_b"]),
                   theta_b=float(cfg["theta_b"]))
    return p, {"sqp_max_loop": int(mpc["sqp_max_loop"]), "N_rep": int(cfg["N_rep"])}


# ---------------------------------------------------------------------------
# SO(3) helpers, orientation_tool.h (batched over leading dims)
# ---------------------------------------------------------------------------
def skew(v):
    z = np.zeros(v.shape[:-1])
    return np.stack([np.stack([z, -v[..., 2], v[..., 1]], -1),
                     np.stack([v[..., 2], z, -v[..., 0]], -1),
                     np.stack([-v[..., 1], v[..., 0], z], -1)], -2)


def _theta(v):
    th = np.sqrt(np.sum(v * v, axis=-1))
    return np.maximum(th, 1e-10)  # h = 1e-10 clamp (orientation_tool.h:82-86)


def expm(v):
    th = _theta(v)[..., None, None]
    V = skew(v)
    I = np.eye(3)
    return I + (np.sin(th) / th) * V + ((1.0 - np.cos(th)) / (th * th)) * (V @ V)


def jl(v):
    th = _theta(v)[..., None, None]
    V = skew(v) / th
    I = np.eye(3)
    return (np.sin(th) / th) * I + (1.0 - np.sin(th) / th) * (V @ V + I) + ((1.0 - np.cos(th)) / th) * V


def jlt(v):
    th = _theta(v)[..., None, None]
    V = skew(v) / th
    I = np.eye(3)
    cot = 1.0 / np.tan(0.5 * th)
    return (0.5 * cot * th) * I + (1.0 - 0.5 * cot * th) * (V @ V + I) - (0.5 * th) * V


def djl(v):
    th = _theta(v)[..., None, None]
    V = skew(v) / th
    s, c = np.sin(th), np.cos(th)
    th2, th3 = th * th, th * th * th
    base = ((th * s + 2.0 * (c - 1.0)) / th3) * V + (-(2.0 * th - 3.0 * s + th * c) / th3) * (V @ V)
    sv = skew(v)
    out = []
    for a in range(3):
        e = np.zeros(3)
        e[a] = 1.0
        se = skew(e)
        d = ((th - s) / th3) * (se @ sv + sv @ se) + ((1.0 - c) / th2) * se
        out.append(d + base * v[..., a][..., None, None])
    return out


def djlt(v):
    J = jlt(v)
    return [-(J @ d @ J) for d in djl(v)]


# ---------------------------------------------------------------------------
# dynamics, SRBD_model.cpp:75-235
# ---------------------------------------------------------------------------
def _consts(p: SrbdParams):
    Lb = np.diag(1.0 / np.array(p.Lbody))  # SetInertia(L) stores L^-1 (SRBD_model.cpp:46-49)
    pf0 = np.array(p.foot_r)
    pf1 = np.array(p.foot_l)
    return Lb, pf0, pf1


def continuous(x, u, p: SrbdParams, jac: bool):
    Lb, pf0, pf1 = _consts(p)
    r, l, pos, v = x[..., 0:3], x[..., 3:6], x[..., 6:9], x[..., 9:12]
    R = expm(r)
    Jlt = jlt(r)
    RLR = R @ Lb @ np.swapaxes(R, -1, -2)
    w = np.einsum("...ij,...j->...i", RLR, l)
    dx = np.empty(x.shape)
    dx[..., 0:3] = np.einsum("...ij,...j->...i", Jlt, w)
    dx[..., 3:6] = (u[..., 3:6] + u[..., 9:12]
                    + np.einsum("...ij,...j->...i", skew(pf0 - pos), u[..., 0:3])
                    + np.einsum("...ij,...j->...i", skew(pf1 - pos), u[..., 6:9]))
    dx[..., 6:9] = v
    dx[..., 9:12] = (u[..., 0:3] + u[..., 6:9]) / p.mass + np.array([0.0, 0.0, -9.8])
    if not jac:
        return dx, None, None
    dJ = djlt(r)
    djw = np.stack([np.einsum("...ij,...j->...i", dJ[a], w) for a in range(3)], -1)
    Jl = jl(r)
    jfx = np.zeros(x.shape[:-1] + (12, 12))
    jfx[..., 0:3, 0:3] = djw + Jlt @ (RLR @ skew(l) - skew(w)) @ Jl
    jfx[..., 0:3, 3:6] = Jlt @ RLR
    jfx[..., 3:6, 6:9] = skew(u[..., 0:3] + u[..., 6:9])
    jfx[..., 6:9, 9:12] = np.eye(3)
    jfu = np.zeros(x.shape[:-1] + (12, 12))
    jfu[..., 3:6, 0:3] = skew(pf0 - pos)
    jfu[..., 3:6, 3:6] = np.eye(3)
    jfu[..., 3:6, 6:9] = skew(pf1 - pos)
    jfu[..., 3:6, 9:12] = np.eye(3)
    jfu[..., 9:12, 0:3] = np.eye(3) / p.mass
    jfu[..., 9:12, 6:9] = np.eye(3) / p.mass
    return dx, jfx, jfu


def shooting_dynamics(x, x_next, u, p: SrbdParams):
    """A = I + dt jfx, B = dt jfu (Euler Jacobians, :179-181), b = RK4(x,u) - x_next."""
    dt = p.dt
    k1, jfx, jfu = continuous(x, u, p, True)
    k2, _, _ = continuous(x + 0.5 * dt * k1, u, p, False)
    k3, _, _ = continuous(x + 0.5 * dt * k2, u, p, False)
    k4, _, _ = continuous(x + dt * k3, u, p, False)
    x_get = x + (dt / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
    A = np.eye(12) + dt * jfx
    B = dt * jfu
    b = x_get - x_next  # b = -f, f = x_next - x_get (:194-197, :225-229)
    return A, B, b


def friction_cone(p: SrbdParams):
    """Ac (24 x 12) and constant term bc of GetConstrain (SRBD_model.cpp:237-260), R_f = I."""
    Rf = np.eye(3)
    Ac = np.zeros((24, 12))
    bc = np.zeros(24)
    for leg in range(2):
        blk = np.zeros((12, 6))
        blk[0] = [-1, 0, p.mu, 0, 0, 0]
        blk[1] = [0, -1, p.mu, 0, 0, 0]
        blk[2] = [1, 0, p.mu, 0, 0, 0]
        blk[3] = [0, 1, p.mu, 0, 0, 0]
        blk[4] = [0, 0, -1, 0, 0, 0]
        blk[5] = [0, 0, 1, 0, 0, 0]
        blk[6] = np.concatenate([p.Lfx * Rf[:, 2], -Rf[:, 1]])
        blk[7] = np.concatenate([p.Lfx * Rf[:, 2], Rf[:, 1]])
        blk[8] = np.concatenate([p.Lfz * Rf[:, 2], -Rf[:, 2]])
        blk[9] = np.concatenate([p.Lfz * Rf[:, 2], Rf[:, 2]])
        blk[10] = np.concatenate([np.zeros(3), -Rf[:, 0]])
        blk[11] = np.concatenate([np.zeros(3), Rf[:, 0]])
        Ac[12 * leg:12 * leg + 12, 6 * leg:6 * leg + 6] = blk
        bc[12 * leg + 4] = p.fmax
        bc[12 * leg + 5] = -p.fmin
    return Ac, bc


def barrier(value, mu, theta):
    """Relaxed log-barrier (SRBD_model.cpp:262-295): returns b, db, ddb."""
    inside = value > theta
    safe = np.where(inside, value, 1.0)
    b_in = -mu * np.log(safe)
    db_in = -mu / safe
    ddb_in = mu / (safe * safe)
    z = (value - 2.0 * theta) / theta
    b_out = 0.5 * mu * (z * z - 1.0) - mu * math.log(theta)
    db_out = mu * (value - 2.0 * theta) / (theta * theta)
    ddb_out = np.full_like(value, mu / (theta * theta))
    return (np.where(inside, b_in, b_out), np.where(inside, db_in, db_out),
            np.where(inside, ddb_in, ddb_out))


# ---------------------------------------------------------------------------
# batch generator
# ---------------------------------------------------------------------------
SIGMA_X = np.array([0.05] * 3 + [0.2] * 3 + [0.02] * 3 + [0.1] * 3)
U_BOX_LO = np.array([-50.0, -50.0, 0.0, -5.0, -5.0, -5.0] * 2)
U_BOX_HI = np.array([50.0, 50.0, 300.0, 5.0, 5.0, 5.0] * 2)


def sample_trajectories(batch, N, seed, p: SrbdParams, first: int = 0):
    """Per-QP linearisation points from seed + global QP index (counter-based)."""
    xr = np.array(p.x_ref, dtype=np.float64)
    xs = np.empty((batch, N + 1, 12))
    us = np.empty((batch, N, 12))
    x0 = np.empty((batch, 12))
    for i in range(batch):
        rng = np.random.default_rng([seed, first + i])
        xs[i] = xr + rng.normal(size=(N + 1, 12)) * SIGMA_X
        f = np.empty((N, 2, 6))
        f[..., 0:2] = rng.uniform(-15.0, 15.0, size=(N, 2, 2))
        f[..., 2] = rng.uniform(40.0, 110.0, size=(N, 2))
        f[..., 3:6] = rng.uniform(-2.0, 2.0, size=(N, 2, 3))
        us[i] = f.reshape(N, 12)
        x0[i] = rng.normal(size=12) * SIGMA_X  # x0 - x_nmpc(:,0) (NMPC_solver.cpp:320)
    return xs, us, x0


def build_qp(xs, us, p: Optional[SrbdParams] = None, constraints: str = "none", meta=None):
    """QP data of NMPCSolver::prepareQpStructures (NMPC_solver.cpp:276-314) at the
    linearisation points xs [B][N+1][12], us [B][N][12].  Returns (OcpQpBatch, fc)."""
    p = p or SrbdParams()
    batch, N = us.shape[0], us.shape[1]
    A, B, b = shooting_dynamics(xs[:, :-1], xs[:, 1:], us, p)
    Ac, bc = friction_cone(p)
    fc = np.einsum("ij,bkj->bki", Ac, us) + bc
    _, db, ddb = barrier(fc, p.mu_b, p.theta_b)
    Qd = np.diag(np.array(p.Q, dtype=np.float64))
    Qf = float(N) * np.diag(np.array(p.Qf, dtype=np.float64))  # Qf_ = N * Qf (NMPC_solver.cpp:58)
    Rm = p.R * np.eye(12)
    xr = np.array(p.x_ref, dtype=np.float64)
    Q = np.empty((batch, N + 1, 12, 12))
    Q[:, :N] = Qd
    Q[:, N] = Qf
    q = np.empty((batch, N + 1, 12))
    q[:, :N] = np.einsum("ij,bkj->bki", Qd, xs[:, :N] - xr)
    q[:, N] = np.einsum("ij,bj->bi", Qf, xs[:, N] - xr)
    R = Rm + np.einsum("ci,bkc,cj->bkij", Ac, ddb, Ac)
    r = np.einsum("ij,bkj->bki", Rm, us) + np.einsum("ci,bkc->bki", Ac, db)
    S = np.zeros((batch, N, 12, 12))
    qp = OcpQpBatch(N=N, nx=12, nu=12, A=A, B=B, b=b, Q=Q, S=S, R=R, q=q, r=r,
                    meta=dict(meta or {}, constraints=constraints))
    if constraints == "box_u":
        qp.lbu = U_BOX_LO - us
        qp.ubu = U_BOX_HI - us
    elif constraints == "cone":
        qp.ng = 24
        qp.D = np.broadcast_to(Ac, (batch, N, 24, 12)).copy()
        qp.C = None  # the cone constrains u only (C = 0): passed as NULL, the C-free kernel path
        qp.lg = np.zeros((batch, N + 1, 24))
        qp.lg[:, :N] = -fc
        qp.ug = np.full((batch, N + 1, 24), 1e10)
        qp.lg_mask = np.zeros((batch, N + 1, 24))
        qp.lg_mask[:, :N] = 1.0
        qp.ug_mask = np.zeros((batch, N + 1, 24))
    elif constraints != "none":
        raise ValueError(f"unknown constraints {constraints!r}")
    return qp, fc


def generate_batch(batch: int, N: int = 20, seed: int = 1001, constraints: str = "none",
                   p: Optional[SrbdParams] = None, first: int = 0):
    """Build `batch` SRBD OCP-QPs exactly as prepareQpStructures does.

    constraints: "none" (the reference's own QP: friction cone as a barrier in
    the cost, no inequalities), "box_u" (config 3: u + du inside per-foot force /
    torque boxes), "cone" (config 5: lg <= Ac du with lg = -f(u), ug masked).
    Returns (OcpQpBatch, x0)."""
    p = p or SrbdParams()
    xs, us, x0 = sample_trajectories(batch, N, seed, p, first)
    qp, _ = build_qp(xs, us, p, constraints, meta={"seed": seed, "first": first})
    return qp, x0
