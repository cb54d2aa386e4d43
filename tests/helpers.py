"""Shared test helpers: problem generators and independent numpy references.

The numpy references here are deliberately written straight from the
reference's own test (hpipm-cpp/test/ocp_qp_ipm_solver.cpp) and from the KKT
conditions, independently of both the C oracle and the HIP path.
"""
from __future__ import annotations

import importlib.util
import json
import math
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden"
PKG_DIR = REPO / "srbd-nmpc-solver_amd"


def load_package():
    """Import the product package (its directory name contains hyphens)."""
    name = "srbd_nmpc_solver_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle  # noqa: E402
    return oracle


def is_approx(a, b, prec):
    """Eigen's isApprox: ||a - b|| <= prec * min(||a||, ||b||) (Frobenius)."""
    a = np.asarray(a, dtype=np.float64).ravel()
    b = np.asarray(b, dtype=np.float64).ravel()
    return np.linalg.norm(a - b) <= prec * min(np.linalg.norm(a), np.linalg.norm(b))


# ---------------------------------------------------------------------------
# problem generators
# ---------------------------------------------------------------------------
def random_unconstrained(batch, N, nx, nu, seed, OcpQpBatch):
    """Batched restatement of test/ocp_qp_ipm_solver.cpp:22-47 with a fixed seed
    (Eigen::Random is uniform on [-1, 1]; its implicit std::rand seed is not portable)."""
    rng = np.random.default_rng(seed)
    U = lambda *s: rng.uniform(-1.0, 1.0, size=s)
    A = U(batch, N, nx, nx)
    B = U(batch, N, nx, nu)
    b = U(batch, N, nx)
    H = U(batch, N, nx + nu, nx + nu)
    HH = H @ np.swapaxes(H, -1, -2)
    Q = np.zeros((batch, N + 1, nx, nx))
    Q[:, :N] = HH[:, :, nu:, nu:]
    S = np.ascontiguousarray(HH[:, :, :nu, nu:])
    R = np.ascontiguousarray(HH[:, :, :nu, :nu])
    R = R + np.abs(U(batch, N, nu))[..., None] * np.eye(nu)
    q = U(batch, N + 1, nx)
    r = U(batch, N, nu)
    HN = U(batch, nx, nx)
    Q[:, N] = HN @ np.swapaxes(HN, -1, -2)
    x0 = U(batch, nx)
    return OcpQpBatch(N=N, nx=nx, nu=nu, A=A, B=B, b=b, Q=Q, S=S, R=R, q=q, r=r), x0


def random_constrained(batch, N, nx, nu, ng, seed, OcpQpBatch, x0_scale=1.0, stable=True):
    """Batched restatement of test/ocp_qp_ipm_solver.cpp:112-158 (box u on {0,1,2},
    box x on {1,3} for stages 1..N, general constraints), fixed seed.

    The reference draws A from Eigen::Random; with its (unportable) std::rand
    seed that draw happens to be feasible.  Random draws of unstable A with
    the x-box of :145-148 are often infeasible, so by default A is rescaled to
    spectral radius 0.95 and b scaled by 0.1 (stable=True) so that every
    generated QP is feasible."""
    rng = np.random.default_rng(seed)
    U = lambda *s: rng.uniform(-1.0, 1.0, size=s)
    qp, x0 = random_unconstrained(batch, N, nx, nu, seed + 7919, OcpQpBatch)
    if stable:
        rho = np.max(np.abs(np.linalg.eigvals(qp.A)), axis=-1)
        qp.A = qp.A * (0.95 / rho)[..., None, None]
        qp.b = 0.1 * qp.b  # keeps |x| well inside the +-10 x-box of :145-148
    x0 = x0 * x0_scale
    # reference 'constrained' keeps R = HH's corner (no diagonal shift): make it PD enough
    lbu = np.zeros((batch, N, nu)); ubu = np.zeros((batch, N, nu))
    lbu_m = np.zeros((batch, N, nu)); ubu_m = np.zeros((batch, N, nu))
    idxu = [i for i in (0, 1, 2) if i < nu]
    for i in idxu:
        lbu[:, :, i] = -0.05 - np.abs(U(batch, N))
        ubu[:, :, i] = 0.05 + np.abs(U(batch, N))
        lbu_m[:, :, i] = 1.0
        ubu_m[:, :, i] = 1.0
    # strictly feasible by construction: bounds are centred on the zero-input
    # trajectory (the reference centres the x-box on x0, :146-147)
    xt = np.zeros((batch, N + 1, nx)); xt[:, 0] = x0
    for k in range(N):
        xt[:, k + 1] = np.einsum("bij,bj->bi", qp.A[:, k], xt[:, k]) + qp.b[:, k]
    lbx = np.zeros((batch, N + 1, nx)); ubx = np.zeros((batch, N + 1, nx))
    lbx_m = np.zeros((batch, N + 1, nx)); ubx_m = np.zeros((batch, N + 1, nx))
    for i in [i for i in (1, 3) if i < nx]:
        lbx[:, 1:, i] = xt[:, 1:, i] - 0.05 - 10 * np.abs(U(batch, N))
        ubx[:, 1:, i] = xt[:, 1:, i] + 0.05 + 10 * np.abs(U(batch, N))
        lbx_m[:, 1:, i] = 1.0
        ubx_m[:, 1:, i] = 1.0
    qp.lbu, qp.ubu, qp.lbu_mask, qp.ubu_mask = lbu, ubu, lbu_m, ubu_m
    qp.lbx, qp.ubx, qp.lbx_mask, qp.ubx_mask = lbx, ubx, lbx_m, ubx_m
    if ng > 0:
        qp.ng = ng
        qp.C = U(batch, N + 1, ng, nx)
        qp.D = U(batch, N, ng, nu)
        cx = np.einsum("bkgj,bkj->bkg", qp.C, xt)
        cx[:, 0] = 0.0  # C_0 is dropped by the x0 embedding (ocp_qp_ipm_solver.cpp:128)
        qp.lg = cx - 0.05 - 10 * np.abs(U(batch, N + 1, ng))
        qp.ug = cx + 0.05 + 10 * np.abs(U(batch, N + 1, ng))
    return qp, x0


def quadcopter(OcpQpBatch):
    """The compareResults problem (test/ocp_qp_ipm_solver.cpp:170-240)."""
    d = json.loads((GOLDEN / "quadcopter.json").read_text())
    N, nx, nu = d["N"], d["nx"], d["nu"]
    A = np.array(d["A"]); B = np.array(d["B"]); b = np.array(d["b"])
    Q = np.diag(d["Q_diag"]); R = np.diag(d["R_diag"]); xr = np.array(d["x_ref"], dtype=float)
    q = -Q @ xr
    ev = lambda v: (math.pi / 6.0 if v == "pi/6" else -math.pi / 6.0 if v == "-pi/6" else float(v))
    lbx_i = [ev(v) for v in d["lbx"]]; ubx_i = [ev(v) for v in d["ubx"]]
    lbx = np.zeros((1, N + 1, nx)); ubx = np.zeros((1, N + 1, nx))
    lbx_m = np.zeros((1, N + 1, nx)); ubx_m = np.zeros((1, N + 1, nx))
    for c, i in enumerate(d["idxbx"]):
        lbx[0, 1:, i] = lbx_i[c]; ubx[0, 1:, i] = ubx_i[c]
        lbx_m[0, 1:, i] = 1.0; ubx_m[0, 1:, i] = d["ubx_mask"][c]
    u0 = d["u0"]
    lbu = np.full((1, N, nu), d["umin"] - u0); ubu = np.full((1, N, nu), d["umax"] - u0)
    qp = OcpQpBatch(
        N=N, nx=nx, nu=nu,
        A=np.broadcast_to(A, (1, N, nx, nx)).copy(), B=np.broadcast_to(B, (1, N, nx, nu)).copy(),
        b=np.broadcast_to(b, (1, N, nx)).copy(), Q=np.broadcast_to(Q, (1, N + 1, nx, nx)).copy(),
        S=np.zeros((1, N, nu, nx)), R=np.broadcast_to(R, (1, N, nu, nu)).copy(),
        q=np.broadcast_to(q, (1, N + 1, nx)).copy(), r=np.zeros((1, N, nu)),
        lbu=lbu, ubu=ubu, lbu_mask=np.ones((1, N, nu)), ubu_mask=np.ones((1, N, nu)),
        lbx=lbx, ubx=ubx, lbx_mask=lbx_m, ubx_mask=ubx_m)
    goldens = [np.loadtxt(GOLDEN / f) for f in d["golden"]]
    return qp, d, goldens, A, B, b


# ---------------------------------------------------------------------------
# independent numpy references
# ---------------------------------------------------------------------------
def textbook_riccati(qp, x0, i=0):
    """Literal numpy transcription of test/ocp_qp_ipm_solver.cpp:60-90 for QP i.
    Returns x, u, lmd, P, s, K, k (s = -p)."""
    N = qp.N
    A, B, b, Q, S, R, q, r = (qp.A[i], qp.B[i], qp.b[i], qp.Q[i], qp.S[i], qp.R[i], qp.q[i], qp.r[i])
    P = [None] * (N + 1); s = [None] * (N + 1); K = [None] * N; k = [None] * N
    P[N] = Q[N]; s[N] = -q[N]
    for j in range(N - 1, -1, -1):
        F = Q[j] + A[j].T @ P[j + 1] @ A[j]
        H = S[j] + B[j].T @ P[j + 1] @ A[j]
        G = R[j] + B[j].T @ P[j + 1] @ B[j]
        Ginv = np.linalg.inv(G)
        K[j] = -Ginv @ H
        k[j] = -Ginv @ (B[j].T @ P[j + 1] @ b[j] - B[j].T @ s[j + 1] + r[j])
        P[j] = F - K[j].T @ G @ K[j]
        s[j] = A[j].T @ (s[j + 1] - P[j + 1] @ b[j]) - q[j] - H.T @ k[j]
    x = [None] * (N + 1); u = [None] * N
    x[0] = x0
    for j in range(N):
        u[j] = K[j] @ x[j] + k[j]
        x[j + 1] = A[j] @ x[j] + B[j] @ u[j] + b[j]
    lmd = [P[j] @ x[j] - s[j] for j in range(N + 1)]
    return (np.array(x), np.array(u), np.array(lmd), np.array(P), np.array(s), np.array(K), np.array(k))


def dense_kkt(qp, x0, i=0):
    """Solve the unconstrained QP of QP i as one dense KKT system (x0 fixed)."""
    N, nx, nu = qp.N, qp.nx, qp.nu
    nv = N * nu + N * nx  # u_0..u_{N-1}, x_1..x_N
    ne = N * nx
    ui = lambda k: k * nu
    xi = lambda k: N * nu + (k - 1) * nx
    H = np.zeros((nv, nv)); g = np.zeros(nv)
    Aeq = np.zeros((ne, nv)); beq = np.zeros(ne)
    for k in range(N):
        H[ui(k):ui(k) + nu, ui(k):ui(k) + nu] = qp.R[i, k]
        g[ui(k):ui(k) + nu] = qp.r[i, k]
        if k == 0:
            g[ui(0):ui(0) + nu] += qp.S[i, 0] @ x0
        else:
            H[xi(k):xi(k) + nx, xi(k):xi(k) + nx] = qp.Q[i, k]
            H[ui(k):ui(k) + nu, xi(k):xi(k) + nx] = qp.S[i, k]
            H[xi(k):xi(k) + nx, ui(k):ui(k) + nu] = qp.S[i, k].T
            g[xi(k):xi(k) + nx] = qp.q[i, k]
        # x_{k+1} = A x_k + B u_k + b_k
        rows = slice(k * nx, (k + 1) * nx)
        Aeq[rows, xi(k + 1):xi(k + 1) + nx] = -np.eye(nx)
        Aeq[rows, ui(k):ui(k) + nu] = qp.B[i, k]
        if k == 0:
            beq[rows] = -(qp.A[i, 0] @ x0 + qp.b[i, 0])
        else:
            Aeq[rows, xi(k):xi(k) + nx] = qp.A[i, k]
            beq[rows] = -qp.b[i, k]
    H[xi(N):xi(N) + nx, xi(N):xi(N) + nx] = qp.Q[i, N]
    g[xi(N):xi(N) + nx] = qp.q[i, N]
    KKT = np.block([[H, Aeq.T], [Aeq, np.zeros((ne, ne))]])
    rhs = np.concatenate([-g, beq])
    sol = np.linalg.solve(KKT, rhs)
    v, lam = sol[:nv], sol[nv:]
    u = v[:N * nu].reshape(N, nu)
    x = np.vstack([x0[None], v[N * nu:].reshape(N, nx)])
    # multipliers of x_{k+1} = ...: stationarity H v + g + Aeq' lam = 0 with the
    # row sign above (-x_{k+1}) gives pi_{k+1} = lam_k.
    pi = np.vstack([np.zeros((1, nx)), lam.reshape(N, nx)])
    return x, u, pi


def kkt_residuals(qp, x0, sol, i=0):
    """Max-norm KKT residuals of a returned primal/dual pair (box/general constraints
    included through multipliers recovered as the stationarity slack).  Returns dict."""
    N, nx, nu = qp.N, qp.nx, qp.nu
    x, u, pi = sol["x"][i], sol["u"][i], sol["pi"][i]
    out = {}
    out["x0"] = float(np.max(np.abs(x[0] - x0)))
    dyn = max(float(np.max(np.abs(qp.A[i, k] @ x[k] + qp.B[i, k] @ u[k] + qp.b[i, k] - x[k + 1])))
              for k in range(N))
    out["dyn"] = dyn
    return out
