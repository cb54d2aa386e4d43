"""The parallel-in-time single-QP kernel (csrc/riccati_scan_impl.h): unconstrained fp64
12 x 12 batches of at most 16 QPs with N <= 20 (N + 1 <= 32 elements and the LDS image).

The stage elements (A, b, C, zeta, J) are combined pairwise in ceil(log2(N + 1)) rounds;
the suffix products carry P_k, p_k, from which every stage forms K_k, k_k at once.  Its
combine solves without pivoting and hands the QP to the serial recursion (same launch) when
a pivot is below 1e-3 of its column: `_scan_pivot_ratio` restates the scan in numpy to show
which path a test QP takes, so the SRBD tests below exercise the scan itself."""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu


def _scan_pivot_ratio(qp, i):
    """Smallest |pivot| / (column max) of the scan's eliminations for QP i (numpy restatement
    of riccati_scan_impl.h, also checking P_k against the serial recursion)."""
    f = lambda n: np.asarray(getattr(qp, n)[i], dtype=np.float64)
    Q, S, R, q, r, A, B, b = (f(n) for n in ("Q", "S", "R", "q", "r", "A", "B", "b"))
    N = qp.N
    worst = [np.inf]

    def solve(M, X):
        M, X = M.copy(), X.copy()
        for k in range(12):
            worst[0] = min(worst[0], abs(M[k, k]) / np.abs(M[k:, k]).max())
            for j in range(k + 1, 12):
                m = M[j, k] / M[k, k]
                M[j, k:] -= m * M[k, k:]
                X[j] -= m * X[k]
        for k in range(11, -1, -1):
            X[k] = (X[k] - M[k, k + 1:] @ X[k + 1:]) / M[k, k]
        return X

    el = []
    for k in range(N):
        Ri = np.linalg.inv(R[k])
        el.append((A[k] - B[k] @ Ri @ S[k], b[k] - B[k] @ Ri @ r[k], B[k] @ Ri @ B[k].T,
                   q[k] - S[k].T @ Ri @ r[k], Q[k] - S[k].T @ Ri @ S[k]))
    el.append((np.zeros((12, 12)), np.zeros(12), np.zeros((12, 12)), q[N], Q[N]))
    d = 1
    while d <= N:
        nxt = []
        for k in range(N + 1):
            if k + d > N:
                nxt.append(el[k])
                continue
            Ai, bi, Ci, zi, Ji = el[k]
            Aj, bj, Cj, zj, Jj = el[k + d]
            X = solve(np.eye(12) + Ci @ Jj, np.column_stack([Ai, bi - Ci @ zj, Ci @ Aj.T]))
            XA, Xb, XC = X[:, :12], X[:, 12], X[:, 13:]
            nxt.append((Aj @ XA, Aj @ Xb + bj, Aj @ XC + Cj, XA.T @ (Jj @ bi + zj) + zi,
                        XA.T @ (Jj @ Ai) + Ji))
        el, d = nxt, 2 * d
    return worst[0], [e[4] for e in el]


def test_scan_srbd_vs_oracle(pkg, oracle):
    """The reference's QP (SRBD linearisation, N = 20) in batches of 1 and 16: the scan path
    (pivot ratio >= 1e-3, restated here), x, u, pi, P, K against the oracle at 1e-9 and against
    the same QPs solved in a batch of 64 (the serial matrix-core kernel) at 1e-11."""
    qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=1003, constraints="none")
    for i in range(16):
        ratio, _ = _scan_pivot_ratio(qp, i)
        assert ratio >= 1e-3, (i, ratio)
    serial = pkg.capi.solve(qp, x0, dict(ric_alg=0), riccati=True)
    ref = oracle.solve(qp.subset(slice(0, 16)), dict(ric_alg=0), x0=x0[:16])
    for idx in (slice(0, 1), slice(0, 16)):
        out = pkg.capi.solve(qp.subset(idx), x0[idx], dict(ric_alg=0), riccati=True)
        assert np.all(out["status"] == 0) and np.all(out["iter"] == 0)
        for i in range(out["x"].shape[0]):
            for key in ("x", "u", "pi", "P", "K"):
                assert helpers.is_approx(out[key][i], ref[key][i], 1e-9), (key, idx, i)
            for key in ("x", "u", "pi", "P", "p", "K", "k"):
                assert helpers.is_approx(out[key][i], serial[key][idx][i], 1e-11), (key, idx, i)


def test_scan_residuals_and_objective(pkg, oracle):
    """The fused residual pass of the scan kernel: res and obj of 4 SRBD QPs equal the oracle's
    compute_residuals on the same solution (HPIPM's nc = 0 exit statistics)."""
    qp, x0 = pkg.srbd_model.generate_batch(4, N=20, seed=606, constraints="none")
    out = pkg.capi.solve(qp, x0, dict(iter_max=30))
    ref = oracle.solve(qp, dict(iter_max=30), x0=x0)
    assert np.all(out["res"][:, 2:] == 0)
    scale = np.abs(ref["obj"]).max()
    np.testing.assert_allclose(out["obj"], ref["obj"], rtol=1e-9, atol=1e-12 * scale)
    assert np.all(out["res"][:, :2] < 1e-8 * max(1.0, scale)), out["res"]


def test_scan_random_qps_vs_oracle(pkg, oracle):
    """Random well-posed QPs (the reference test's generator, spectral radius scaled to 1):
    the scan's P_k agree with the serial recursion in numpy, and the kernel's x, u, pi, P, K
    with the oracle at 1e-9 (whichever path each QP takes)."""
    qp, x0 = helpers.random_unconstrained(8, 20, 12, 12, 5, pkg.OcpQpBatch)
    rho = np.max(np.abs(np.linalg.eigvals(qp.A)), axis=-1)
    qp.A = qp.A / rho[..., None, None]
    ref = oracle.solve(qp, dict(ric_alg=0), x0=x0)
    for i in range(qp.batch):
        _, Ps = _scan_pivot_ratio(qp, i)
        for k in range(qp.N + 1):
            assert helpers.is_approx(Ps[k], ref["P"][i, k], 1e-9), (i, k)
    out = pkg.capi.solve(qp, x0, dict(ric_alg=0), riccati=True)
    for i in range(qp.batch):
        for key in ("x", "u", "pi", "P", "K"):
            assert helpers.is_approx(out[key][i], ref[key][i], 1e-9), (key, i)


def test_scan_falls_back_on_indefinite_R(pkg, oracle):
    """A stage whose R is indefinite (R^-1 of the scan's elements does not exist; the serial
    recursion only needs G = R + B'PB > 0): the kernel solves the QP by the serial recursion
    in the same launch, equal to the oracle."""
    qp, x0 = helpers.random_unconstrained(3, 20, 12, 12, 9, pkg.OcpQpBatch)
    rho = np.max(np.abs(np.linalg.eigvals(qp.A)), axis=-1)
    qp.A = qp.A / rho[..., None, None]
    qp.R[:, 7] = -1e-3 * np.eye(12)
    ref = oracle.solve(qp, dict(ric_alg=0), x0=x0)
    out = pkg.capi.solve(qp, x0, dict(ric_alg=0), riccati=True)
    assert np.all(out["status"] == 0)
    for i in range(qp.batch):
        for key in ("x", "u", "pi", "P", "K"):
            assert helpers.is_approx(out[key][i], ref[key][i], 1e-9), (key, i)
