"""GPU parity of the unconstrained batched Riccati kernel (through the C-ABI).

Mirrors hpipm-cpp/test/ocp_qp_ipm_solver.cpp:22-110 (unconstrained): status
Success, iter 0, x/u/pi/P/-p/K/k against the textbook recursion at isApprox
1e-10 -- for every QP of a batch -- plus the C oracle and a dense-KKT solve.
"""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu


def _assert_riccati_matches(qp, x0, out, prec=1e-10, qps=None):
    for i in (range(qp.batch) if qps is None else qps):
        x, u, lmd, P, s, K, k = helpers.textbook_riccati(qp, x0[i], i)
        for j in range(qp.N + 1):
            assert helpers.is_approx(x[j], out["x"][i, j], prec), (i, j, "x")
            assert helpers.is_approx(lmd[j], out["pi"][i, j], prec), (i, j, "pi")
            if "P" in out:
                assert helpers.is_approx(P[j], out["P"][i, j], prec), (i, j, "P")
                assert helpers.is_approx(s[j], -out["p"][i, j], prec), (i, j, "p")
        for j in range(qp.N):
            assert helpers.is_approx(u[j], out["u"][i, j], prec), (i, j, "u")
            if "K" in out:
                assert helpers.is_approx(K[j], out["K"][i, j], prec), (i, j, "K")
                assert helpers.is_approx(k[j], out["k"][i, j], prec), (i, j, "k")


def test_reference_unconstrained_dims(pkg):
    """nx=5, nu=3, N=20 exactly as the reference test (padded path)."""
    qp, x0 = helpers.random_unconstrained(37, 20, 5, 3, 1, pkg.OcpQpBatch)
    out = pkg.capi.solve(qp, x0, {"mode": "Balance"}, riccati=True)
    assert np.all(out["status"] == 0) and np.all(out["iter"] == 0)
    assert np.all(out["x"][:, 0] == x0)
    _assert_riccati_matches(qp, x0, out)


@pytest.mark.parametrize("N", [1, 10, 20, 40])
def test_full_12x12_fast_path(pkg, N):
    qp, x0 = helpers.random_unconstrained(67, N, 12, 12, 100 + N, pkg.OcpQpBatch)
    if N > 10:
        # random 12x12 A has spectral radius ~2: over 20+ stages P grows like
        # rho^(2N) and pi = P x + p cancels catastrophically in any fp64
        # implementation (numpy included).  Keep the long horizons well-posed.
        rho = np.max(np.abs(np.linalg.eigvals(qp.A)), axis=-1)
        qp.A = qp.A / rho[..., None, None]
    out = pkg.capi.solve(qp, x0, None, riccati=True)
    assert np.all(out["status"] == 0)
    _assert_riccati_matches(qp, x0, out, prec=1e-9, qps=range(0, 67, 11))


@pytest.mark.parametrize("dims", [(12, 4), (7, 7), (1, 1), (12, 1), (3, 12)])
def test_padded_dims_vs_oracle(pkg, oracle, dims):
    nx, nu = dims
    qp, x0 = helpers.random_unconstrained(9, 8, nx, nu, nx * 31 + nu, pkg.OcpQpBatch)
    out = pkg.capi.solve(qp, x0, None, riccati=True)
    ref = oracle.solve(qp, None, x0=x0)
    for key in ("x", "u", "pi", "P", "p", "K", "k"):
        for i in range(qp.batch):
            assert helpers.is_approx(out[key][i], ref[key][i], 1e-10), (key, i)


def test_dense_kkt(pkg):
    qp, x0 = helpers.random_unconstrained(5, 20, 12, 12, 77, pkg.OcpQpBatch)
    rho = np.max(np.abs(np.linalg.eigvals(qp.A)), axis=-1)  # well-posed long horizon
    qp.A = qp.A / rho[..., None, None]
    out = pkg.capi.solve(qp, x0)
    for i in range(qp.batch):
        x, u, pi = helpers.dense_kkt(qp, x0[i], i)
        assert helpers.is_approx(x, out["x"][i], 1e-9)
        assert helpers.is_approx(u, out["u"][i], 1e-9)
        assert helpers.is_approx(pi[1:], out["pi"][i, 1:], 1e-9)


def test_batch_edges_and_ragged_batches(pkg):
    """batch not a multiple of the 16-QP workgroup; empty batch is a no-op."""
    for nb in (1, 15, 17, 33):
        qp, x0 = helpers.random_unconstrained(nb, 6, 12, 12, nb, pkg.OcpQpBatch)
        out = pkg.capi.solve(qp, x0)
        _assert_riccati_matches(qp, x0, out, prec=1e-9, qps=[0, nb - 1])
    h = pkg.capi.Handle(6, 12, 12, capacity=4)
    qp, x0 = helpers.random_unconstrained(1, 6, 12, 12, 3, pkg.OcpQpBatch)
    dt, st, data, sol = pkg.capi.device_buffers(qp, x0)
    h.solve_device(0, pkg.capi.settings_struct(), data, sol)  # no-op
    h.synchronize()
    with pytest.raises(pkg.capi.SrbdQpError, match="capacity"):
        h.solve_device(5, pkg.capi.settings_struct(), data, sol)


def test_host_entry_point_matches_device(pkg):
    qp, x0 = helpers.random_unconstrained(3, 10, 12, 12, 5, pkg.OcpQpBatch)
    import ctypes as C
    capi = pkg.capi
    p = qp.packed()
    p["x0"] = np.ascontiguousarray(x0)
    x = np.zeros((3, 11, 12)); u = np.zeros((3, 10, 12)); pi = np.zeros((3, 11, 12))
    st = np.zeros(3, dtype=np.int32)
    data = capi.Data(**{k: (None if p.get(k) is None else p[k].ctypes.data) for k in capi.DATA_FIELDS})
    sol = capi.Solution(x=x.ctypes.data, u=u.ctypes.data, pi=pi.ctypes.data, status=st.ctypes.data)
    h = capi.Handle(10, 12, 12, capacity=3)
    h.solve_host(3, capi.settings_struct(), data, sol)
    dev = capi.solve(qp, x0)
    assert np.array_equal(x, dev["x"]) and np.array_equal(u, dev["u"]) and np.array_equal(pi, dev["pi"])
    assert np.all(st == 0)


def test_srbd_qps_vs_oracle(pkg, oracle):
    """The reference's own QP: SRBD NMPC linearisation (N=20, nx=nu=12)."""
    gen = pkg.srbd_model
    qp, x0 = gen.generate_batch(24, N=20, seed=2024)
    out = pkg.capi.solve(qp, x0, None, riccati=True)
    ref = oracle.solve(qp, None, x0=x0)
    assert np.all(out["status"] == 0)
    for key in ("x", "u", "pi", "P", "K"):
        for i in range(qp.batch):
            assert helpers.is_approx(out[key][i], ref[key][i], 1e-9), (key, i)


def test_stage_major_layout_identical(pkg):
    """SRBD_QP_LAYOUT_STAGE_MAJOR inputs ([stage][batch][block]) give bit-identical
    results to the QP-major (Eigen-order) inputs."""
    import torch
    qp, x0 = pkg.srbd_model.generate_batch(40, N=20, seed=31, constraints="none")
    ref = pkg.capi.solve(qp, x0)
    h = pkg.capi.Handle(qp.N, 12, 12, 0, False, False, capacity=qp.batch, layout=1)
    dt, st, data, sol = pkg.capi.device_buffers(qp, x0)
    keep = {}
    for k in ("A", "B", "b", "Q", "S", "R", "q", "r"):
        keep[k] = dt[k].transpose(0, 1).contiguous()
        setattr(data, k, keep[k].data_ptr())
    h.solve_device(qp.batch, pkg.capi.settings_struct(None), data, sol)
    h.synchronize()
    for k in ("x", "u", "pi"):
        np.testing.assert_array_equal(st[k].cpu().numpy(), ref[k])
