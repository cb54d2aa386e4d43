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


@pytest.mark.parametrize("ric_alg", [0, 1])
def test_reference_unconstrained_dims(pkg, ric_alg):
    """nx=5, nu=3, N=20 exactly as the reference test (padded path); both Riccati
    variants (1, the square root, is hpipm-cpp's default)."""
    qp, x0 = helpers.random_unconstrained(37, 20, 5, 3, 1, pkg.OcpQpBatch)
    out = pkg.capi.solve(qp, x0, {"mode": "Balance", "ric_alg": ric_alg}, riccati=True)
    assert np.all(out["status"] == 0) and np.all(out["iter"] == 0)
    assert np.all(out["x"][:, 0] == x0)
    _assert_riccati_matches(qp, x0, out)


@pytest.mark.parametrize("ric_alg", [0, 1])
@pytest.mark.parametrize("N", [1, 10, 20, 40])
def test_full_12x12_fast_path(pkg, N, ric_alg):
    qp, x0 = helpers.random_unconstrained(67, N, 12, 12, 100 + N, pkg.OcpQpBatch)
    if N > 10:
        # random 12x12 A has spectral radius ~2: over 20+ stages P grows like
        # rho^(2N) and pi = P x + p cancels catastrophically in any fp64
        # implementation (numpy included).  Keep the long horizons well-posed.
        rho = np.max(np.abs(np.linalg.eigvals(qp.A)), axis=-1)
        qp.A = qp.A / rho[..., None, None]
    out = pkg.capi.solve(qp, x0, dict(ric_alg=ric_alg), riccati=True)
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


def test_host_staging_growth_keeps_pinned_mirror(pkg):
    """One handle serves host solves of 1, 64 and 1 QPs: the device staging buffer grows on
    the second call and the pinned mirror with it; every result equals the device call's.
    (Growing the device staging once also freed the pinned mirror without forgetting it, so
    the third call staged through freed host memory.)"""
    capi = pkg.capi
    qp, x0 = helpers.random_unconstrained(64, 20, 12, 12, 31, pkg.OcpQpBatch)
    dev = capi.solve(qp, x0)
    h = capi.Handle(20, 12, 12, capacity=64)
    try:
        for b in (1, 64, 1):
            p = {k: (None if v is None else np.ascontiguousarray(v[:b])) for k, v in qp.packed().items()}
            p["x0"] = np.ascontiguousarray(x0[:b])
            out = {k: np.zeros_like(dev[k][:b]) for k in ("x", "u", "pi", "status")}
            data = capi.Data(**{k: (None if p.get(k) is None else p[k].ctypes.data) for k in capi.DATA_FIELDS})
            h.solve_host(b, capi.settings_struct(), data, capi.Solution(**{k: v.ctypes.data for k, v in out.items()}))
            for key in out:
                assert np.array_equal(out[key], dev[key][:b]), (b, key)
    finally:
        h.close()


@pytest.mark.parametrize("ric_alg", [0, 1])
def test_srbd_qps_vs_oracle(pkg, oracle, ric_alg):
    """The reference's own QP: SRBD NMPC linearisation (N=20, nx=nu=12); its Q has
    zero weights, so the square-root variant meets singular P_N (zero pivots)."""
    gen = pkg.srbd_model
    qp, x0 = gen.generate_batch(24, N=20, seed=2024)
    st = dict(ric_alg=ric_alg)
    out = pkg.capi.solve(qp, x0, st, riccati=True)
    ref = oracle.solve(qp, st, x0=x0)
    assert np.all(out["status"] == 0)
    for key in ("x", "u", "pi", "P", "K"):
        for i in range(qp.batch):
            assert helpers.is_approx(out[key][i], ref[key][i], 1e-9), (key, i)


def test_stage_major_layout_identical(pkg):
    """SRBD_QP_LAYOUT_STAGE_MAJOR inputs ([stage][batch][block]) give bit-identical
    results to the QP-major (Eigen-order) inputs (a batch past the single-QP kernels'
    256: the streaming kernel reads both layouts)."""
    import torch
    qp, x0 = pkg.srbd_model.generate_batch(300, N=20, seed=31, constraints="none")
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


@pytest.mark.parametrize("case", ["srbd", "random", "padded", "stage_major", "fp32"])
def test_unconstrained_residuals_and_objective(pkg, oracle, case):
    """nc = 0: res (max |res_stat|, |res_eq|, 0, 0) and obj of the Riccati solution
    (HPIPM's comp_res_exit; d_ocp_qp_res_compute) against the oracle's
    compute_residuals on the same solution; compute_residuals = 0 zero-fills."""
    import torch
    N = 20
    if case in ("srbd", "stage_major", "fp32"):
        qp, x0 = pkg.srbd_model.generate_batch(24, N=N, seed=606, constraints="none")
    else:
        nx, nu = (12, 12) if case == "random" else (7, 5)
        qp, x0 = helpers.random_unconstrained(24, N, nx, nu, 607, pkg.OcpQpBatch)
        # well-posed horizon (see test_full_12x12_fast_path: with spectral radius ~2,
        # pi = P x + p cancels catastrophically over 20 stages in any fp64 order)
        rho = np.max(np.abs(np.linalg.eigvals(qp.A)), axis=-1)
        qp.A = qp.A / rho[..., None, None]
    ref = oracle.solve(qp, dict(iter_max=30), x0=x0)
    if case == "fp32":
        out = pkg.capi.solve(qp, x0, dict(iter_max=30), dtype=np.float32)
        # fp32 solution: residuals at fp32 rounding of the terms, objective to fp32
        assert np.all(out["res"][:, 2:] == 0)
        assert np.all(out["res"][:, :2] < 1e-2), out["res"].max(0)
        np.testing.assert_allclose(out["obj"], ref["obj"], rtol=1e-4, atol=1e-3)
        return
    if case == "stage_major":
        N, B = qp.N, qp.batch
        h = pkg.capi.Handle(N, 12, 12, 0, False, False, capacity=B, layout=1)
        p = qp.packed()
        p["x0"] = np.ascontiguousarray(x0)
        dev = {}
        for k, v in p.items():
            if v is None:
                continue
            t = torch.from_numpy(v).cuda()
            dev[k] = t.transpose(0, 1).contiguous() if k != "x0" else t
        f64 = dict(dtype=torch.float64, device="cuda")
        sol = {"x": torch.zeros(B, N + 1, 12, **f64), "u": torch.zeros(B, N, 12, **f64),
               "pi": torch.zeros(B, N + 1, 12, **f64), "res": torch.zeros(B, 4, **f64),
               "obj": torch.zeros(B, **f64)}
        data = pkg.capi.Data(**{k: (dev[k].data_ptr() if k in dev else None) for k in pkg.capi.DATA_FIELDS})
        S = pkg.capi.Solution(**{k: (sol[k].data_ptr() if k in sol else None) for k in pkg.capi.SOL_FIELDS})
        h.solve_device(B, pkg.capi.settings_struct(dict(iter_max=30)), data, S)
        h.synchronize()
        out = {k: v.cpu().numpy() for k, v in sol.items()}
    else:
        out = pkg.capi.solve(qp, x0, dict(iter_max=30), stats=True)
        # iteration 0's row of the stat table holds the same numbers (cols 6, 7, 10)
        np.testing.assert_array_equal(out["stat"][:, 0, 6], out["res"][:, 0])
        np.testing.assert_array_equal(out["stat"][:, 0, 7], out["res"][:, 1])
        np.testing.assert_array_equal(out["stat"][:, 0, 10], out["obj"])
        assert np.all(out["stat"][:, 1:] == 0)
    assert np.all(out["res"][:, 2:] == 0)
    scale = max(1.0, float(np.abs(ref["obj"]).max()))
    np.testing.assert_allclose(out["obj"], ref["obj"], rtol=1e-10, atol=1e-12 * scale)
    # both are rounding-level numbers of the same size (the two solutions differ at ~1e-15):
    # bounded by the magnitudes of the terms (the random data's unstable A makes x, pi large)
    mag = np.array([max(np.abs(out[k][i]).max() for k in ("x", "u", "pi")) for i in range(qp.batch)])
    for j in (0, 1):
        assert np.all(out["res"][:, j] <= 1e-12 * mag), (j, out["res"][:, j] / mag)
        assert np.all(ref["res"][:, j] <= 1e-12 * mag), (j, ref["res"][:, j] / mag)
    zero = pkg.capi.solve(qp, x0, dict(iter_max=30, compute_residuals=0))
    assert np.all(zero["res"] == 0) and np.all(zero["obj"] == 0)


@pytest.mark.parametrize("case", ["srbd", "padded", "stage_major", "nan"])
def test_residuals_large_batch_group_kernel(pkg, oracle, case):
    """Batches over 256 QPs take the group-mapped residual kernel (one 16-lane group per
    QP, the solve's column-owned loads): obj against the oracle's compute_residuals at
    1e-10, res at rounding level of the terms, NaN data -> NaNDetected, and on the same
    QPs the small-batch (stage-parallel) kernel's obj to 1e-12."""
    import torch
    B, N = 300, 12
    if case == "padded":
        qp, x0 = helpers.random_unconstrained(B, N, 7, 5, 611, pkg.OcpQpBatch)
        rho = np.max(np.abs(np.linalg.eigvals(qp.A)), axis=-1)
        qp.A = qp.A / rho[..., None, None]
    else:
        qp, x0 = pkg.srbd_model.generate_batch(B, N=N, seed=612, constraints="none")
    if case == "nan":
        qp.R[7, 3, 2, 2] = np.nan
    if case == "stage_major":
        h = pkg.capi.Handle(N, 12, 12, 0, False, False, capacity=B, layout=1)
        p = qp.packed()
        p["x0"] = np.ascontiguousarray(x0)
        dev = {k: (torch.from_numpy(v).cuda().transpose(0, 1).contiguous() if k != "x0"
                   else torch.from_numpy(v).cuda()) for k, v in p.items() if v is not None}
        f64 = dict(dtype=torch.float64, device="cuda")
        sol = {"x": torch.zeros(B, N + 1, 12, **f64), "u": torch.zeros(B, N, 12, **f64),
               "pi": torch.zeros(B, N + 1, 12, **f64), "res": torch.zeros(B, 4, **f64),
               "obj": torch.zeros(B, **f64), "status": torch.zeros(B, dtype=torch.int32, device="cuda")}
        data = pkg.capi.Data(**{k: (dev[k].data_ptr() if k in dev else None) for k in pkg.capi.DATA_FIELDS})
        S = pkg.capi.Solution(**{k: (sol[k].data_ptr() if k in sol else None) for k in pkg.capi.SOL_FIELDS})
        h.solve_device(B, pkg.capi.settings_struct(dict(iter_max=30)), data, S)
        h.synchronize()
        out = {k: v.cpu().numpy() for k, v in sol.items()}
    else:
        out = pkg.capi.solve(qp, x0, dict(iter_max=30), stats=True)
    if case == "nan":
        assert out["status"][7] == 3 and np.isnan(out["res"][7, 0])
        ok = np.arange(B) != 7
        assert np.all(out["status"][ok] == 0)
        return
    ref = oracle.solve(qp, dict(iter_max=30), x0=x0)
    scale = max(1.0, float(np.abs(ref["obj"]).max()))
    np.testing.assert_allclose(out["obj"], ref["obj"], rtol=1e-10, atol=1e-12 * scale)
    # rounding-level numbers (both solutions differ at ~1e-15): over 300 QPs the worst one
    # reaches 1.0e-12 of the terms' magnitude, so the bar is 4e-12 here, for the oracle too
    mag = np.array([max(np.abs(out[k][i]).max() for k in ("x", "u", "pi")) for i in range(B)])
    for j in (0, 1):
        assert np.all(out["res"][:, j] <= 4e-12 * mag), (j, np.max(out["res"][:, j] / mag))
        assert np.all(ref["res"][:, j] <= 4e-12 * mag), (j, np.max(ref["res"][:, j] / mag))
    assert np.all(out["res"][:, 2:] == 0)
    if case != "stage_major":
        assert np.array_equal(out["stat"][:, 0, 6], out["res"][:, 0])
        assert np.array_equal(out["stat"][:, 0, 10], out["obj"])
        assert np.all(out["stat"][:, 1:] == 0)
        small = pkg.capi.solve(qp.subset(slice(0, 200)), x0[:200], dict(iter_max=30))
        np.testing.assert_allclose(out["obj"][:200], small["obj"], rtol=1e-12, atol=1e-13 * scale)


@pytest.mark.parametrize("ric_alg", [0, 1])
@pytest.mark.parametrize("dtype,N", [(np.float64, 20), (np.float64, 26), (np.float32, 40)])
def test_latency_kernel_bit_identical(pkg, dtype, N, ric_alg):
    """Batches of up to 256 QPs (QP-major, image within a workgroup's LDS) run on a
    single-QP latency kernel, larger ones on the streaming kernel.  The LDS kernel runs
    the same instructions on the same values, so a QP's outputs are bit-identical either
    way -- also the reference's batch of one.  The fp64 classical solve at N <= 20 (the
    reference's NMPC QP) runs on the matrix-core kernel instead (riccati_latency_impl.h:
    the same algorithm, MFMA summation order): its outputs match to rounding, 1e-11."""
    qp, x0 = pkg.srbd_model.generate_batch(300, N=N, seed=77, constraints="none")
    st = dict(ric_alg=ric_alg)
    mfma = dtype == np.float64 and ric_alg == 0 and N <= 20
    big = pkg.capi.solve(qp, x0, st, riccati=True, dtype=dtype)         # streaming
    for idx in (slice(0, 1), slice(100, 164), slice(44, 300)):          # latency kernels
        small = pkg.capi.solve(qp.subset(idx), x0[idx], st, riccati=True, dtype=dtype)
        for key in ("x", "u", "pi", "P", "p", "K", "k", "status", "iter"):
            if mfma and key not in ("status", "iter"):
                for i in range(small[key].shape[0]):
                    assert helpers.is_approx(small[key][i], big[key][idx][i], 1e-11), (key, idx, i)
            else:
                assert np.array_equal(small[key], big[key][idx]), (key, idx)
    assert np.all(big["status"] == 0)


def test_latency_kernel_nan_and_singular_r(pkg):
    """The matrix-core single-QP kernel (batch <= 256, fp64, ric_alg 0, N <= 20: the
    reference's own call) against the streaming kernel on the same QPs with bad data: a NaN in
    one QP's R -> NaNDetected with a NaN stationarity residual in both; an input that is absent
    from another QP (its R row / column, S row, B column and r entry zero at every stage, so
    G's pivot is exactly 0: BLASFEO's dpotrf_l zeroes the direction) -> that input is 0,
    Success, and the residuals, the objective and x, u agree with the streaming kernel."""
    qp, x0 = pkg.srbd_model.generate_batch(300, N=20, seed=515, constraints="none")
    qp.R[3, 7, 4, 4] = np.nan
    i = 5
    qp.R[10, :, i, :] = 0.0
    qp.R[10, :, :, i] = 0.0
    qp.S[10, :, i, :] = 0.0
    qp.B[10, :, :, i] = 0.0
    qp.r[10, :, i] = 0.0
    st = dict(ric_alg=0)
    big = pkg.capi.solve(qp, x0, st)                                     # streaming kernel
    small = pkg.capi.solve(qp.subset(slice(0, 16)), x0[:16], st)         # matrix-core kernel
    for out in (big, small):
        assert out["status"][3] == 3 and np.isnan(out["res"][3, 0]), out["status"][:16]
        ok = np.arange(16) != 3
        assert np.all(out["status"][:16][ok] == 0)
        assert np.all(out["u"][10, :, i] == 0.0)
    for j in (0, 1):
        assert np.all(np.abs(small["res"][ok, j] - big["res"][:16][ok, j]) <= 1e-10 + 1e-6 * np.abs(big["res"][:16][ok, j]))
    np.testing.assert_allclose(small["obj"][ok], big["obj"][:16][ok], rtol=1e-11)
    for key in ("x", "u"):
        for q in np.nonzero(ok)[0]:
            assert helpers.is_approx(small[key][q], big[key][q], 1e-11), (key, q)


@pytest.mark.parametrize("ric_alg", [0, 1])
def test_streaming_kernel_partial_waves(pkg, oracle, ric_alg):
    """N = 30 (over the LDS image cap: the streaming kernel at every batch size) with
    batches of 1, 2, 3, 5 and 37 QPs: the last wave holds fewer than four QP groups, and
    its records still leave through the wave's LDS image in whole pieces.  Every QP's
    outputs are bit-identical to the same QP inside a full batch, and match the oracle."""
    qp, x0 = pkg.srbd_model.generate_batch(64, N=30, seed=91, constraints="none")
    st = dict(ric_alg=ric_alg)
    big = pkg.capi.solve(qp, x0, st, riccati=True)
    ref = oracle.solve(qp.subset(slice(0, 5)), dict(ric_alg=ric_alg), x0=x0[:5])
    for key in ("x", "u", "pi"):
        assert helpers.is_approx(big[key][:5], ref[key], 1e-9), key
    for nb in (1, 2, 3, 5, 37):
        idx = slice(7, 7 + nb)
        small = pkg.capi.solve(qp.subset(idx), x0[idx], st, riccati=True)
        for key in ("x", "u", "pi", "P", "p", "K", "k", "status"):
            assert np.array_equal(small[key], big[key][idx]), (key, nb)


def test_host_staging_in_place(pkg):
    """srbd_qp_host_staging_f64 (ABI 10): the staging pointers a caller packs its QPs into
    and passes back to srbd_qp_solve_host_f64 are solved in place (no staging copy; for a
    small unconstrained batch the kernel reads and writes the pinned buffer itself) and give
    the device call's results bit for bit; a second staging call of the same shape returns
    the same pointers."""
    import ctypes as C
    capi = pkg.capi
    for nb in (1, 3):
        qp, x0 = pkg.srbd_model.generate_batch(nb, N=20, seed=404 + nb, constraints="none")
        dev = capi.solve(qp, x0, dict(ric_alg=0), riccati=True)
        h = capi.Handle(20, 12, 12, capacity=nb)
        try:
            s = capi.settings_struct(dict(ric_alg=0))
            mark = 16
            d = capi.Data(**{k: mark for k in ("A", "B", "b", "Q", "S", "R", "q", "r", "x0")})
            o = capi.Solution(**{k: mark for k in ("x", "u", "pi", "P", "p", "K", "k", "status", "iter", "res", "obj")})
            h.host_staging(nb, s, d, o)
            d2 = capi.Data(**{k: mark for k in ("A", "B", "b", "Q", "S", "R", "q", "r", "x0")})
            o2 = capi.Solution(**{k: mark for k in ("x", "u", "pi", "P", "p", "K", "k", "status", "iter", "res", "obj")})
            h.host_staging(nb, s, d2, o2)
            assert d2.A == d.A and o2.stat == o.stat is None and o2.x == o.x
            p = qp.packed()
            p["x0"] = np.ascontiguousarray(x0)
            for k in ("A", "B", "b", "Q", "S", "R", "q", "r", "x0"):
                src = np.ascontiguousarray(p[k], dtype=np.float64)
                C.memmove(getattr(d, k), src.ctypes.data, src.nbytes)
            h.solve_host(nb, s, d, o)

            def arr(ptr, shape, ct=C.c_double):
                n = int(np.prod(shape))
                return np.ctypeslib.as_array((ct * n).from_address(ptr)).reshape(shape).copy()
            assert np.array_equal(arr(o.x, dev["x"].shape), dev["x"])
            assert np.array_equal(arr(o.u, dev["u"].shape), dev["u"])
            assert np.array_equal(arr(o.pi, dev["pi"].shape), dev["pi"])
            assert np.array_equal(np.swapaxes(arr(o.K, (nb, 20, 12, 12)), -1, -2), dev["K"])
            assert np.all(arr(o.status, (nb,), C.c_int) == 0)
        finally:
            h.close()


def test_host_solve_early_factors(pkg):
    """srbd_qp_solve_host_cb_f64 (ABI 12): the callback runs exactly once, and at that point
    P, p, K, k in the staged outputs already hold their final values (on the zero-copy
    single-QP path the latency kernel writes them and raises a flag per QP before its forward
    sweep ends); every output equals the plain host solve's bit for bit.  N = 20 takes the
    early path (batch 1 and 8 flags); N = 26 (zero copy, not the latency kernel) and staging
    through non-pinned caller buffers call back after the solve."""
    import ctypes as C
    capi = pkg.capi
    keys_in = ("A", "B", "b", "Q", "S", "R", "q", "r", "x0")
    keys_out = ("x", "u", "pi", "P", "p", "K", "k", "status", "iter", "res", "obj")

    def arr(ptr, n, ct=C.c_double):
        return np.ctypeslib.as_array((ct * n).from_address(ptr)).copy()

    for N, nb in ((20, 1), (20, 8), (26, 2)):
        qp, x0 = pkg.srbd_model.generate_batch(nb, N=N, seed=90 + N + nb, constraints="none")
        p = qp.packed()
        p["x0"] = np.ascontiguousarray(x0)
        sizes = dict(x=nb * (N + 1) * 12, u=nb * N * 12, pi=nb * (N + 1) * 12, P=nb * (N + 1) * 144,
                     p=nb * (N + 1) * 12, K=nb * N * 144, k=nb * N * 12, res=nb * 4, obj=nb)
        results = []
        for early in (False, True):
            h = capi.Handle(N, 12, 12, capacity=nb)
            try:
                s = capi.settings_struct(dict(ric_alg=0))
                d = capi.Data(**{k: 16 for k in keys_in})
                o = capi.Solution(**{k: 16 for k in keys_out})
                h.host_staging(nb, s, d, o)
                for k in keys_in:
                    src = np.ascontiguousarray(p[k], dtype=np.float64)
                    C.memmove(getattr(d, k), src.ctypes.data, src.nbytes)
                seen = []
                if early:
                    h.solve_host(nb, s, d, o, on_factors=lambda: seen.append(
                        {k: arr(getattr(o, k), sizes[k]) for k in ("P", "p", "K", "k")}))
                else:
                    h.solve_host(nb, s, d, o)
                out = {k: arr(getattr(o, k), n) for k, n in sizes.items()}
                out["status"] = arr(o.status, nb, C.c_int)
                if early:
                    assert len(seen) == 1, (N, nb)
                    for k, v in seen[0].items():
                        assert np.array_equal(v, out[k]), (N, nb, k)
                results.append(out)
            finally:
                h.close()
        for k in results[0]:
            assert np.array_equal(results[0][k], results[1][k]), (N, nb, k)
        assert np.all(results[1]["status"] == 0)

    # caller-owned (non-staged) output buffers: the factors are copied out before the callback
    qp, x0 = pkg.srbd_model.generate_batch(1, N=20, seed=7, constraints="none")
    ref = capi.solve(qp, x0, dict(ric_alg=0), riccati=True)
    p = qp.packed()
    p["x0"] = np.ascontiguousarray(x0)
    ins = {k: np.ascontiguousarray(p[k], dtype=np.float64) for k in keys_in}
    outs = dict(x=np.zeros(21 * 12), u=np.zeros(20 * 12), pi=np.zeros(21 * 12), P=np.zeros(21 * 144),
                p=np.zeros(21 * 12), K=np.zeros(20 * 144), k=np.zeros(20 * 12))
    h = capi.Handle(20, 12, 12, capacity=1)
    try:
        s = capi.settings_struct(dict(ric_alg=0))
        d = capi.Data(**{k: v.ctypes.data for k, v in ins.items()})
        o = capi.Solution(**{k: v.ctypes.data for k, v in outs.items()})
        seen = []
        h.solve_host(1, s, d, o, on_factors=lambda: seen.append(outs["K"].copy()))
        assert len(seen) == 1 and np.array_equal(seen[0], outs["K"])
        assert np.array_equal(np.swapaxes(outs["K"].reshape(1, 20, 12, 12), -1, -2), ref["K"])
        assert np.array_equal(outs["u"].reshape(ref["u"].shape), ref["u"])
    finally:
        h.close()


def test_host_solve_resident_server(pkg, monkeypatch):
    """The one-QP host call's resident server (riccati_latency_server_kernel): a sequence of
    different QPs through one handle -- back to back, after the server has idled out (5 ms),
    across a change of settings (the server is relaunched with the new arguments) and with the
    early-factor callback -- gives the launched kernel's results bit for bit
    (SRBD_LAT_SERVER=0: every call launches)."""
    import ctypes as C
    import time
    capi = pkg.capi
    keys_in = ("A", "B", "b", "Q", "S", "R", "q", "r", "x0")
    keys_out = ("x", "u", "pi", "P", "p", "K", "k", "status", "iter", "res", "obj")
    sizes = dict(x=21 * 12, u=20 * 12, pi=21 * 12, P=21 * 144, p=21 * 12, K=20 * 144, k=20 * 12, res=4, obj=1)

    def run(server, seeds, gaps, cfgs, cbs):
        monkeypatch.setenv("SRBD_LAT_SERVER", "1" if server else "0")
        h = capi.Handle(20, 12, 12, capacity=1)
        outs = []
        try:
            for seed, gap, cfg, cb in zip(seeds, gaps, cfgs, cbs):
                time.sleep(gap)
                qp, x0 = pkg.srbd_model.generate_batch(1, N=20, seed=seed, constraints="none")
                p = qp.packed()
                p["x0"] = np.ascontiguousarray(x0)
                s = capi.settings_struct(cfg)
                d = capi.Data(**{k: 16 for k in keys_in})
                o = capi.Solution(**{k: 16 for k in keys_out})
                h.host_staging(1, s, d, o)
                for k in keys_in:
                    src = np.ascontiguousarray(p[k], dtype=np.float64)
                    C.memmove(getattr(d, k), src.ctypes.data, src.nbytes)
                calls = []
                h.solve_host(1, s, d, o, on_factors=(lambda: calls.append(1)) if cb else None)
                r = {k: np.ctypeslib.as_array((C.c_double * n).from_address(getattr(o, k))).copy()
                     for k, n in sizes.items() if getattr(o, k)}
                r["status"] = np.ctypeslib.as_array((C.c_int * 1).from_address(o.status)).copy()
                assert len(calls) == (1 if cb else 0)
                outs.append(r)
        finally:
            h.close()
        return outs

    seeds = [11, 12, 13, 14, 15, 16, 17]
    gaps = [0, 0, 0, 0.03, 0, 0, 0.03]
    cfgs = [dict(ric_alg=0)] * 3 + [dict(ric_alg=0, compute_residuals=0), dict(ric_alg=0)] * 2
    cbs = [False, True, True, False, True, False, False]
    a = run(True, seeds, gaps, cfgs, cbs)
    b = run(False, seeds, gaps, cfgs, cbs)
    for i, (ra, rb) in enumerate(zip(a, b)):
        assert ra.keys() == rb.keys()
        for k in ra:
            assert np.array_equal(ra[k], rb[k]), (i, k)
        assert ra["status"][0] == 0
    # distinct QPs gave distinct answers (no stale staging data)
    assert not np.array_equal(a[0]["u"], a[1]["u"])


def _one_qp_calls(pkg, seeds, cbs):
    """One-QP host calls through one handle (the reference's call pattern); returns the staged
    outputs of every call and each call's wall time."""
    import ctypes as C
    import time
    capi = pkg.capi
    keys_in = ("A", "B", "b", "Q", "S", "R", "q", "r", "x0")
    keys_out = ("x", "u", "pi", "P", "p", "K", "k", "status", "iter", "res", "obj")
    sizes = dict(x=21 * 12, u=20 * 12, pi=21 * 12, P=21 * 144, p=21 * 12, K=20 * 144, k=20 * 12, res=4, obj=1)
    h = capi.Handle(20, 12, 12, capacity=1)
    outs, times = [], []
    try:
        s = capi.settings_struct(dict(ric_alg=0))
        for seed, cb in zip(seeds, cbs):
            qp, x0 = pkg.srbd_model.generate_batch(1, N=20, seed=seed, constraints="none")
            p = qp.packed()
            p["x0"] = np.ascontiguousarray(x0)
            d = capi.Data(**{k: 16 for k in keys_in})
            o = capi.Solution(**{k: 16 for k in keys_out})
            h.host_staging(1, s, d, o)
            for k in keys_in:
                src = np.ascontiguousarray(p[k], dtype=np.float64)
                C.memmove(getattr(d, k), src.ctypes.data, src.nbytes)
            calls = []
            t0 = time.perf_counter()
            h.solve_host(1, s, d, o, on_factors=(lambda: calls.append(1)) if cb else None)
            times.append(time.perf_counter() - t0)
            assert len(calls) == (1 if cb else 0)
            r = {k: np.ctypeslib.as_array((C.c_double * n).from_address(getattr(o, k))).copy()
                 for k, n in sizes.items()}
            r["status"] = np.ctypeslib.as_array((C.c_int * 1).from_address(o.status)).copy()
            outs.append(r)
    finally:
        h.close()
    return outs, times


def test_resident_server_relaunch_after_post(pkg, monkeypatch):
    """The server leaves between the host's liveness check and its post on EVERY call: zero
    idle time (SRBD_LAT_SERVER_IDLE_MS=0: it leaves at its first empty poll) and the post held
    back 1 ms after the check (SRBD_LAT_SERVER_POST_DELAY_US).  The wait loop must relaunch it
    with the pending request still to serve (round 5 relaunched it with last_done = the posted
    number, so the request was never served and the call failed after 30 s).  60 calls, with
    and without the early-factor callback (a per-request mailbox word: no relaunch for it),
    each answered bit-identically to the launched kernel (SRBD_LAT_SERVER=0) and each in
    under 5 ms."""
    seeds = list(range(300, 360))
    cbs = [i % 3 == 1 for i in range(60)]
    monkeypatch.setenv("SRBD_LAT_SERVER", "1")
    monkeypatch.setenv("SRBD_LAT_SERVER_IDLE_MS", "0")
    monkeypatch.setenv("SRBD_LAT_SERVER_POST_DELAY_US", "1000")
    a, ta = _one_qp_calls(pkg, seeds, cbs)
    monkeypatch.delenv("SRBD_LAT_SERVER_IDLE_MS")
    monkeypatch.delenv("SRBD_LAT_SERVER_POST_DELAY_US")
    monkeypatch.setenv("SRBD_LAT_SERVER", "0")
    b, _ = _one_qp_calls(pkg, seeds, cbs)
    for i, (ra, rb) in enumerate(zip(a, b)):
        for k in ra:
            assert np.array_equal(ra[k], rb[k]), (i, k)
        assert ra["status"][0] == 0
    assert max(ta) < 5e-3, sorted(ta)[-5:]


def test_resident_server_leaves_other_streams_running(pkg, monkeypatch):
    """A busy server (calls back to back on one handle, so it never idles out) must not hold
    back kernels of other streams: HIP maps streams onto a few hardware queues (4 per process
    here) that process their packets in order, so a kernel queued behind the resident server
    on a shared queue would wait until the server leaves.  The server's stream is created so
    that it does not share a queue with other streams (srbd_qp_capi.hip server_launch); here a
    small kernel on each of 8 fresh torch streams, and on torch's default stream, finishes
    within 50 ms while the server keeps serving; so does one on each of 2 high-priority streams,
    which may share the server's queue but wait at most its 20 ms lifetime."""
    import threading
    import time
    import torch
    monkeypatch.setenv("SRBD_LAT_SERVER", "1")
    stop = threading.Event()
    n_calls = [0]
    err = []

    def caller():
        import ctypes as C
        try:
            capi = pkg.capi
            keys_in = ("A", "B", "b", "Q", "S", "R", "q", "r", "x0")
            qp, x0 = pkg.srbd_model.generate_batch(1, N=20, seed=5, constraints="none")
            p = qp.packed()
            p["x0"] = np.ascontiguousarray(x0)
            h = capi.Handle(20, 12, 12, capacity=1)
            try:
                s = capi.settings_struct(dict(ric_alg=0))
                d = capi.Data(**{k: 16 for k in keys_in})
                o = capi.Solution(**{k: 16 for k in ("x", "u", "pi", "status")})
                h.host_staging(1, s, d, o)
                for k in keys_in:
                    src = np.ascontiguousarray(p[k], dtype=np.float64)
                    C.memmove(getattr(d, k), src.ctypes.data, src.nbytes)
                while not stop.is_set():
                    h.solve_host(1, s, d, o)
                    assert C.c_int.from_address(o.status).value == 0
                    n_calls[0] += 1
            finally:
                h.close()
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    x = torch.zeros(1024, device="cuda")
    torch.cuda.synchronize()
    # 8 default-priority streams (they never share the server's queue) and 2 high-priority ones
    # (they may: the server leaves after its first answer past 20 ms, so they wait < 50 ms)
    streams = [torch.cuda.Stream() for _ in range(8)] + [torch.cuda.Stream(priority=-1) for _ in range(2)]
    for s in streams:  # bind each stream to its hardware queue before the server starts
        with torch.cuda.stream(s):
            x.add_(1)
    torch.cuda.synchronize()
    t = threading.Thread(target=caller)
    t.start()
    try:
        t_wait = time.perf_counter() + 10
        while n_calls[0] < 20 and not err and time.perf_counter() < t_wait:
            time.sleep(0.001)
        assert n_calls[0] >= 20, (n_calls, err)
        lat = []
        for s in streams + [torch.cuda.default_stream()]:
            ev = torch.cuda.Event()
            t0 = time.perf_counter()
            with torch.cuda.stream(s):
                x.add_(1)
                ev.record(s)
            while not ev.query() and time.perf_counter() - t0 < 2.0:
                time.sleep(0.0002)
            lat.append(time.perf_counter() - t0)
        calls_during = n_calls[0]
    finally:
        stop.set()
        t.join()
    assert not err, err
    assert calls_during >= 20
    assert max(lat) < 0.05, [round(v * 1e3, 2) for v in lat]
