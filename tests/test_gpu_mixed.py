"""settings.f32_iters: the mixed-precision IPM for fp64 solves.  The first n IPM
iterations run in fp32 on a narrowed copy of the data (half the bytes per sweep);
the fp64 IPM then continues from that iterate (x, u, pi and every lam / t: HPIPM's
warm_start = 2 level) on the caller's fp64 data to the fp64 tolerances.  The bar is
the fp64 path's own: the oracle at the tolerances of test_gpu_ipm.py (1e-7 on x / u
at tol 1e-8), and the fp64 solution at the NMPC settings."""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)


def test_mixed_box_u_nmpc_settings(pkg):
    """Config 3's problem at the reference caller's settings (NMPC_solver.cpp:70-82):
    the continuation picks up where fp32 stopped (fp64 iterations = the fp64 solve's
    minus n) and lands on the fp64 solution well inside the tolerance."""
    qp, x0 = pkg.srbd_model.generate_batch(256, N=20, seed=5, constraints="box_u")
    o64 = pkg.capi.solve(qp, x0, NMPC, stats=True)
    mix = pkg.capi.solve(qp, x0, dict(NMPC, f32_iters=6), stats=True, riccati=True)
    assert np.all(o64["status"] == 0) and np.all(mix["status"] == 0)
    assert np.all(mix["res"] <= 1e-4)
    assert np.all(mix["iter"] <= o64["iter"] - 6 + 1), (mix["iter"], o64["iter"])
    for key in ("x", "u"):
        d = np.abs(mix[key] - o64[key]).reshape(qp.batch, -1).max(1)
        scale = np.abs(o64[key]).reshape(qp.batch, -1).max(1)
        assert np.all(d <= 1e-5 * scale), (key, (d / scale).max())
    # the stat table is the fp64 continuation's: row 0 is the fp32 iterate's residuals
    # in fp64, mu no longer mu0
    assert np.all(mix["stat"][:, 0, 5] < 1.0)


@pytest.mark.parametrize("case", ["box_u", "cone", "general_with_c"])
def test_mixed_vs_oracle_tight(pkg, oracle, case):
    """tol 1e-8 (hpipm-cpp's defaults): the fp64 continuation reaches the oracle's
    solution like the fp64 path does -- fp32 only supplies the starting point."""
    if case == "general_with_c":
        qp, x0 = helpers.random_constrained(20, 12, 12, 12, 14, 211, pkg.OcpQpBatch)
        st = dict(iter_max=50, mode="Balance")
    else:
        qp, x0 = pkg.srbd_model.generate_batch(24, N=20, seed=12, constraints=case)
        st = dict(iter_max=40)
    ref = oracle.solve(qp, st, x0=x0)
    out = pkg.capi.solve(qp, x0, dict(st, f32_iters=5))
    plain = pkg.capi.solve(qp, x0, st)
    assert np.all(ref["status"] == 0), ref["status"]
    ok = plain["status"] == 0
    assert np.all(out["status"][ok] == 0), (out["status"], out["res"])
    for i in np.nonzero(ok)[0]:
        for key in ("x", "u"):
            assert helpers.is_approx(out[key][i], ref[key][i], 1e-7), (key, i)
        assert helpers.is_approx(out["pi"][i, 1:], ref["pi"][i, 1:], 1e-6), ("pi", i)


def test_mixed_ignored_when_padded_or_unconstrained(pkg):
    """nx or nu < 12 (the 12 x 12 embedding) and nc = 0: f32_iters changes no bit."""
    qp, x0 = helpers.random_constrained(16, 8, 5, 3, 4, 7, pkg.OcpQpBatch)
    a = pkg.capi.solve(qp, x0, dict(iter_max=40))
    b = pkg.capi.solve(qp, x0, dict(iter_max=40, f32_iters=5))
    for key in a:
        assert np.array_equal(a[key], b[key]), key
    qp, x0 = pkg.srbd_model.generate_batch(16, N=10, seed=3, constraints="none")
    a = pkg.capi.solve(qp, x0)
    b = pkg.capi.solve(qp, x0, dict(f32_iters=5))
    for key in a:
        assert np.array_equal(a[key], b[key]), key


def test_mixed_iter_max_bounds_the_fp32_pass(pkg):
    """f32_iters >= iter_max: the fp32 pass runs iter_max - 1 iterations and the fp64
    continuation the one left of the budget; a QP that one step does not finish is solved
    again by the plain fp64 path (never worse than fp64: ADVICE r02).  Warm-started calls
    narrow the caller's x / u for the fp32 pass."""
    qp, x0 = pkg.srbd_model.generate_batch(32, N=20, seed=9, constraints="box_u")
    o64 = pkg.capi.solve(qp, x0, NMPC)
    plain8 = pkg.capi.solve(qp, x0, dict(NMPC, iter_max=8), stats=True)
    mix = pkg.capi.solve(qp, x0, dict(NMPC, iter_max=8, f32_iters=50), stats=True)
    assert np.all(mix["status"] <= plain8["status"]), (mix["status"], plain8["status"])
    cont = mix["iter"] == 1  # finished by the one fp64 step of the continuation
    assert np.all(mix["status"][cont] == 0) and np.all(mix["res"][cont] <= 1e-4)
    for key in ("x", "u", "pi", "status", "iter", "res", "obj", "stat"):
        assert np.array_equal(mix[key][~cont], plain8[key][~cont]), key
    # the fp64 path converges at iter_max = 30: so does the mixed path with f32_iters >= iter_max
    assert np.all(o64["status"] == 0)
    mix30 = pkg.capi.solve(qp, x0, dict(NMPC, f32_iters=50))
    assert np.all(mix30["status"] == 0), mix30["status"]
    assert np.all(mix30["res"] <= 1e-4)
    warm = pkg.capi.solve(qp, x0, dict(NMPC, warm_start=1, f32_iters=4),
                          x_init=o64["x"], u_init=o64["u"])
    assert np.all(warm["status"] == 0), warm["status"]
    assert np.all(warm["res"] <= 1e-4)
    # (a different tol-1e-4 KKT point than the cold solve's: the warm start re-centres
    # lam = mu0 / t, and the SRBD R has 1e-4 curvature directions, so no closeness bound)


def test_mixed_fallback_keeps_the_callers_warm_start(pkg):
    """warm_start = 1: a QP the continuation leaves unsolved is solved again by the fp64
    path from the caller's own x / u (kept on entry), so it ends bit for bit as the plain
    warm-started fp64 call ends it."""
    qp, x0 = pkg.srbd_model.generate_batch(200, N=20, seed=29, constraints="box_u")
    o64 = pkg.capi.solve(qp, x0, NMPC)
    xi = o64["x"] + 0.01 * np.sin(np.arange(o64["x"].size)).reshape(o64["x"].shape)
    ui = o64["u"] + 0.5 * np.cos(np.arange(o64["u"].size)).reshape(o64["u"].shape)
    st = dict(NMPC, iter_max=3, warm_start=1)
    plain = pkg.capi.solve(qp, x0, st, x_init=xi, u_init=ui, stats=True)
    mix = pkg.capi.solve(qp, x0, dict(st, f32_iters=2), x_init=xi, u_init=ui, stats=True)
    bad = mix["status"] != 0
    assert bad.sum() > 10, np.bincount(mix["status"])
    for key in ("x", "u", "pi", "status", "iter", "res", "obj", "stat"):
        assert np.array_equal(mix[key][bad], plain[key][bad]), key


def test_mixed_host_entry_point_matches_device(pkg):
    """srbd_qp_solve_host_f64 runs the same mixed path: bit-identical to the device call."""
    capi = pkg.capi
    qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=17, constraints="box_u")
    st = dict(NMPC, f32_iters=6)
    dev = capi.solve(qp, x0, st)
    p = {k: (None if v is None else np.ascontiguousarray(v)) for k, v in qp.packed().items()}
    p["x0"] = np.ascontiguousarray(x0)
    out = {k: np.zeros_like(dev[k]) for k in ("x", "u", "pi", "status", "iter")}
    data = capi.Data(**{k: (None if p.get(k) is None else p[k].ctypes.data) for k in capi.DATA_FIELDS})
    sol = capi.Solution(**{k: v.ctypes.data for k, v in out.items()})
    h = capi.Handle(qp.N, qp.nx, qp.nu, 0, True, False, capacity=qp.batch)
    try:
        h.solve_host(qp.batch, capi.settings_struct(st), data, sol)
    finally:
        h.close()
    for key in out:
        assert np.array_equal(out[key], dev[key]), key


def test_mixed_fallback_is_the_fp64_solve(pkg):
    """A QP the fp64 continuation ends with a numerical breakdown (here NaNDetected: a NaN
    in its data) is solved again cold in fp64, so it ends exactly as the fp64 path ends it,
    bit for bit; the rest of the batch is not re-solved."""
    qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=23, constraints="box_u")
    bad = [5, 40]
    for i in bad:
        qp.q[i, 7, 3] = np.nan
    st = dict(NMPC)
    plain = pkg.capi.solve(qp, x0, st, stats=True)
    mix = pkg.capi.solve(qp, x0, dict(st, f32_iters=6), stats=True)
    assert np.all(plain["status"][bad] == 3) and np.all(mix["status"][bad] == 3)
    for key in ("x", "u", "pi", "status", "iter", "res", "obj", "stat"):
        assert np.array_equal(mix[key][bad], plain[key][bad], equal_nan=key not in ("status", "iter")), key
    ok = np.setdiff1d(np.arange(qp.batch), bad)
    assert np.all(mix["status"][ok] == 0) and np.all(mix["res"][ok] <= 1e-4)


@pytest.mark.parametrize("f32_iters", [2, 3, 8])
def test_mixed_iteration_budget(pkg, f32_iters):
    """The fp32 iterations count against iter_max: m = min(f32_iters, iter_max - 1) fp32
    iterations, then at most iter_max - m fp64 ones (reported in iter).  At iter_max = 3
    most QPs are not finished there; each of those is solved again by the fp64 path and
    returns exactly its result (here MaxIterReached after 3 fp64 iterations)."""
    qp, x0 = pkg.srbd_model.generate_batch(300, N=20, seed=23, constraints="box_u")
    st = dict(NMPC, iter_max=3)
    plain = pkg.capi.solve(qp, x0, st, stats=True)
    mix = pkg.capi.solve(qp, x0, dict(st, f32_iters=f32_iters), stats=True)
    m = min(f32_iters, 2)
    ok = mix["status"] == 0
    assert np.all(mix["iter"][ok] <= 3 - m) and np.all(mix["iter"] >= 1)
    assert (~ok).sum() > 100, np.bincount(mix["status"])
    for key in ("x", "u", "pi", "status", "iter", "res", "obj", "stat"):
        assert np.array_equal(mix[key][~ok], plain[key][~ok]), key
    assert np.all(mix["status"] <= plain["status"])
    # the stat table keeps the caller's iter_max + 2 rows; rows past the last fp64 one are 0
    assert mix["stat"].shape[1] == 5
    for i in range(qp.batch):
        assert np.all(mix["stat"][i, mix["iter"][i] + 1:] == 0)


def test_one_handle_mixed_rescue_mixed_bit_identical(pkg):
    """One handle serves, in turn, an fp64 solve with f32_iters, an fp32 solve with
    f64_rescue whose unsolved set makes the rescue buffer grow, and the fp64 f32_iters
    solve again: every result bit-identical to the same solve on a fresh handle.
    (Growing the rescue buffer once freed the handle's mixed-precision buffer without
    forgetting it, so the third solve wrote into freed device memory.)"""
    N = 20
    qp, x0 = pkg.srbd_model.generate_batch(64, N=N, seed=21, constraints="cone")
    st64 = dict(NMPC, f32_iters=6)
    # fp32 tolerances out of the fp32 pass's reach in 3 iterations: most of the batch
    # continues in fp64
    st32 = dict(iter_max=30, tol_stat=1e-6, tol_eq=1e-6, tol_ineq=1e-6, tol_comp=1e-6,
                split_step=1, f64_rescue=3)
    h = pkg.capi.Handle(N, 12, 12, 24, False, False, capacity=qp.batch)
    a1 = pkg.capi.solve(qp, x0, st64, handle=h)
    b1 = pkg.capi.solve(qp, x0, st32, handle=h, dtype=np.float32)
    a2 = pkg.capi.solve(qp, x0, st64, handle=h)
    h.close()
    a_ref = pkg.capi.solve(qp, x0, st64)
    b_ref = pkg.capi.solve(qp, x0, st32, dtype=np.float32)
    assert np.all(a_ref["status"] == 0) and np.all(b_ref["status"] == 0)
    for key in a_ref:
        assert np.array_equal(a1[key], a_ref[key]), ("first fp64", key)
        assert np.array_equal(a2[key], a_ref[key]), ("second fp64", key)
        assert np.array_equal(b1[key], b_ref[key]), ("fp32 rescue", key)
