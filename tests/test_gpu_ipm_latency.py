"""GPU parity of the one-launch latency IPM (srbd-nmpc-solver_amd/csrc/ipm_latency.hip): the
C-ABI sends fp64 classical-Riccati (ric_alg 0) solves -- Speed, and since round 6 Balance /
Robust with HPIPM's iterative refinement -- of up to SRBD_IPM_LATENCY_MAX QPs (default 512)
there, one workgroup per QP, and everything else to the batched kernels.

Checked against the oracle (oracle/ocp_qp_oracle.c oracle_solve, HPIPM d_ocp_qp_ipm_solve
restated) and against the batched kernels on the same QPs (SRBD_IPM_LATENCY_MAX=0 forces
those): status, iteration counts, x / u / pi at the solve's accuracy, the residual norms,
the Riccati getters and the per-iteration statistics.  The settings are the reference's NMPC
ones (NMPC_solver.cpp:70-82: Speed, ric_alg 0, split_step) unless a test varies them."""
import os

import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

NMPC = dict(mode="Speed", iter_max=30, ric_alg=0, split_step=1, pred_corr=1, warm_start=0,
            reg_prim=1e-12, tol_stat=1e-8, tol_eq=1e-8, tol_ineq=1e-8, tol_comp=1e-8)


class _Path:
    """Run the block with the latency IPM on (default switch) or off (batched kernels)."""

    def __init__(self, on):
        self.on = on

    def __enter__(self):
        self.old = os.environ.get("SRBD_IPM_LATENCY_MAX")
        os.environ["SRBD_IPM_LATENCY_MAX"] = "512" if self.on else "0"

    def __exit__(self, *exc):
        if self.old is None:
            del os.environ["SRBD_IPM_LATENCY_MAX"]
        else:
            os.environ["SRBD_IPM_LATENCY_MAX"] = self.old


def both(pkg, qp, x0, st, **kw):
    with _Path(True):
        lat = pkg.capi.solve(qp, x0, st, **kw)
    with _Path(False):
        bat = pkg.capi.solve(qp, x0, st, **kw)
    return lat, bat


def _check_vs_oracle(out, ref, batch, tol=1e-7, it_slack=1, oracle_misses=0):
    """Every QP the oracle solves: Success here too, in its iterations +-it_slack, x and u
    within tol.  oracle_misses: QPs the oracle may leave at MaxIter (random C / D rows)."""
    ok = ref["status"] == 0
    assert (~ok).sum() <= oracle_misses, ref["status"]
    assert np.all(out["status"][ok] == 0), (out["status"], out["res"])
    assert np.all(np.abs(out["iter"] - ref["iter"])[ok] <= it_slack), (out["iter"], ref["iter"])
    for i in np.nonzero(ok)[0]:
        for key in ("x", "u"):
            assert helpers.is_approx(out[key][i], ref[key][i], tol), (key, i)


@pytest.mark.parametrize("constraints", ["box_u", "cone"])
def test_srbd_vs_oracle_and_batched(pkg, oracle, constraints):
    """BASELINE configs 3 / 5's SRBD QPs (N = 20, fp64): the latency IPM within 1e-7 of the
    oracle on x, u, in the oracle's iterations +-1, and the batched kernels' solution to the
    solve's accuracy with the same status."""
    qp, x0 = pkg.srbd_model.generate_batch(16, N=20, seed=515, constraints=constraints)
    lat, bat = both(pkg, qp, x0, NMPC, riccati=True, stats=True)
    ref = oracle.solve(qp, NMPC, x0=x0)
    _check_vs_oracle(lat, ref, qp.batch)
    assert np.array_equal(lat["status"], bat["status"])
    assert np.all(np.abs(lat["iter"] - bat["iter"]) <= 1), (lat["iter"], bat["iter"])
    for i in range(qp.batch):
        for key in ("x", "u"):
            assert helpers.is_approx(lat[key][i], bat[key][i], 1e-7), (key, i)
        assert helpers.is_approx(lat["pi"][i, 1:], ref["pi"][i, 1:], 1e-6), ("pi", i)
        assert np.all(lat["res"][i] <= 1e-8), lat["res"][i]


@pytest.mark.parametrize("ng,with_c", [(0, False), (14, False), (14, True)])
@pytest.mark.parametrize("dims", [(12, 12), (12, 4), (5, 3)])
def test_random_constrained_vs_oracle(pkg, oracle, dims, ng, with_c):
    """Boxes on u and x plus general rows (D only, or C and D), embedded dims: the oracle's
    solution at 1e-7 and its iteration counts +-1."""
    nx, nu = dims
    qp, x0 = helpers.random_constrained(12, 15, nx, nu, ng, 41 + nx + ng, pkg.OcpQpBatch)
    if ng and not with_c:  # C-free rows (the friction cone's shape), feasible at u = 0
        qp.C = None
        qp.lg = -0.05 - np.abs(qp.lg)
        qp.ug = 0.05 + np.abs(qp.ug)
    st = dict(NMPC, iter_max=40)
    out = pkg.capi.solve(qp, x0, st)
    ref = oracle.solve(qp, st, x0=x0)
    # (one (12, 4) QP with C rows ends at MaxIter in the oracle (40 iterations) and converges
    # here in 22: measured, seed 67)
    _check_vs_oracle(out, ref, qp.batch, oracle_misses=1 if with_c else 0)
    for i in range(qp.batch):
        assert np.array_equal(out["x"][i, 0], x0[i])


@pytest.mark.parametrize("mode", ["Speed", "Balance"])
def test_zero_c_equals_no_c(pkg, mode):
    """The C-row instantiation of the latency IPM on C = 0 equals the C-free one bit for bit
    (it only adds zeros): a guard on the shipped instantiations' code generation -- the square
    root's C instantiation, not shipped, fails exactly this at -O3."""
    qp, x0 = helpers.random_constrained(12, 15, 12, 12, 14, 167, pkg.OcpQpBatch)
    qz = qp.subset(np.arange(qp.batch))
    qz.C = np.zeros_like(np.asarray(qz.C))
    qn = qp.subset(np.arange(qp.batch))
    qn.C = None
    st = dict(iter_max=40, mode=mode, ric_alg=0)
    with _Path(True):
        rz = pkg.capi.solve(qz, x0, st, stats=True)
        rn = pkg.capi.solve(qn, x0, st, stats=True)
    for key in ("x", "u", "pi", "status", "iter", "res", "stat"):
        assert np.array_equal(rz[key], rn[key]), key


def test_outputs_match_batched(pkg):
    """The whole output set of the two paths on one problem family: res / obj to rounding,
    the Riccati getters P, p, K, k of the last factorization, and the statistics rows
    (alpha_aff, mu_aff, sigma, alpha_prim, alpha_dual, mu, res, obj) of every iteration."""
    qp, x0 = pkg.srbd_model.generate_batch(8, N=20, seed=77, constraints="box_u")
    lat, bat = both(pkg, qp, x0, NMPC, riccati=True, stats=True)
    assert np.array_equal(lat["iter"], bat["iter"]), (lat["iter"], bat["iter"])
    for i in range(qp.batch):
        it = int(lat["iter"][i])
        assert helpers.is_approx(lat["res"][i], bat["res"][i], 1e-2) or np.all(lat["res"][i] < 1e-9)
        assert abs(lat["obj"][i] - bat["obj"][i]) <= 1e-8 * max(1.0, abs(bat["obj"][i]))
        for key in ("P", "K"):
            assert helpers.is_approx(lat[key][i], bat[key][i], 1e-6), (key, i)
        for key in ("p", "k"):
            assert helpers.is_approx(lat[key][i], bat[key][i], 1e-5), (key, i)
        # statistics: early rows agree closely; the last ones carry tolerance-level numbers
        rows = slice(0, max(1, it - 1))
        for col in (0, 1, 2, 3, 4, 5, 10):
            a, b = lat["stat"][i, rows, col], bat["stat"][i, rows, col]
            assert np.allclose(a, b, rtol=1e-6, atol=1e-10), (i, col, a, b)
        assert np.all(lat["stat"][i, it + 2:] == 0.0)


@pytest.mark.parametrize("variant", ["no_pred_corr", "no_split_step", "warm_start", "iter_max"])
def test_setting_variants(pkg, oracle, variant):
    """pred_corr 0, split_step 0, a warm start and a binding iter_max (status MaxIter) run the
    same way on both paths and as the oracle."""
    qp, x0 = pkg.srbd_model.generate_batch(6, N=20, seed=303, constraints="box_u")
    st = dict(NMPC)
    kw = {}
    if variant == "no_pred_corr":
        st["pred_corr"] = 0
        st["iter_max"] = 60
    elif variant == "no_split_step":
        st["split_step"] = 0
    elif variant == "iter_max":
        st["iter_max"] = 3
    else:
        cold = pkg.capi.solve(qp, x0, st)
        st["warm_start"] = 1
        kw = dict(x_init=cold["x"] + 1e-3, u_init=cold["u"] + 1e-3)
    lat, bat = both(pkg, qp, x0, st, **kw)
    assert np.array_equal(lat["status"], bat["status"]), (lat["status"], bat["status"])
    assert np.all(np.abs(lat["iter"] - bat["iter"]) <= 1), (lat["iter"], bat["iter"])
    if variant == "iter_max":
        assert np.all(lat["status"] == 1) and np.all(lat["iter"] == 3)
        for i in range(qp.batch):
            assert helpers.is_approx(lat["x"][i], bat["x"][i], 1e-9)
        return
    if variant != "warm_start":
        ref = oracle.solve(qp, st, x0=x0)
        _check_vs_oracle(lat, ref, qp.batch)
    for i in range(qp.batch):
        assert helpers.is_approx(lat["u"][i], bat["u"][i], 1e-7)


def test_nan_and_batch_one(pkg):
    """A NaN in one QP's data ends that QP with NaNDetected and leaves the others untouched;
    a batch of one solves the same QP as a batch of eight."""
    qp, x0 = pkg.srbd_model.generate_batch(8, N=20, seed=11, constraints="box_u")
    ok = pkg.capi.solve(qp, x0, NMPC)
    bad = qp.subset(np.arange(8))
    bad.Q = bad.Q.copy()
    bad.Q[3, 7, 2, 2] = np.nan
    out = pkg.capi.solve(bad, x0, NMPC)
    assert out["status"][3] == 3, out["status"]
    others = [i for i in range(8) if i != 3]
    assert np.all(out["status"][others] == 0)
    for key in ("x", "u", "pi"):
        assert np.array_equal(out[key][others], ok[key][others]), key
    one = pkg.capi.solve(qp.subset(np.array([5])), x0[5:6], NMPC)
    for key in ("x", "u", "pi", "iter", "status"):
        assert np.array_equal(one[key][0], ok[key][5]), key
    # the NaN QP's outputs are its own (the factorization of its initial iterate, not what a
    # previous solve left in the workspace), in either form of the Riccati recursion
    for ric_alg in (0, 1):
        st = dict(NMPC, ric_alg=ric_alg)
        first = pkg.capi.solve(bad, x0, st, stats=True)
        pkg.capi.solve(qp, x0, st)
        again = pkg.capi.solve(bad.subset(np.array([3])), x0[3:4], st, stats=True)
        for key in ("x", "u", "pi", "status", "iter", "res", "stat"):
            assert np.array_equal(again[key][0], first[key][3], equal_nan=key not in ("status", "iter")), key


@pytest.mark.parametrize("N", [1, 10, 30, 40])
def test_horizons_and_lds_fallback(pkg, oracle, N):
    """Horizons around the LDS budget: N = 1, 10 and 30 run the latency IPM (30: 155 KB of LDS),
    N = 40 does not fit (197 KB) and falls back to the batched kernels; every one solves the
    oracle's QP at 1e-7 in its iterations +-1."""
    qp, x0 = pkg.srbd_model.generate_batch(4, N=N, seed=900 + N, constraints="box_u")
    out = pkg.capi.solve(qp, x0, NMPC)
    ref = oracle.solve(qp, NMPC, x0=x0)
    _check_vs_oracle(out, ref, qp.batch)


def test_many_general_rows(pkg, oracle):
    """ng = 40 (four 12-row chunks per stage, C and D) with boxes on u and x, N = 8."""
    qp, x0 = helpers.random_constrained(6, 8, 12, 12, 40, 77, pkg.OcpQpBatch)
    st = dict(NMPC, iter_max=40)
    out = pkg.capi.solve(qp, x0, st)
    ref = oracle.solve(qp, st, x0=x0)
    _check_vs_oracle(out, ref, qp.batch, oracle_misses=1)


@pytest.mark.parametrize("mode,nmax", [("Balance", 2), ("Robust", 4)])
@pytest.mark.parametrize("dims", [(12, 12, 0, 41), (12, 4, 14, 45), (5, 3, 14, 47)])
def test_itref_forced_corrections_both_paths(pkg, oracle, mode, nmax, dims):
    """HPIPM's iterative refinement of the step (Balance: at most 2 corrections per iteration,
    Robust 4) on the latency IPM (ric_alg 0; the reference test's compareResults runs Balance,
    test/ocp_qp_ipm_solver.cpp:243).  Tolerances of 1e-30 make every check fail, so every
    iteration runs all its corrections: the latency IPM, the batched kernels and the oracle
    (which refines the same way) follow the same iterates to 1e-7, and the stat table counts
    the corrections (column 13, as the batched kernels do) and holds the checks' norms (14, 15)."""
    nx, nu, ng, seed = dims
    qp, x0 = helpers.random_constrained(16, 10, nx, nu, ng, seed, pkg.OcpQpBatch)
    tiny = dict(tol_stat=1e-30, tol_eq=1e-30, tol_ineq=1e-30, tol_comp=1e-30)
    st = dict(NMPC, iter_max=8, mode=mode, **tiny)
    lat, bat = both(pkg, qp, x0, st, stats=True)
    ref = oracle.solve(qp, st, x0=x0)
    assert np.all(lat["status"] == 1) and np.all(bat["status"] == 1), (lat["status"], bat["status"])
    for i in range(qp.batch):
        for key in ("x", "u"):
            assert helpers.is_approx(lat[key][i], ref[key][i], 1e-7), (key, i)
            assert helpers.is_approx(lat[key][i], bat[key][i], 1e-7), (key, i)
    cnt = lat["stat"][:, 1:9, 13]
    assert np.all((cnt >= 1) & (cnt <= nmax)), cnt
    assert np.array_equal(cnt, bat["stat"][:, 1:9, 13]), (cnt, bat["stat"][:, 1:9, 13])
    assert np.all(np.isfinite(lat["stat"][:, 1:9, 14:16])) and np.all(lat["stat"][:, 1:9, 14:16] >= 0)


@pytest.mark.parametrize("mode", ["Balance", "Robust"])
@pytest.mark.parametrize("constraints", ["box_u", "cone"])
def test_itref_srbd_converged(pkg, oracle, mode, constraints):
    """The SRBD QPs of configs 3 / 5 (N = 20, fp64) in Balance / Robust mode on the latency IPM:
    the oracle's solution at 1e-7 in its iterations +-1, the batched kernels' status, and
    residuals at the tolerance."""
    qp, x0 = pkg.srbd_model.generate_batch(16, N=20, seed=616, constraints=constraints)
    st = dict(NMPC, mode=mode)
    lat, bat = both(pkg, qp, x0, st, stats=True)
    ref = oracle.solve(qp, st, x0=x0)
    _check_vs_oracle(lat, ref, qp.batch)
    assert np.array_equal(lat["status"], bat["status"])
    for i in range(qp.batch):
        for key in ("x", "u"):
            assert helpers.is_approx(lat[key][i], bat[key][i], 1e-7), (key, i)
        assert np.all(lat["res"][i] <= 1e-8), lat["res"][i]



SQRT = dict(NMPC, ric_alg=1)


@pytest.mark.parametrize("constraints", ["box_u", "cone"])
@pytest.mark.parametrize("mode", ["Speed", "Balance"])
def test_sqrt_srbd_vs_oracle_and_batched(pkg, oracle, constraints, mode):
    """ric_alg 1 (hpipm-cpp's default, ocp_qp_ipm_solver_settings.hpp:81) on the latency IPM: the
    chain carries the factor Lp of P and s = Lp^-1 p (riccati_step_sqrt's sums of squares on the
    matrix cores, a second Cholesky per stage) and the records keep Lp, so every sweep applies P
    as Lp (Lp' v), as the batched kernels do.  Speed (lq_fact 0) and Balance (lq_fact 1: the
    predictor check passes on these QPs, so they stay on the latency IPM; refinement as above).
    The oracle's square-root solution at 1e-7 in its iterations +-1, the batched kernels' status
    and solution at 1e-7, residuals at the tolerance, the Riccati getters at rounding."""
    qp, x0 = pkg.srbd_model.generate_batch(16, N=20, seed=717, constraints=constraints)
    st = dict(SQRT, mode=mode)
    lat, bat = both(pkg, qp, x0, st, stats=True, riccati=True)
    ref = oracle.solve(qp, st, x0=x0)
    _check_vs_oracle(lat, ref, qp.batch)
    assert np.array_equal(lat["status"], bat["status"])
    assert np.all(bat["stat"][:, :, 11] == 0)  # the batched kernels switched no QP to LQ either
    for i in range(qp.batch):
        for key in ("x", "u"):
            assert helpers.is_approx(lat[key][i], bat[key][i], 1e-7), (key, i)
        # the last factorization's getters: the same iterate to the solve's accuracy; the cone
        # rows' Gamma (~1e8-1e10 when active) amplifies that into K
        tol = 1e-6 if constraints == "box_u" else 1e-3
        for key in ("P", "K"):
            assert helpers.is_approx(lat[key][i], bat[key][i], tol), (key, i)
        assert np.all(lat["res"][i] <= 1e-8), lat["res"][i]


@pytest.mark.parametrize("ng,with_c", [(0, False), (14, False), (14, True)])
@pytest.mark.parametrize("dims", [(12, 12), (12, 4), (5, 3)])
def test_sqrt_random_constrained_vs_oracle(pkg, oracle, dims, ng, with_c):
    """ric_alg 1 Speed on random boxes + general rows (embedded dims): the oracle's square-root
    solution at 1e-7, its iterations +-1.  (Rows with C go to the batched kernels with ric_alg 1:
    on the latency IPM 2 of these 12 QPs stopped at min step, round 6.)"""
    nx, nu = dims
    qp, x0 = helpers.random_constrained(12, 15, nx, nu, ng, 141 + nx + ng, pkg.OcpQpBatch)
    if ng and not with_c:
        qp.C = None
        qp.lg = -0.05 - np.abs(qp.lg)
        qp.ug = 0.05 + np.abs(qp.ug)
    st = dict(SQRT, iter_max=40)
    out = pkg.capi.solve(qp, x0, st)
    ref = oracle.solve(qp, st, x0=x0)
    _check_vs_oracle(out, ref, qp.batch, oracle_misses=1 if with_c else 0)


@pytest.mark.parametrize("dims", [(12, 4, 226), (5, 3, 219)])
def test_sqrt_lq_switch_resolves_those_qps(pkg, dims):
    """lq_fact 1 (Balance's with ric_alg 1, here set explicitly in Speed): a QP whose predictor
    step's linear residual exceeds 1e-5 switches to the LQ factorization, which only the batched
    kernels have.  The latency IPM checks the predictor and ends such a QP with an internal
    status; the C-ABI solves those QPs (and only those) again on the batched kernels.  On random
    boxes + D-only rows (about 27 of these 64 switch, round 6): every QP whose stat column 11
    shows the switch ends exactly as the batched kernels (SRBD_IPM_LATENCY_MAX=0) end it, bit for
    bit; the others stay on the latency IPM (some do); and each QP ends as it does in any batch
    (half the batch solved alone gives the same outputs bit for bit).  5 x 3: embedded in 12 x 12,
    the re-solve pads its compact batch again."""
    nx, nu, seed = dims
    qp, x0 = helpers.random_constrained(64, 15, nx, nu, 14, seed, pkg.OcpQpBatch)
    qp.C = None
    st = dict(iter_max=50, mode="Speed", ric_alg=1, lq_fact=1)
    lat, bat = both(pkg, qp, x0, st, stats=True)
    sw = np.any(lat["stat"][:, :, 11] == 1.0, axis=1)
    assert 0 < sw.sum() < qp.batch, sw.sum()
    assert set(np.unique(lat["status"])) <= {0, 1, 2}, lat["status"]
    for key in ("x", "u", "pi", "status", "iter", "res", "stat"):
        assert np.array_equal(lat[key][sw], bat[key][sw]), key
    both_ok = ~sw & (lat["status"] == 0) & (bat["status"] == 0)
    assert both_ok.sum() >= 8, both_ok.sum()
    for i in np.nonzero(both_ok)[0]:
        for key in ("x", "u"):
            assert helpers.is_approx(lat[key][i], bat[key][i], 1e-6), (key, i)
    half = np.arange(0, qp.batch, 2)
    with _Path(True):
        sub = pkg.capi.solve(qp.subset(half), x0[half], st, stats=True)
    for key in ("x", "u", "pi", "status", "iter", "res", "stat"):
        assert np.array_equal(sub[key], lat[key][half]), key
