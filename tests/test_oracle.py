"""Pin the CPU oracle against the reference's own tests and golden vectors.

* unconstrained: textbook Riccati of hpipm-cpp/test/ocp_qp_ipm_solver.cpp:22-110
  (status Success, iter == 0, x/u/pi/P/-p/K/k at isApprox 1e-10), plus an
  independent dense-KKT solve.
* compareResults: OSQP golden trajectories sol0..14.txt
  (test/ocp_qp_ipm_solver.cpp:170-315) -- box constraints, one-sided masks,
  warm start, 15 closed-loop steps, isApprox 1e-9.
* constrained: test/ocp_qp_ipm_solver.cpp:112-168 (status Success, x[0] == x0)
  plus KKT optimality checks the reference test does not make.
"""
import numpy as np
import pytest

import helpers


@pytest.mark.parametrize("ric_alg", [0, 1])
def test_unconstrained_textbook(OcpQpBatch, oracle, ric_alg):
    """Both Riccati variants (ric_alg 0: classical, 1: square root, the hpipm-cpp
    default) against the reference test's textbook recursion."""
    for seed in range(4):
        qp, x0 = helpers.random_unconstrained(1, 20, 5, 3, seed, OcpQpBatch)
        out = oracle.solve(qp, dict(iter_max=15, ric_alg=ric_alg), x0=x0)
        assert out["status"][0] == 0
        assert out["iter"][0] == 0
        x, u, lmd, P, s, K, k = helpers.textbook_riccati(qp, x0[0])
        prec = 1e-10
        assert helpers.is_approx(out["x"][0, 0], x0[0], 1e-15)
        for i in range(qp.N + 1):
            assert helpers.is_approx(x[i], out["x"][0, i], prec)
            assert helpers.is_approx(lmd[i], out["pi"][0, i], prec)
            assert helpers.is_approx(P[i], out["P"][0, i], prec)
            assert helpers.is_approx(s[i], -out["p"][0, i], prec)
        for i in range(qp.N):
            assert helpers.is_approx(u[i], out["u"][0, i], prec)
            assert helpers.is_approx(K[i], out["K"][0, i], prec)
            assert helpers.is_approx(k[i], out["k"][0, i], prec)


@pytest.mark.parametrize("dims", [(20, 5, 3), (10, 12, 12), (20, 12, 12), (7, 3, 5)])
def test_unconstrained_dense_kkt(OcpQpBatch, oracle, dims):
    N, nx, nu = dims
    qp, x0 = helpers.random_unconstrained(2, N, nx, nu, 11 + nx, OcpQpBatch)
    out = oracle.solve(qp, None, x0=x0)
    for i in range(2):
        x, u, pi = helpers.dense_kkt(qp, x0[i], i)
        assert helpers.is_approx(x, out["x"][i], 1e-9)
        assert helpers.is_approx(u, out["u"][i], 1e-9)
        assert helpers.is_approx(pi[1:], out["pi"][i, 1:], 1e-9)
        assert out["res"][i, 0] < 1e-9 and out["res"][i, 1] < 1e-9


@pytest.mark.parametrize("ric_alg", [0, 1])
def test_compare_results_osqp_golden(OcpQpBatch, oracle, ric_alg):
    """test/ocp_qp_ipm_solver.cpp:170-315 against sol{t}.txt (the reference runs it at
    ric_alg 0; the square-root variant must land on the same goldens)."""
    qp, d, goldens, A, B, b = helpers.quadcopter(OcpQpBatch)
    st = dict(d["settings"], ric_alg=ric_alg)
    N, nx, nu = qp.N, qp.nx, qp.nu
    x = np.zeros(nx)
    xw = np.zeros((1, N + 1, nx))
    uw = np.full((1, N, nu), d["u0"])
    for t in range(d["sim_steps"]):
        out = oracle.solve(qp, st, x0=x[None], x_init=xw, u_init=uw)
        assert out["status"][0] == 0, (t, out["status"][0], out["res"][0])
        cat = np.concatenate([out["x"][0].ravel(), out["u"][0].ravel()])
        assert helpers.is_approx(cat, goldens[t], d["rel_prec"]), (
            t, np.linalg.norm(cat - goldens[t]) / np.linalg.norm(goldens[t]))
        xw, uw = out["x"], out["u"]  # warm start from the previous solution
        x = A @ x + B @ out["u"][0, 0] + b


@pytest.mark.parametrize("ng", [0, 2])
def test_constrained_kkt(OcpQpBatch, oracle, ng):
    qp, x0 = helpers.random_constrained(3, 20, 5, 3, ng, 5 + ng, OcpQpBatch)
    st = dict(iter_max=30)  # hpipm-cpp default tolerances (1e-8), settings.hpp:26-86
    out = oracle.solve(qp, st, x0=x0)
    for i in range(3):
        assert out["status"][i] == 0, out["res"][i]
        assert helpers.is_approx(out["x"][i, 0], x0[i], 1e-15)
        assert np.all(out["res"][i] <= 1e-8)
        # primal feasibility of the box constraints
        u = out["u"][i]
        assert np.all(u[:, :3] >= qp.lbu[i][:, :3] - 1e-9) and np.all(u[:, :3] <= qp.ubu[i][:, :3] + 1e-9)


def test_constrained_matches_unconstrained_when_inactive(OcpQpBatch, oracle):
    """Far-away bounds: the IPM must land on the unconstrained Riccati solution."""
    qp, x0 = helpers.random_unconstrained(2, 15, 6, 4, 3, OcpQpBatch)
    ref = oracle.solve(qp, None, x0=x0)
    qp.lbu = np.full((2, 15, 4), -1e4); qp.ubu = np.full((2, 15, 4), 1e4)
    out = oracle.solve(qp, dict(iter_max=60, tol_stat=1e-12, tol_eq=1e-12, tol_ineq=1e-12,
                                tol_comp=1e-9), x0=x0)
    assert np.all(out["status"] == 0)
    for i in range(2):
        assert helpers.is_approx(out["x"][i], ref["x"][i], 1e-8)
        assert helpers.is_approx(out["u"][i], ref["u"][i], 1e-8)


@pytest.mark.parametrize("threads", [1, 3])
def test_fast_unconstr_port_matches_oracle(pkg, oracle, threads):
    """The cpu_baseline port (oracle/fast_unconstr.c, fixed 12 x 12) computes the oracle's
    x, u, pi on SRBD QPs and on the reference test's random QPs (12 x 12)."""
    qp, x0 = pkg.srbd_model.generate_batch(7, N=20, seed=1003)
    ref = oracle.solve(qp, None, x0=x0)
    out, _ = oracle.fast_unconstr_batch(qp, x0, threads=threads)
    for key in ("x", "u", "pi"):
        assert helpers.is_approx(out[key], ref[key], 1e-10), key
    qp, x0 = helpers.random_unconstrained(5, 10, 12, 12, 77, pkg.OcpQpBatch)
    ref = oracle.solve(qp, None, x0=x0)
    out, _ = oracle.fast_unconstr_batch(qp, x0, threads=threads)
    for key in ("x", "u", "pi"):
        assert helpers.is_approx(out[key], ref[key], 1e-10), key


@pytest.mark.parametrize("ng", [0, 14])
def test_itref_oracle(OcpQpBatch, oracle, ng):
    """The oracle's restatement of HPIPM's iterative refinement of the corrector (mode
    Balance: 2 corrections at most, Robust: 4).  At the default tolerances
    the refined solve lands on the unrefined one; with tolerances nothing reaches, every
    iteration refines and the iterates move only at the linear solve's rounding level."""
    qp, x0 = helpers.random_constrained(4, 10, 12, 4, ng, 45 + ng, OcpQpBatch)
    speed = oracle.solve(qp, dict(iter_max=40, mode="Speed"), x0=x0)
    for mode in ("Balance", "Robust"):
        out = oracle.solve(qp, dict(iter_max=40, mode=mode), x0=x0)
        assert np.all(out["status"] == 0) and np.all(speed["status"] == 0)
        assert np.all(out["res"] <= 1e-8)
        for i in range(qp.batch):
            assert helpers.is_approx(out["u"][i], speed["u"][i], 1e-7), (mode, i)
    tiny = dict(iter_max=6, tol_stat=1e-30, tol_eq=1e-30, tol_ineq=1e-30, tol_comp=1e-30)
    ref = oracle.solve(qp, dict(tiny, itref_corr_max=2), x0=x0)
    plain = oracle.solve(qp, dict(tiny, itref_corr_max=0), x0=x0)
    for i in range(qp.batch):
        assert helpers.is_approx(ref["u"][i], plain["u"][i], 1e-6), i


@pytest.mark.parametrize("ric_alg", [0, 1])
@pytest.mark.parametrize("dims", [(12, 12, 0), (6, 4, 3), (12, 12, 4)])
def test_lq_fact_oracle(OcpQpBatch, oracle, dims, ric_alg):
    """The oracle's restatement of HPIPM's lq_fact (the stage factor by an LQ
    factorization of [chol(RSQ) | sqrt(Gamma) rows | [B'; A'] Lx_{k+1}], Gamma never added to
    the data).  lq_fact 2 takes the same iterations as the Cholesky and lands on its solution
    at rounding level; lq_fact 1 keeps the Cholesky while the predictor's linear residual stays
    below 1e-5, which it does on these regular QPs.  With the classical Riccati lq_fact is
    ignored, as in HPIPM ("for square_root_alg==1").  (HPIPM is not vendored: parity against
    HPIPM itself is unpinned; tests/test_gpu_lq.py holds the HIP library to this restatement.)"""
    nx, nu, ng = dims
    qp, x0 = helpers.random_constrained(8, 10, nx, nu, ng, 5, OcpQpBatch)
    base = dict(iter_max=30, ric_alg=ric_alg)
    chol = oracle.solve(qp, base, x0=x0)
    if ric_alg == 0:  # lq_fact belongs to the square-root Riccati: ignored with the classical one
        lq = oracle.solve(qp, dict(base, lq_fact=2), x0=x0)
        assert np.all(lq["lq_iters"] == 0) and np.array_equal(lq["u"], chol["u"])
        return
    assert np.all(chol["status"] == 0) and np.all(chol["lq_iters"] == 0)
    lq = oracle.solve(qp, dict(base, lq_fact=2), x0=x0)
    assert np.array_equal(lq["status"], chol["status"]) and np.array_equal(lq["iter"], chol["iter"])
    assert np.array_equal(lq["lq_iters"], lq["iter"])
    # x, u agree to ~1e-11 (measured); pi, the dynamics multipliers, only to the stationarity
    # tolerance scaled by the active bounds' barrier weights (measured up to 3e-6)
    for i in range(qp.batch):
        for key, tol in (("x", 1e-9), ("u", 1e-9), ("pi", 1e-5)):
            assert helpers.is_approx(lq[key][i], chol[key][i], tol), (key, i)
    mix = oracle.solve(qp, dict(base, lq_fact=1), x0=x0)
    assert np.all(mix["lq_iters"] == 0)
    assert np.array_equal(mix["u"], chol["u"])


def test_lq_fact_oracle_degenerate_endgame(OcpQpBatch, oracle):
    """The near-degenerate family of tests/test_gpu_ipm.py test_degenerate_endgame_family (QP
    #12 of (12, 4, 14) seed 200, 64 copies perturbed at 1e-15) in Speed with the square-root
    Riccati in HPIPM's form (the carried joint stage factor): the Cholesky converges on 48 of 64
    (measured; the rest stop at min step once the unrefined step's linear residual, ~eps x the
    1e13 barrier Hessians, passes tol_stat -- DESIGN.md 4.4), the LQ factorization, which never
    forms the ~1e13 barrier sums, on all 64 in 13-14 iterations.  lq_fact 1 switches on the copies
    whose predictor residual exceeds 1e-5 -- in Speed (no refinement) only once a stalled
    Cholesky step has already been taken, so it does not rescue them; Balance adds the
    refinement that does."""
    qp, x0 = helpers.random_constrained(20, 12, 12, 4, 14, 200, OcpQpBatch)
    M = 64
    rng = np.random.default_rng(7)
    fields = {}
    for name in ("Q", "R", "S", "A", "B", "q", "r", "b", "C", "D", "lg", "ug", "lbu", "ubu", "lbx",
                 "ubx", "lg_mask", "ug_mask", "lbu_mask", "ubu_mask", "lbx_mask", "ubx_mask"):
        a = getattr(qp, name, None)
        if a is None:
            continue
        a = np.repeat(np.asarray(a)[12:13], M, axis=0)
        if name in ("Q", "R", "S", "A", "B", "q", "r", "b"):
            a = a * (1 + 1e-15 * rng.standard_normal(a.shape))
        fields[name] = a
    fam = OcpQpBatch(N=qp.N, nx=qp.nx, nu=qp.nu, ng=qp.ng, **fields)
    xb = np.repeat(np.asarray(x0)[12:13], M, axis=0)
    st = dict(iter_max=50, mode="Speed", ric_alg=1)
    chol = oracle.solve(fam, st, x0=xb)
    lq = oracle.solve(fam, dict(st, lq_fact=2), x0=xb)
    mix = oracle.solve(fam, dict(st, lq_fact=1), x0=xb)
    assert (chol["status"] == 0).sum() >= 44
    assert (lq["status"] == 0).sum() == 64 and np.all(lq["iter"] <= 14)
    assert mix["lq_iters"].sum() > 0 and np.all(mix["lq_iters"][mix["iter"] <= 13] == 0)
    for i in range(M):
        if chol["status"][i] == 0:
            assert helpers.is_approx(lq["u"][i], chol["u"][i], 1e-6), i
