"""Parity at BASELINE.json's full sizes (65536 SRBD QPs per GPU, N = 20 / 40).

The oracle is too slow for a whole 65536-QP batch, so at full size the HIP path is
checked through size-independent properties of every QP of the batch, computed
in torch fp64 on the device from the same input buffers the kernel read:

* the KKT conditions of the solution (dynamics, stationarity in u and x with the
  multiplier convention of SURVEY 8 a12: pi_{k+1} multiplies x_{k+1} = A x + B u + b);
* bounds and the solver's own residual report for the IPM configurations;

and by oracle parity on windows of QPs spread over the batch (first, middle, last),
copied back from the device buffers so the oracle sees bit-identical inputs.
"""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)
TIGHT = dict(iter_max=40, tol_stat=1e-8, tol_eq=1e-8, tol_ineq=1e-8, tol_comp=1e-8, split_step=1)
F32 = dict(iter_max=30, tol_stat=3e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1)
SEED = 1003
BATCH = 65536
WINDOWS = (slice(0, 8), slice(BATCH // 2 - 4, BATCH // 2 + 4), slice(BATCH - 8, BATCH))


def device_batch(pkg, N, constraints, batch=BATCH, seed=SEED):
    """Every QP distinct: linearisation points from seed + global index, linearised
    on the device (the bench's generator)."""
    import torch
    ng = 24 if constraints == "cone" else 0
    h = pkg.capi.Handle(N, 12, 12, ng, constraints == "box_u", False, capacity=batch)
    xs, us, x0 = pkg.srbd_model.sample_trajectories(batch, N, seed, pkg.srbd_model.SrbdParams())
    xs_t, us_t = torch.from_numpy(xs).cuda(), torch.from_numpy(us).cuda()
    t, _ = pkg.capi.srbd_linearize(h, xs_t, us_t, constraints)
    h.synchronize()
    t["x0"] = torch.from_numpy(np.ascontiguousarray(x0)).cuda()
    return h, t


def solve_on_device(pkg, h, t, N, settings, dtype="f64"):
    import torch
    batch = t["x0"].shape[0]
    tt = torch.float32 if dtype == "f32" else torch.float64
    tin = {k: (None if v is None else v.to(tt).contiguous()) for k, v in t.items()}
    sol_t = {"x": torch.zeros(batch, N + 1, 12, dtype=tt, device="cuda"),
             "u": torch.zeros(batch, N, 12, dtype=tt, device="cuda"),
             "pi": torch.zeros(batch, N + 1, 12, dtype=tt, device="cuda"),
             "status": torch.zeros(batch, dtype=torch.int32, device="cuda"),
             "iter": torch.zeros(batch, dtype=torch.int32, device="cuda"),
             "res": torch.zeros(batch, 4, dtype=tt, device="cuda")}
    DataT, SolT = ((pkg.capi.Data32, pkg.capi.Solution32) if dtype == "f32"
                   else (pkg.capi.Data, pkg.capi.Solution))
    data = DataT(**{k: (None if tin.get(k) is None else tin[k].data_ptr())
                    for k in pkg.capi.DATA_FIELDS})
    sol = SolT(**{k: (sol_t[k].data_ptr() if k in sol_t else None) for k in pkg.capi.SOL_FIELDS})
    h.solve_device(batch, pkg.capi.settings_struct(settings), data, sol)
    h.synchronize()
    return {k: v.double() if v.is_floating_point() else v for k, v in sol_t.items()}


def blocks(t, N):
    """Row-major views of the column-major C-ABI blocks (torch, fp64)."""
    B = t["x0"].shape[0]
    cm = lambda v, n, r, c: v.view(B, n, c, r).transpose(-1, -2)
    return {"A": cm(t["A"], N, 12, 12), "B": cm(t["B"], N, 12, 12), "b": t["b"].view(B, N, 12),
            "Q": cm(t["Q"], N + 1, 12, 12), "S": cm(t["S"], N, 12, 12),
            "R": cm(t["R"], N, 12, 12), "q": t["q"].view(B, N + 1, 12), "r": t["r"].view(B, N, 12)}


def kkt_residuals(m, s, x0):
    """Relative KKT residuals of every QP: each residual divided by the sum of the
    magnitudes of its terms (so cancellation in large terms is not mistaken for error)."""
    import torch
    x, u, pi = s["x"], s["u"], s["pi"]
    mv = lambda M, v: torch.einsum("bkij,bkj->bki", M, v)
    mtv = lambda M, v: torch.einsum("bkji,bkj->bki", M, v)
    ab = lambda M: M.abs()
    # dynamics x_{k+1} = A x_k + B u_k + b_k, x_0 = x0
    dyn = x[:, 1:] - (mv(m["A"], x[:, :-1]) + mv(m["B"], u) + m["b"])
    dyn_s = x[:, 1:].abs() + mv(ab(m["A"]), x[:, :-1].abs()) + mv(ab(m["B"]), u.abs()) + m["b"].abs()
    # u: R u + S x + r + B' pi_{k+1} = 0
    gu = mv(m["R"], u) + mv(m["S"], x[:, :-1]) + m["r"] + mtv(m["B"], pi[:, 1:])
    gu_s = (mv(ab(m["R"]), u.abs()) + mv(ab(m["S"]), x[:, :-1].abs()) + m["r"].abs()
            + mtv(ab(m["B"]), pi[:, 1:].abs()))
    # x, stages 1..N-1: Q x + S' u + q + A' pi_{k+1} - pi_k = 0 ; stage N: Q x + q - pi_N = 0
    Q, q = m["Q"], m["q"]
    gx = (mv(Q[:, 1:-1], x[:, 1:-1]) + mtv(m["S"][:, 1:], u[:, 1:]) + q[:, 1:-1]
          + mtv(m["A"][:, 1:], pi[:, 2:]) - pi[:, 1:-1])
    gx_s = (mv(ab(Q[:, 1:-1]), x[:, 1:-1].abs()) + mtv(ab(m["S"][:, 1:]), u[:, 1:].abs())
            + q[:, 1:-1].abs() + mtv(ab(m["A"][:, 1:]), pi[:, 2:].abs()) + pi[:, 1:-1].abs())
    gN = torch.einsum("bij,bj->bi", Q[:, -1], x[:, -1]) + q[:, -1] - pi[:, -1]
    gN_s = torch.einsum("bij,bj->bi", Q[:, -1].abs(), x[:, -1].abs()) + q[:, -1].abs() + pi[:, -1].abs()
    x0err = (x[:, 0] - x0).abs().max().item()
    rel = lambda r, sc: (r.abs() / (sc + 1e-300)).amax(dim=tuple(range(1, r.dim())))
    return {"x0": x0err, "dyn": rel(dyn, dyn_s), "gu": rel(gu, gu_s), "gx": rel(gx, gx_s),
            "gN": rel(gN, gN_s), "abs_gu": gu.abs().amax(dim=(1, 2)), "abs_dyn": dyn.abs().amax(dim=(1, 2))}


def host_subset(pkg, t, N, constraints, idx):
    """OcpQpBatch of QPs `idx` holding exactly the device buffers' numbers."""
    n = len(range(*idx.indices(t["x0"].shape[0])))
    g = lambda k: t[k][idx].cpu().numpy()
    cm = lambda k, nb, r, c: np.swapaxes(g(k).reshape(n, nb, c, r), -1, -2).copy()
    kw = dict(A=cm("A", N, 12, 12), B=cm("B", N, 12, 12), b=g("b").reshape(n, N, 12),
              Q=cm("Q", N + 1, 12, 12), S=cm("S", N, 12, 12), R=cm("R", N, 12, 12),
              q=g("q").reshape(n, N + 1, 12), r=g("r").reshape(n, N, 12))
    qp = pkg.OcpQpBatch(N=N, nx=12, nu=12, **kw)
    if constraints == "box_u":
        for k in ("lbu", "ubu"):
            setattr(qp, k, g(k).reshape(n, N, 12))
        for k in ("lbu_mask", "ubu_mask"):
            if t.get(k) is not None:
                setattr(qp, k, g(k).reshape(n, N, 12))
    if constraints == "cone":
        qp.ng = 24
        qp.D = np.swapaxes(g("D").reshape(n, N, 12, 24), -1, -2).copy()
        for k in ("lg", "ug", "lg_mask", "ug_mask"):
            setattr(qp, k, g(k).reshape(n, N + 1, 24))
    return qp, t["x0"][idx].cpu().numpy()


def test_unconstrained_full_batch_kkt_and_oracle_windows(pkg, oracle):
    """Config 3's batch without bounds (the reference NMPC QP, the bench default):
    every QP satisfies its KKT system to 1e-10 relative to the magnitude of its terms
    (reg_prim = 0: the default 1e-12 on the pivots of G shifts R u by 1e-12 u, which
    is ~2e-9 of the SRBD terms, R ~ 1e-4 -- the oracle does the same); three windows
    equal the oracle at 1e-10 (the unconstrained tolerance of SURVEY 8(c))."""
    import torch
    N = 20
    h, t = device_batch(pkg, N, "none")
    st = dict(NMPC, reg_prim=0.0)
    s = solve_on_device(pkg, h, t, N, st)
    assert int((s["status"] != 0).sum()) == 0
    r = kkt_residuals(blocks(t, N), s, t["x0"])
    assert r["x0"] == 0.0
    for k in ("dyn", "gu", "gx", "gN"):
        worst = r[k].max().item()
        assert worst < 1e-10, (k, worst, int(torch.argmax(r[k])))
    for w in WINDOWS:
        qp, x0 = host_subset(pkg, t, N, "none", w)
        ref = oracle.solve(qp, st, x0=x0)
        for k in ("x", "u", "pi"):
            got = s[k][w].cpu().numpy()
            assert helpers.is_approx(got, ref[k], 1e-10), (k, w)


def test_config2_n10_b4096_kkt_and_oracle_windows(pkg, oracle):
    """BASELINE config 2 at its stated size: 4096 SRBD QPs, N = 10 (the one-lane-group-
    per-QP bring-up shape: 1 wave per SIMD on the chip).  Every QP satisfies its KKT
    system to 1e-10 relative to its terms (reg_prim = 0, as above) and three windows
    across the batch equal the oracle at 1e-10."""
    import torch
    N, batch = 10, 4096
    h, t = device_batch(pkg, N, "none", batch=batch)
    st = dict(NMPC, reg_prim=0.0)
    s = solve_on_device(pkg, h, t, N, st)
    assert int((s["status"] != 0).sum()) == 0
    assert int((s["iter"] != 0).sum()) == 0  # nc = 0: one Riccati sweep, iter 0
    r = kkt_residuals(blocks(t, N), s, t["x0"])
    assert r["x0"] == 0.0
    for k in ("dyn", "gu", "gx", "gN"):
        worst = r[k].max().item()
        assert worst < 1e-10, (k, worst, int(torch.argmax(r[k])))
    for w in (slice(0, 8), slice(batch // 2 - 4, batch // 2 + 4), slice(batch - 8, batch)):
        qp, x0 = host_subset(pkg, t, N, "none", w)
        ref = oracle.solve(qp, st, x0=x0)
        for k in ("x", "u", "pi"):
            got = s[k][w].cpu().numpy()
            assert helpers.is_approx(got, ref[k], 1e-10), (k, w)


def test_box_u_full_batch(pkg, oracle):
    """Config 3 (box on u, IPM, NMPC settings): every QP converges, stays inside its
    bounds, satisfies the dynamics to tol_eq, reports residuals below the
    tolerances; at tight tolerances three windows equal the oracle."""
    import torch
    N = 20
    h, t = device_batch(pkg, N, "box_u")
    s = solve_on_device(pkg, h, t, N, NMPC)
    st = s["status"].cpu().numpy()
    assert np.all(st == 0), np.bincount(st)
    it = s["iter"].cpu().numpy()
    assert 1 <= it.min() and it.max() <= NMPC["iter_max"]
    res = s["res"].cpu().numpy()
    tol = np.array([NMPC["tol_stat"], NMPC["tol_eq"], NMPC["tol_ineq"], NMPC["tol_comp"]])
    assert np.all(res <= tol), res.max(0)
    m = blocks(t, N)
    r = kkt_residuals(m, s, t["x0"])
    assert r["x0"] == 0.0
    assert r["abs_dyn"].max().item() <= NMPC["tol_eq"]
    B = t["x0"].shape[0]
    lb, ub, u = t["lbu"].view(B, N, 12), t["ubu"].view(B, N, 12), s["u"]
    assert torch.all(u >= lb - NMPC["tol_ineq"]) and torch.all(u <= ub + NMPC["tol_ineq"])
    # stationarity in u, away from the bounds (the multipliers there are <= mu / slack)
    free = (u - lb > 1.0) & (ub - u > 1.0)
    gu = (torch.einsum("bkij,bkj->bki", m["R"], u) + torch.einsum("bkij,bkj->bki", m["S"], s["x"][:, :-1])
          + m["r"] + torch.einsum("bkji,bkj->bki", m["B"], s["pi"][:, 1:]))
    assert gu[free].abs().max().item() < 1e-3
    # tight tolerances: iterate-level parity with the oracle on windows across the batch
    s2 = solve_on_device(pkg, h, t, N, TIGHT)
    assert np.all(s2["status"].cpu().numpy() == 0)
    for w in WINDOWS:
        qp, x0 = host_subset(pkg, t, N, "box_u", w)
        ref = oracle.solve(qp, TIGHT, x0=x0)
        assert np.all(ref["status"] == 0)
        for k in ("x", "u"):
            got = s2[k][w].cpu().numpy()
            np.testing.assert_allclose(got, ref[k], rtol=1e-6, atol=1e-7 * np.abs(ref[k]).max(),
                                       err_msg=f"{k} window {w}")


def test_cone_n40_fp32_full_batch(pkg, oracle):
    """Config 5 (N = 40, friction-cone rows, fp32): the fp32 tolerances of DESIGN 4.5
    are met by >= 98.5% of the batch (99.1% measured, f64_rescue = 0), every solution is finite, satisfies the fp32
    dynamics to tol_eq and the cone rows to tol_ineq; windows stay within the fp32
    KKT tolerance of the fp64 oracle solution."""
    import torch
    N = 40
    h, t = device_batch(pkg, N, "cone")
    s = solve_on_device(pkg, h, t, N, F32, dtype="f32")
    st = s["status"].cpu().numpy()
    assert (st == 0).mean() >= 0.985, np.bincount(st)
    assert set(np.unique(st)) <= {0, 1, 2}  # never NaNDetected
    for k in ("x", "u", "pi"):
        assert bool(torch.isfinite(s[k]).all()), k
    B = t["x0"].shape[0]
    m = blocks(t, N)
    r = kkt_residuals(m, s, t["x0"].float().double())
    ok = torch.from_numpy(st == 0).cuda()
    assert r["abs_dyn"][ok].max().item() <= 10 * F32["tol_eq"]
    D = t["D"].view(B, N, 12, 24).transpose(-1, -2)  # 24 x 12 row-major
    v = torch.einsum("bkij,bkj->bki", D, s["u"])
    lg = t["lg"].view(B, N + 1, 24)[:, :N]
    assert (lg - v)[ok].max().item() <= 10 * F32["tol_ineq"]
    ru = []
    for w in WINDOWS:
        qp, x0 = host_subset(pkg, t, N, "cone", w)
        ref = oracle.solve(qp, NMPC, x0=x0)
        assert np.all(ref["status"] == 0)
        got = s["u"][w].cpu().numpy()
        ru += [np.linalg.norm(got[i] - ref["u"][i]) / np.linalg.norm(ref["u"][i])
               for i in np.nonzero(st[w] == 0)[0]]
    # the bound of tests/test_gpu_fp32.py (fp32 iterate at fp32 tolerances vs fp64 at 1e-4)
    assert np.median(ru) <= 3e-3 and np.max(ru) <= 2e-2, (np.median(ru), np.max(ru))


def test_repeated_solves_bitwise_identical(pkg):
    """The same inputs solved three times on one handle, each time from freshly
    converted torch buffers and freshly zeroed outputs: bit-identical results.
    (Guards the ordering of the handle's stream after torch's stream: without it
    the solve raced the fp64 -> fp32 conversion and the zero fill of x / u.)"""
    N = 40
    h, t = device_batch(pkg, N, "cone", batch=16384)
    outs = [solve_on_device(pkg, h, t, N, F32, dtype="f32") for _ in range(3)]
    for o in outs[1:]:
        for k in ("x", "u", "pi", "status", "iter"):
            assert bool((o[k] == outs[0][k]).all()), k
