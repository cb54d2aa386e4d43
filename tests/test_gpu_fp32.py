"""fp32 twins (srbd_qp_solve_f32; BASELINE config 5, HPIPM's s_ocp_qp_ipm) against
the fp64 oracle.  fp32 carries ~7 digits, so the bar is the accuracy the fp32
arithmetic supports, stated per test: relative 1e-4 for the Riccati solve (one
sweep, no iteration), and for the IPM the NMPC tolerance (1e-4 KKT residual,
NMPC_solver.cpp:74-77) reached with status Success plus agreement with the fp64
solution at 1e-3 relative."""
import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)


def test_unconstrained_fp32_vs_oracle(pkg, oracle):
    qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=91, constraints="none")
    out = pkg.capi.solve(qp, x0, dtype=np.float32, riccati=True)
    ref = oracle.solve(qp, {}, x0=x0)
    assert out["x"].dtype == np.float32
    assert np.all(out["status"] == 0)
    for i in range(qp.batch):
        for key in ("x", "u", "pi"):
            assert helpers.is_approx(out[key][i].astype(np.float64), ref[key][i], 1e-4), (key, i)


def test_box_u_fp32_vs_fp64(pkg):
    qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=92, constraints="box_u")
    o32 = pkg.capi.solve(qp, x0, NMPC, dtype=np.float32)
    o64 = pkg.capi.solve(qp, x0, NMPC)
    assert np.all(o64["status"] == 0)
    # (measured r03: 64 / 64 Success, u within 8.9e-4 and x within 6.6e-4 of fp64)
    assert np.all(o32["status"] == 0), o32["status"]
    ok = o32["status"] == 0
    assert np.all(o32["res"][ok] <= 1e-4)
    for i in np.nonzero(ok)[0]:
        assert helpers.is_approx(o32["u"][i].astype(np.float64), o64["u"][i], 1e-3), i
        assert helpers.is_approx(o32["x"][i].astype(np.float64), o64["x"][i], 1e-3), i


# fp32 stationarity floor: with forces ~1e2 and barrier curvature ~1e3 in R, an
# fp32 iterate carries |R| ulp(u) ~ 1e-2 of res_stat, so the fp32 path is run at
# fp32-reachable tolerances; HPIPM's s_ocp_qp_ipm has the same floor.
F32 = dict(iter_max=30, tol_stat=1e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1)


def test_friction_cone_fp32_vs_oracle(pkg, oracle):
    qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=93, constraints="cone")
    o32 = pkg.capi.solve(qp, x0, F32, dtype=np.float32)
    ref = oracle.solve(qp, NMPC, x0=x0)
    assert np.all(ref["status"] == 0)
    # (measured r03: 63 / 64 Success, one MinStepLengthReached at the fp32 floor)
    assert (o32["status"] == 0).sum() >= 63, np.bincount(o32["status"])
    ok = o32["status"] == 0
    assert np.all(o32["res"][ok][:, 0] <= F32["tol_stat"])
    assert np.all(o32["res"][ok][:, 1:] <= 1e-3)
    # the fp32 KKT point at tol_stat 1e-2 differs from the fp64 one at 1e-4 by the
    # tolerance / curvature, not by rounding: bound the typical and the worst error
    # (measured r03: median 2.9e-3 / max 1.2e-2 in u, 2.3e-3 / 1.5e-2 in x)
    ru = [np.linalg.norm(o32["u"][i] - ref["u"][i]) / np.linalg.norm(ref["u"][i])
          for i in np.nonzero(ok)[0]]
    rx = [np.linalg.norm(o32["x"][i] - ref["x"][i]) / np.linalg.norm(ref["x"][i])
          for i in np.nonzero(ok)[0]]
    assert np.median(ru) <= 5e-3 and np.max(ru) <= 3e-2, (np.median(ru), np.max(ru))
    assert np.median(rx) <= 5e-3 and np.max(rx) <= 3e-2, (np.median(rx), np.max(rx))


def test_friction_cone_n40_fp32(pkg):
    """BASELINE config 5's problem class: N = 40, 24 friction-cone rows per stage;
    status Success on >= 99 % of QPs at tol_stat 3e-2 with f64_rescue = 0 (the stage
    factorization runs in fp64; before that 92.6 % here, the rest stopping
    at the fp32 floor with MinStepLengthReached), fp64 reaches 1e-4 on all."""
    qp, x0 = pkg.srbd_model.generate_batch(256, N=40, seed=93, constraints="cone")
    st = dict(F32, tol_stat=3e-2)
    o32 = pkg.capi.solve(qp, x0, st, dtype=np.float32)
    o64 = pkg.capi.solve(qp, x0, NMPC)
    assert np.all(o64["status"] == 0)
    assert np.mean(o32["status"] == 0) >= 0.99, np.bincount(o32["status"])
    assert np.all(o32["status"] <= 2)  # no NaN at these settings
    ok = o32["status"] == 0
    ru = [np.linalg.norm(o32["u"][i] - o64["u"][i]) / np.linalg.norm(o64["u"][i])
          for i in np.nonzero(ok)[0]]
    # (measured r03: median 1.5e-3, max 7.2e-3)
    assert np.median(ru) <= 3e-3 and np.max(ru) <= 2e-2, (np.median(ru), np.max(ru))


def _rounded_to_f32(qp):
    """The same batch with every array rounded to fp32 (what the fp32 path reads)."""
    import dataclasses
    kw = {}
    for f in dataclasses.fields(qp):
        v = getattr(qp, f.name)
        kw[f.name] = v.astype(np.float32).astype(np.float64) if isinstance(v, np.ndarray) else v
    return type(qp)(**kw)


@pytest.mark.parametrize("cap,stats,batch", [(30, False, 512), (30, True, 512), (12, False, 512),
                                             (12, False, 2500)])
def test_f64_rescue_cone_n40(pkg, cap, stats, batch):
    """settings.f64_rescue = cap: the fp32 pass runs at most `cap` iterations, and the
    QPs it leaves unsolved continue in fp64 from the iterate it ended on (x, u, pi and
    the barrier state: HPIPM's warm_start = 2).  Every QP ends with status Success
    within the tolerances; the QPs fp32 solved keep their fp32 outputs bit for bit (an
    fp32 solve with iter_max = cap); the rescued ones land at the fp64 KKT point to the
    accuracy the stationarity tolerance allows (the bound of test_friction_cone_n40_fp32),
    each either continued in fewer fp64 iterations than its cold fp64 solve or -- when the
    continuation does not converge (an fp32 pass can end with its barrier collapsed far
    from the solution) -- solved again cold in fp64: then exactly the cold fp64 solve of
    its fp32-rounded data.  batch 2500: the unsolved-QP list spans three ragged 1024-QP
    tiles of the selection kernel."""
    qp, x0 = pkg.srbd_model.generate_batch(batch, N=40, seed=1005, constraints="cone")
    st = dict(F32, tol_stat=3e-2)
    plain = pkg.capi.solve(qp, x0, dict(st, iter_max=cap), dtype=np.float32, riccati=True,
                           stats=stats)
    resc = pkg.capi.solve(qp, x0, dict(st, f64_rescue=cap), dtype=np.float32, riccati=True,
                          stats=stats)
    o64 = pkg.capi.solve(qp, x0, NMPC)
    bad = plain["status"] != 0
    assert bad.any(), "seed 1005 at N = 40 has fp32 failures (DESIGN.md 4.5)"
    assert np.all(o64["status"] == 0)
    assert np.all(resc["status"] == 0), np.bincount(resc["status"])
    keys = ["x", "u", "pi", "P", "p", "K", "k", "iter", "res", "obj"] + (["stat"] if stats else [])
    for key in keys:
        assert np.array_equal(resc[key][~bad], plain[key][~bad]), key
    assert np.all(resc["res"][bad][:, 0] <= st["tol_stat"])
    assert np.all(resc["res"][bad][:, 1:] <= 1e-3)
    ru = [np.linalg.norm(resc["u"][i] - o64["u"][i]) / np.linalg.norm(o64["u"][i])
          for i in np.nonzero(bad)[0]]
    # (measured r03: median 5e-5..1.9e-4, max 6.6e-4 at cap 12 and 2.0e-3 at cap 30)
    assert np.median(ru) <= 1e-3 and np.max(ru) <= 5e-3, (np.median(ru), np.max(ru))
    # continued in fewer iterations than a cold fp64 solve, or re-solved cold
    cold = pkg.capi.solve(_rounded_to_f32(qp), x0.astype(np.float32).astype(np.float64), st)
    n_cont = 0
    for i in np.nonzero(bad)[0]:
        same = all(np.array_equal(resc[k][i], cold[k][i].astype(np.float32)) for k in ("x", "u", "pi"))
        if not same:
            assert resc["iter"][i] < o64["iter"][i], (i, resc["iter"][i], o64["iter"][i])
            n_cont += 1
        else:
            assert resc["iter"][i] == cold["iter"][i], i
    assert n_cont >= 1, "no rescued QP was continued"


def test_f64_rescue_padded_is_a_cold_fp64_solve(pkg):
    """nx, nu < 12 (the 12 x 12 embedding): the rescue re-solves cold, so a rescued QP's
    outputs are exactly the fp64 solve of its fp32-rounded data, narrowed (per-QP
    arithmetic does not depend on the QP's place in a batch).  fp32 cannot reach tol
    1e-8, so every QP is rescued."""
    qp, x0 = helpers.random_constrained(64, 8, 8, 4, 6, 31, pkg.OcpQpBatch)
    st = dict(iter_max=30, tol_stat=1e-8, tol_eq=1e-8, tol_ineq=1e-8, tol_comp=1e-8)
    plain = pkg.capi.solve(qp, x0, st, dtype=np.float32)
    resc = pkg.capi.solve(qp, x0, dict(st, f64_rescue=30), dtype=np.float32, riccati=True)
    o64 = pkg.capi.solve(_rounded_to_f32(qp), x0.astype(np.float32).astype(np.float64), st,
                         riccati=True)
    bad = plain["status"] != 0
    assert bad.mean() > 0.5
    assert np.all(o64["status"] == 0) and np.all(resc["status"] == 0)
    for key in ["x", "u", "pi", "P", "p", "K", "k", "iter", "res", "obj"]:
        want = o64[key][bad]
        want = want if key == "iter" else want.astype(np.float32)
        assert np.array_equal(resc[key][bad], want), key


def test_f64_rescue_noop_without_failures(pkg):
    """Nothing unsolved (box-u, fp32 converges everywhere at these settings): f64_rescue
    changes no output bit."""
    qp, x0 = pkg.srbd_model.generate_batch(64, N=20, seed=92, constraints="box_u")
    st = dict(F32, tol_stat=3e-2)
    a = pkg.capi.solve(qp, x0, st, dtype=np.float32)
    b = pkg.capi.solve(qp, x0, dict(st, f64_rescue=30), dtype=np.float32)
    assert np.all(a["status"] == 0)
    for key in a:
        assert np.array_equal(a[key], b[key]), key


def test_f64_rescue_without_status_output_and_host_path(pkg):
    """The rescue keeps its own status list when the caller passes no status buffer,
    and the host-buffer entry point rescues the same QPs: x / u agree bit for bit."""
    import torch
    qp, x0 = pkg.srbd_model.generate_batch(256, N=40, seed=1005, constraints="cone")
    st = dict(F32, tol_stat=3e-2, f64_rescue=12)
    ref = pkg.capi.solve(qp, x0, st, dtype=np.float32)
    h = pkg.capi.Handle(qp.N, qp.nx, qp.nu, qp.ng, qp.has_box_u, qp.has_box_x, capacity=qp.batch)
    try:
        s = pkg.capi.settings_struct(st)
        dt, out, data, sol = pkg.capi.device_buffers(qp, x0, "cuda:0", dtype=np.float32)
        sol.status = None
        sol.iter = None
        h.solve_device(qp.batch, s, data, sol)
        h.synchronize()
        torch.cuda.synchronize()
        for key in ("x", "u", "pi"):
            assert np.array_equal(out[key].cpu().numpy(), ref[key]), key
        capi = pkg.capi
        p = {k: (None if v is None else np.ascontiguousarray(v, dtype=np.float32))
             for k, v in qp.packed().items()}
        p["x0"] = np.ascontiguousarray(x0, dtype=np.float32)
        hx = {k: np.zeros_like(ref[k]) for k in ("x", "u", "pi", "status")}
        hdata = capi.Data32(**{k: (None if p.get(k) is None else p[k].ctypes.data)
                               for k in capi.DATA_FIELDS})
        hsol = capi.Solution32(**{k: v.ctypes.data for k, v in hx.items()})
        h.solve_host(qp.batch, s, hdata, hsol)
        for key in ("x", "u", "pi", "status"):
            assert np.array_equal(hx[key], ref[key]), key
    finally:
        h.close()
