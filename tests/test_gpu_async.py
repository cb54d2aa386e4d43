"""The constrained (IPM) device solve is asynchronous on its stream (include/srbd_qp.h
srbd_qp_solve_f64): the stop decision lives on the device (ipm_box_impl.h report_running /
solve_done), so the host enqueues the whole launch sequence and returns.  One host thread can
therefore keep several handles busy at once -- the reference's hpipm-cpp is reentrant with
separate memory per solver, and this is the batched equivalent."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1,
            ric_alg=0, mode="Speed")


def _setup(pkg, batch, seed):
    qp, x0 = pkg.srbd_model.generate_batch(batch, N=20, seed=seed, constraints="box_u")
    h = pkg.capi.Handle(qp.N, qp.nx, qp.nu, qp.ng, qp.has_box_u, qp.has_box_x, capacity=batch)
    s = pkg.capi.settings_struct(NMPC)
    dt, st, data, sol = pkg.capi.device_buffers(qp, x0, "cuda:0")
    return qp, x0, h, s, (dt, st, data, sol)


def test_ipm_solve_returns_before_its_stream_drains(pkg):
    import torch
    qp, x0, h, s, (dt, st, data, sol) = _setup(pkg, 8192, 41)
    torch.cuda.synchronize()
    h.solve_device(qp.batch, s, data, sol, order=False)  # warm-up (module load, first launch)
    h.synchronize()
    t0 = time.perf_counter()
    h.solve_device(qp.batch, s, data, sol, order=False)
    t_call = time.perf_counter() - t0
    busy = not h.torch_stream().query()
    h.synchronize()
    t_all = time.perf_counter() - t0
    assert busy, "the stream had drained when the call returned"
    # (timing ratio logged, not asserted: host scheduling on a shared box moves it)
    print(f"call returned after {t_call * 1e3:.2f} ms of a {t_all * 1e3:.2f} ms solve")
    out = {k: v.cpu().numpy() for k, v in st.items()}
    ref = pkg.capi.solve(qp, x0, NMPC)
    assert np.all(out["status"] == 0)
    for key in ("x", "u", "pi", "status", "iter"):
        np.testing.assert_array_equal(out[key], ref[key])
    h.close()


def test_two_handles_overlap_from_one_thread(pkg):
    """Two small latency-bound solves (64 QPs each: one chain of sweeps per QP group) on two
    handles, launched from one thread: together they take well under the sum of their times."""
    import torch
    A = _setup(pkg, 64, 51)
    B = _setup(pkg, 64, 52)
    torch.cuda.synchronize()

    def run(both):
        t0 = time.perf_counter()
        for qp, _, h, s, (_, _, data, sol) in (A, B):
            h.solve_device(qp.batch, s, data, sol, order=False)
            if not both:
                h.synchronize()
        A[2].synchronize()
        B[2].synchronize()
        return time.perf_counter() - t0

    run(False)
    seq = min(run(False) for _ in range(3))
    par = min(run(True) for _ in range(3))
    # two independent latency chains on two streams: well under the sequential time (measured
    # ~0.55); the margin absorbs box-to-box and load variation
    print(f"two handles: sequential {seq * 1e3:.2f} ms, overlapped {par * 1e3:.2f} ms")
    assert par < 0.95 * seq, (par, seq)
    for qp, x0, h, _, (_, st, _, _) in (A, B):
        ref = pkg.capi.solve(qp, x0, NMPC)
        for key in ("x", "u", "status", "iter"):
            np.testing.assert_array_equal(st[key].cpu().numpy(), ref[key])
        h.close()


def test_multi_device_shards_and_gather(pkg):
    """srbd_qp_multi (one solver over several devices, one host thread): two shards -- both
    on device 0 here, the pool's boxes have one GPU -- of 64 and 96 box-u QPs are solved
    concurrently and their x, u, pi gathered to the root device in shard order by peer
    copies; every QP equals the single-handle solve of the whole batch bit for bit."""
    import torch
    capi = pkg.capi
    qp, x0 = pkg.srbd_model.generate_batch(160, N=20, seed=61, constraints="box_u")
    ref = capi.solve(qp, x0, NMPC)
    s = capi.settings_struct(NMPC)
    shards = [(0, 64), (64, 160)]
    m = capi.Multi(20, 12, 12, [0, 0], has_box_u=True, capacity=96)
    keep, datas, sols = [], [], []
    for lo, hi in shards:
        dt, st, data, sol = capi.device_buffers(qp.subset(slice(lo, hi)), x0[lo:hi], "cuda:0")
        keep.append((dt, st))
        datas.append(data)
        sols.append(sol)
    f = dict(dtype=torch.float64, device="cuda:0")
    rx, ru, rpi = torch.zeros(160, 21, 12, **f), torch.zeros(160, 20, 12, **f), torch.zeros(160, 21, 12, **f)
    torch.cuda.synchronize()
    m.solve([hi - lo for lo, hi in shards], s, datas, sols, rx, ru, rpi)
    for key, t in (("x", rx), ("u", ru), ("pi", rpi)):
        np.testing.assert_array_equal(t.cpu().numpy(), ref[key])
    for (lo, hi), (_, st) in zip(shards, keep):
        np.testing.assert_array_equal(st["status"].cpu().numpy(), ref["status"][lo:hi])
    m.close()


def test_multi_device_fp32_shards(pkg):
    """srbd_qp_multi_solve_f32 (ABI 11): config 5's fp32 friction-cone problem in two shards
    (both on device 0 here) -- every QP's x, u, pi gathered in shard order equals the
    single-handle fp32 solve of the whole batch bit for bit, status included."""
    import torch
    capi = pkg.capi
    qp, x0 = pkg.srbd_model.generate_batch(96, N=20, seed=62, constraints="cone")
    st_d = dict(iter_max=30, tol_stat=1e-2, tol_eq=1e-3, tol_ineq=1e-3, tol_comp=1e-3, split_step=1)
    ref = capi.solve(qp, x0, st_d, dtype=np.float32)
    s = capi.settings_struct(st_d)
    shards = [(0, 40), (40, 96)]
    m = capi.Multi(20, 12, 12, [0, 0], ng=qp.ng, has_box_u=qp.has_box_u, has_box_x=qp.has_box_x, capacity=56)
    keep, datas, sols = [], [], []
    for lo, hi in shards:
        dt, st, data, sol = capi.device_buffers(qp.subset(slice(lo, hi)), x0[lo:hi], "cuda:0",
                                                dtype=np.float32)
        keep.append((dt, st))
        datas.append(data)
        sols.append(sol)
    f = dict(dtype=torch.float32, device="cuda:0")
    rx, ru, rpi = torch.zeros(96, 21, 12, **f), torch.zeros(96, 20, 12, **f), torch.zeros(96, 21, 12, **f)
    torch.cuda.synchronize()
    m.solve([hi - lo for lo, hi in shards], s, datas, sols, rx, ru, rpi)
    for key, t in (("x", rx), ("u", ru), ("pi", rpi)):
        np.testing.assert_array_equal(t.cpu().numpy(), ref[key])
    for (lo, hi), (_, st) in zip(shards, keep):
        np.testing.assert_array_equal(st["status"].cpu().numpy(), ref["status"][lo:hi])
    m.close()
