"""Dev aid: batch-1 (the reference's one QP per call) latency breakdown.

device:  kernel time per solve (HIP events over back-to-back solves) and one
         launch + synchronize, device buffers;
host:    srbd_qp_solve_host_f64 from host buffers with the outputs the hpipm-cpp
         shim requests (x, u, pi, P, p, K, k, status, iter, res, obj, stat)."""
import sys, time
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import torch
import helpers
pkg = helpers.load_package()
capi = pkg.capi
NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1, ric_alg=0)


def med(f, n=51):
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        t.append(time.perf_counter() - t0)
    return float(np.median(t[1:])) * 1e3


for cons in ("none", "box_u"):
    for B in (1, 16, 256):
        qp, x0 = pkg.srbd_model.generate_batch(B, N=20, seed=5, constraints=cons)
        h = capi.Handle(20, 12, 12, 0, cons == "box_u", False, capacity=B)
        dt, st, data, sol = capi.device_buffers(qp, x0)
        s = capi.settings_struct(NMPC)
        ext = h.torch_stream()
        for _ in range(3):
            h.solve_device(B, s, data, sol)
        h.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(ext)
        for _ in range(20):
            h.solve_device(B, s, data, sol, order=False)
        e1.record(ext)
        h.synchronize()
        dev_ms = e0.elapsed_time(e1) / 20

        def dev_call():
            h.solve_device(B, s, data, sol, order=False)
            h.synchronize()
        lat = med(dev_call)
        # host buffers, every output the shim asks for
        p = qp.packed()
        p["x0"] = np.ascontiguousarray(x0).reshape(B, 12)
        N = 20
        out = {"x": np.zeros((B, N + 1, 12)), "u": np.zeros((B, N, 12)), "pi": np.zeros((B, N + 1, 12)),
               "P": np.zeros((B, N + 1, 144)), "p": np.zeros((B, N + 1, 12)), "K": np.zeros((B, N, 144)),
               "k": np.zeros((B, N, 12)), "status": np.zeros(B, np.int32), "iter": np.zeros(B, np.int32),
               "res": np.zeros((B, 4)), "obj": np.zeros(B), "stat": np.zeros((B, 32, 18))}
        hd = capi.Data(**{k: (None if p.get(k) is None else p[k].ctypes.data) for k in capi.DATA_FIELDS})
        hs = capi.Solution(**{k: out[k].ctypes.data for k in capi.SOL_FIELDS})
        hlat = med(lambda: h.solve_host(B, s, hd, hs))
        hs2 = capi.Solution(**{k: (out[k].ctypes.data if k in ("x", "u", "pi", "status", "iter") else None)
                               for k in capi.SOL_FIELDS})
        hlat2 = med(lambda: h.solve_host(B, s, hd, hs2))
        print(f"{cons:6s} B={B:4d} kernel {dev_ms * 1e3:8.1f} us | device launch+sync {lat * 1e3:8.1f} us | "
              f"host all outputs {hlat * 1e3:8.1f} us | host x/u/pi {hlat2 * 1e3:8.1f} us | "
              f"status {np.bincount(out['status'])}", flush=True)
        h.close()
