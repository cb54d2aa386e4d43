"""Dev aid: batch-1 (the reference's one QP per call) latency, device vs host buffers."""
import sys, time
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import torch
import helpers
pkg = helpers.load_package()
capi = pkg.capi
NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)
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
        lat = []
        for _ in range(20):
            t0 = time.perf_counter()
            h.solve_device(B, s, data, sol, order=False)
            h.synchronize()
            lat.append(time.perf_counter() - t0)
        print(cons, B, "device stream ms/solve %.3f" % dev_ms, "launch+sync ms %.3f" % (np.median(lat) * 1e3),
              "iters", st["iter"].cpu().numpy()[:4], flush=True)
