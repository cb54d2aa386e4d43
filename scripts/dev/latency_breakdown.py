"""Dev aid (GPU, diagnostic build -DSRBD_TSTAMP=1 via SRBD_QP_LIB): the critical path of
the reference's single-QP solve on the LDS latency kernel, from the phase timestamps lane 0
appends (riccati.h tstamp): cycles per phase of a backward stage, averaged over the stages,
the forward sweep, the copy into LDS, and the kernel time from HIP events to convert.

  SRBD_QP_LIB=build/variants/tstamp/libsrbd_qp.so python scripts/dev/latency_breakdown.py"""
import ctypes as C
import importlib.util
import json
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
import torch  # noqa: E402

pkg = bench.import_pkg()
capi = pkg.capi
L = capi.lib()
L.srbd_qp_diag_tstamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
L.srbd_qp_diag_tstamps.restype = C.c_int
N = 20
qp, x0 = pkg.srbd_model.generate_batch(1, N=N, seed=1003)
h = capi.Handle(N, 12, 12, 0, False, False, capacity=1)
s = capi.settings_struct(dict(bench.NMPC_SETTINGS, compute_residuals=0))
dt, st, data, sol = capi.device_buffers(qp, x0)
buf = (C.c_ulonglong * (2 * 4096))()
ext = torch.cuda.ExternalStream(h.stream(), device=torch.device("cuda", 0))
names = {16: "entry", 14: "copy issued", 15: "copy landed", 0: "stage start", 1: "WB=P B", 2: "G=R+B'WB",
         3: "chol(G)", 4: "W=P[A|b]", 5: "H=S+B'W", 6: "F=Q+A'W", 7: "L^-1 H", 8: "K=-L^-T Y",
         9: "P=F-Y'Y", 10: "Acl=A+BK", 11: "record stored", 12: "backward done", 13: "forward done"}
runs = []
for rep in range(6):
    L.srbd_qp_diag_tstamps(buf, 4096)  # reset
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ext)
    h.solve_device(1, s, data, sol)
    e1.record(ext)
    h.synchronize()
    n = L.srbd_qp_diag_tstamps(buf, 4096)
    arr = np.frombuffer(buf, dtype=np.uint64)[:2 * n].reshape(n, 2).astype(np.int64)
    runs.append((e0.elapsed_time(e1) * 1e3, arr))
kus, arr = runs[-1]
ids, cyc = arr[:, 0], arr[:, 1] - arr[0, 1]
total = cyc[-1]
per = {}
prev = None
for i in range(1, len(ids)):
    key = f"{names.get(int(ids[i - 1]), ids[i - 1])} -> {names.get(int(ids[i]), ids[i])}"
    per.setdefault(key, []).append(int(cyc[i] - cyc[i - 1]))
out = {"kernel_us_hip_events": kus, "stamped_cycles": int(total),
       "us_per_cycle": kus / max(int(total), 1),
       "phases_cycles": {k: {"n": len(v), "mean": float(np.mean(v)), "sum": int(np.sum(v))}
                         for k, v in per.items()}}
print(json.dumps(out, indent=1))
