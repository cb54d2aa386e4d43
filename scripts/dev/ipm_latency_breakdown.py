"""Dev aid (GPU, diagnostic build -DSRBD_TSTAMP=1 via SRBD_QP_LIB): where one IPM QP's
iteration goes when it runs alone (the tail of config 5: the few QPs still running after
the batch has converged). Lane 0 of workgroup 0 stamps the cycle counter at the phase
boundaries of every stage (ipm_box_impl.h: 20-23 RB, 1-10 the factorization inside it,
30 / 31 F1 / F2, 40 B2); printed: cycles per transition averaged over the stamped stages.

  SRBD_QP_LIB=build/variants/tstamp/libsrbd_qp.so python scripts/dev/ipm_latency_breakdown.py [box_u_n20|cone_n40_f32] [batch]"""
import ctypes as C
import importlib.util
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
import torch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cone_n40_f32"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
pkg = bench.import_pkg()
capi = pkg.capi
L = capi.lib()
STAMPS = hasattr(L, "srbd_qp_diag_tstamps_ipm")  # a -DSRBD_TSTAMP=1 build; else timing only
if STAMPS:
    L.srbd_qp_diag_tstamps_ipm.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    L.srbd_qp_diag_tstamps_ipm.restype = C.c_int
N, constraints = bench.WORKLOADS[name][:2]
dtype = bench.WORKLOADS[name][4] if len(bench.WORKLOADS[name]) > 4 else "f64"
ng = 24 if constraints == "cone" else 0
device = torch.device("cuda", 0)
h = capi.Handle(N, 12, 12, ng, constraints == "box_u", False, capacity=batch)
dt, _, _, _ = bench.device_shard(pkg, h, N, constraints, batch, 0, 1, device,
                                 np.float32 if dtype == "f32" else np.float64)
tt = dict(dtype=torch.float32 if dtype == "f32" else torch.float64, device=device)
sol_t = {"x": torch.zeros(batch, N + 1, 12, **tt), "u": torch.zeros(batch, N, 12, **tt),
         "pi": torch.zeros(batch, N + 1, 12, **tt),
         "status": torch.zeros(batch, dtype=torch.int32, device=device),
         "iter": torch.zeros(batch, dtype=torch.int32, device=device)}
DataT, SolT = (capi.Data32, capi.Solution32) if dtype == "f32" else (capi.Data, capi.Solution)
data = DataT(**{k: (None if dt.get(k) is None else dt[k].data_ptr()) for k in capi.DATA_FIELDS})
sol = SolT(**{k: (sol_t[k].data_ptr() if k in sol_t else None) for k in capi.SOL_FIELDS})
s = capi.settings_struct(bench.F32_SETTINGS if dtype == "f32" else bench.NMPC_SETTINGS)
buf = (C.c_ulonglong * (2 * 4096))()
ext = torch.cuda.ExternalStream(h.stream(), device=device)
names = {20: "RB stage", 21: "RB step applied, rows", 22: "RB A,B,S, residuals", 23: "RB record stored",
         1: "WB=P B", 2: "G=R+B'WB", 3: "chol(G)", 4: "W=P[A|b]", 5: "H=S+B'W", 6: "F=Q+A'W",
         7: "L^-1 H", 8: "K=-L^-T Y", 9: "P=F-Y'Y", 10: "Acl=A+BK", 30: "F1 stage", 31: "F2 stage",
         40: "B2 stage"}
res = []
for rep in range(4):
    if STAMPS:
        L.srbd_qp_diag_tstamps_ipm(buf, 4096)  # reset
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ext)
    h.solve_device(batch, s, data, sol)
    e1.record(ext)
    h.synchronize()
    n = L.srbd_qp_diag_tstamps_ipm(buf, 4096) if STAMPS else 0
    res.append((e0.elapsed_time(e1) * 1e3, np.frombuffer(buf, dtype=np.uint64)[:2 * n].reshape(n, 2).astype(np.int64)))
us = min(r[0] for r in res)
arr = res[-1][1]
ids, cyc = arr[:, 0], arr[:, 1]
per = {}
for i in range(1, len(ids)):
    d = int(cyc[i] - cyc[i - 1])
    if d < 0 or d > 10_000_000:  # a launch boundary
        continue
    key = f"{names.get(int(ids[i - 1]), int(ids[i - 1]))} -> {names.get(int(ids[i]), int(ids[i]))}"
    per.setdefault(key, []).append(d)
out = {"workload": name, "batch": batch, "solve_us_hip_events": us, "stamps": int(len(ids)),
       "iters": sol_t["iter"].cpu().numpy().tolist()[:4],
       "note": "cycles of the shader clock (s_memtime); each stamp adds ~700 cycles",
       "transitions": {k: {"n": len(v), "mean": float(np.mean(v)), "median": float(np.median(v))}
                       for k, v in sorted(per.items(), key=lambda kv: -np.sum(kv[1]))}}
print(json.dumps(out, indent=1))
