"""Dev aid: box-u config 3 (65536 QPs, N = 20): fp64 IPM time vs fp32 IPM time for a
fixed number of iterations (tolerances out of reach), to size a mixed-precision IPM."""
import sys, time
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import torch
import helpers
import bench
pkg = helpers.load_package()
capi = pkg.capi
dev = torch.device("cuda:0")
B, N = 65536, 20
h = capi.Handle(N, 12, 12, 0, True, False, capacity=B)
dt, _, _, _ = bench.device_shard(pkg, h, N, "box_u", B, 0, 1234, dev)


def run(dtype, st, reps=2):
    tt = torch.float32 if dtype == "f32" else torch.float64
    d = {k: v.to(tt).contiguous() for k, v in dt.items()}
    sol = {"x": torch.zeros(B, N + 1, 12, dtype=tt, device=dev), "u": torch.zeros(B, N, 12, dtype=tt, device=dev),
           "pi": torch.zeros(B, N + 1, 12, dtype=tt, device=dev),
           "status": torch.zeros(B, dtype=torch.int32, device=dev), "iter": torch.zeros(B, dtype=torch.int32, device=dev)}
    DataT, SolT = (capi.Data32, capi.Solution32) if dtype == "f32" else (capi.Data, capi.Solution)
    data = DataT(**{k: (None if d.get(k) is None else d[k].data_ptr()) for k in capi.DATA_FIELDS})
    so = SolT(**{k: (sol[k].data_ptr() if k in sol else None) for k in capi.SOL_FIELDS})
    s = capi.settings_struct(st)
    torch.cuda.synchronize()
    h.solve_device(B, s, data, so)
    h.synchronize()
    ext = h.torch_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ext)
    for _ in range(reps):
        h.solve_device(B, s, data, so, order=False)
    e1.record(ext)
    h.synchronize()
    ms = e0.elapsed_time(e1) / reps
    it = sol["iter"].cpu().numpy()
    stt = sol["status"].cpu().numpy()
    run.last = sol
    return ms, it.mean(), it.max(), np.bincount(stt, minlength=4)


NMPC = dict(bench.NMPC_SETTINGS)
print("fp64 NMPC", run("f64", NMPC), flush=True)
ref = {k: v.clone() for k, v in run.last.items()}
for k in [int(a) for a in sys.argv[1:]] or [4, 5, 6, 7, 8]:
    r = run("f64", dict(NMPC, f32_iters=k))
    du = (run.last["u"] - ref["u"]).abs().amax(dim=(1, 2)) / ref["u"].abs().amax(dim=(1, 2))
    print("mixed f32_iters=%d" % k, r, "u rel diff max %.2e median %.2e" % (du.max().item(), du.median().item()),
          flush=True)
