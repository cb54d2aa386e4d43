"""Dev aid: why does the unconstrained solve take longer on linearised data?"""
import sys, time
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import torch
import helpers
import bench
pkg = helpers.load_package()
capi = pkg.capi
B, N = 65536, 20
dev = torch.device("cuda", 0)
qp, x0 = bench.make_shard(pkg, N, "none", B, 0, 1003, 4096)
dt = bench.to_device(pkg, qp, x0, B, dev)
h = capi.Handle(N, 12, 12, 0, False, False, capacity=B)
f64 = dict(dtype=torch.float64, device=dev)
sol = {"x": torch.zeros(B, N + 1, 12, **f64), "u": torch.zeros(B, N, 12, **f64), "pi": torch.zeros(B, N + 1, 12, **f64)}
S = capi.Solution(**{k: (sol[k].data_ptr() if k in sol else None) for k in capi.SOL_FIELDS})
st = capi.settings_struct(bench.NMPC_SETTINGS)
D1 = capi.Data(**{k: (None if dt.get(k) is None else dt[k].data_ptr()) for k in capi.DATA_FIELDS})
p = pkg.srbd_model.SrbdParams()
xs, us, x0p = pkg.srbd_model.sample_trajectories(4096, N, 1003, p, 0)
tile = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev).repeat((16,) + (1,) * (a.ndim - 1)).contiguous()
xs_t, us_t, x0_t = tile(xs), tile(us), tile(x0p)
t, D2 = capi.srbd_linearize(h, xs_t, us_t, "none")
dx0 = (x0_t - xs_t[:, 0]).contiguous()
D2.x0 = dx0.data_ptr()
h.synchronize()
for k in ("A", "B", "b", "Q", "S", "R", "q", "r"):
    a1, a2 = dt[k].float(), t[k].float()
    print(k, "bench absmax %.3g" % a1.abs().max().item(), "lin absmax %.3g" % a2.abs().max().item(),
          "nan", torch.isnan(t[k]).sum().item(), "denorm", ((t[k] != 0) & (t[k].abs() < 2.3e-308)).sum().item(),
          "tiny<1e-300", ((t[k] != 0) & (t[k].abs() < 1e-300)).sum().item())
ext = torch.cuda.ExternalStream(h.stream(), device=dev)
for name, D in (("bench", D1), ("linearised", D2), ("bench", D1), ("linearised", D2)):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ext)
    for _ in range(3):
        h.solve_device(B, st, D, S)
    e1.record(ext)
    h.synchronize()
    print(name, "%.3f ms" % (e0.elapsed_time(e1) / 3), "x nan", torch.isnan(sol["x"]).sum().item(),
          "x absmax %.3g" % sol["x"].abs().max().item())
