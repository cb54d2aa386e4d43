"""Dev aid: run the device linearisation and line search a few times on 65536 x N=20
(for rocprofv3 --kernel-trace --stats)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import torch
import helpers
pkg = helpers.load_package()
capi = pkg.capi
B, N = 65536, 20
xs, us, x0 = pkg.srbd_model.sample_trajectories(B, N, 1003, pkg.srbd_model.SrbdParams(), 0)
xs = torch.from_numpy(np.ascontiguousarray(xs)).cuda(); us = torch.from_numpy(np.ascontiguousarray(us)).cuda()
h = capi.Handle(N, 12, 12, 0, False, False, capacity=B)
for mode in sys.argv[1:] or ["none"]:
    out = None
    for _ in range(4):
        dt, data = capi.srbd_linearize(h, xs, us, mode, out=out)
        out = dt
    h.synchronize()
dx = torch.zeros_like(xs); du = torch.zeros_like(us) + 0.01
al = torch.ones(B, dtype=torch.float64, device="cuda")
for _ in range(4):
    capi.srbd_linesearch(h, xs.clone(), us.clone(), dx, du, al.clone())
h.synchronize()
torch.cuda.synchronize()
print("done")
