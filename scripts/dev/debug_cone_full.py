"""Dev aid: config-5 status counts: repeated solves, fresh handles, settings variants."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import torch
import helpers
import test_gpu_fullsize as T
import bench
pkg = helpers.load_package()
N = 40
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
h, t = T.device_batch(pkg, N, "cone", batch=B)
prev = None
def run(tag, hh, st, dtype="f32"):
    global prev
    s = T.solve_on_device(pkg, hh, t, N, st, dtype=dtype)
    u = s["u"].cpu().numpy()
    d = None if prev is None else float(np.nanmax(np.abs(u - prev)))
    prev = u
    print(tag, np.bincount(s["status"].cpu().numpy(), minlength=4), "iters mean %.2f" % s["iter"].float().mean().item(), "max|u-prev|", d, flush=True)
for i in range(3):
    run(f"testF32 same-handle #{i}", h, T.F32)
run("benchF32 same-handle", h, bench.F32_SETTINGS)
run("benchF32 same-handle again", h, bench.F32_SETTINGS)
run("testF32 ric_alg0", h, dict(T.F32, ric_alg=0))
h2 = pkg.capi.Handle(N, 12, 12, 24, False, False, capacity=B)
run("testF32 fresh handle", h2, T.F32)
run("benchF32 fresh handle", h2, bench.F32_SETTINGS)
