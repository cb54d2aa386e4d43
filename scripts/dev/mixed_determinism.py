"""Dev aid: does the mixed-precision path depend on what freshly allocated device memory
holds?  Poison the memory the library's hipMalloc will get back (a large torch tensor
filled with a value, then freed to the driver), solve, compare."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
import torch
import helpers
pkg = helpers.load_package()
NMPC = dict(iter_max=30, tol_stat=1e-4, tol_eq=1e-4, tol_ineq=1e-4, tol_comp=1e-4, split_step=1)
qp, x0 = pkg.srbd_model.generate_batch(256, N=20, seed=5, constraints="box_u")
ref = None
for poison in (None, 0.0, -1.0, float("nan"), 1e30, -3.5):
    if poison is not None:
        t = torch.full((1 << 28,), poison, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        del t
        torch.cuda.empty_cache()
    out = pkg.capi.solve(qp, x0, dict(NMPC, f32_iters=6))
    if ref is None:
        ref = out
    same = all(np.array_equal(out[k], ref[k]) for k in ("x", "u", "pi", "iter", "status"))
    print(f"poison {poison}: iter mean {out['iter'].mean():.3f} status {np.bincount(out['status'])} "
          f"bit-identical to first: {same}", flush=True)
