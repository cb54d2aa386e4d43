"""Dev aid (GPU): the reference call pattern (build/call_pattern_bench) with the shim's host-time
profile (SRBD_SHIM_PROFILE=1): staging pointers, packing, the C-ABI solve, unpacking per call."""
import importlib.util
import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
pkg = bench.import_pkg()
N = 20
qp, x0 = pkg.srbd_model.generate_batch(1, N=N, seed=1003)
p = qp.packed()
vals = [np.array([float(N)])]
for k in range(N):
    for name in ("A", "B", "b", "Q", "S", "R", "q", "r"):
        vals.append(p[name][0].reshape(N + (1 if name in ("Q", "q") else 0), -1)[k])
vals += [p["Q"][0].reshape(N + 1, -1)[N], p["q"][0].reshape(N + 1, -1)[N], x0[0]]
with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
    f.write(np.concatenate(vals).astype("<f8").tobytes())
env = dict(os.environ, SRBD_SHIM_PROFILE="1")
r = subprocess.run([str(REPO / "build" / "call_pattern_bench"), f.name, "20"], capture_output=True, text=True,
                   env=env, timeout=300)
os.unlink(f.name)
print(r.stdout.strip().splitlines()[-1])
print(r.stderr.strip().splitlines()[-1])
