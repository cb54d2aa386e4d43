"""Dev aid: A/B the SQP-pipeline kernels (linearise, solve, line search) of library
variants (build/variants/*/libsrbd_qp.so), interleaved, each run in its own process."""
import json
import os
import subprocess
import sys
from pathlib import Path

repo = Path(__file__).resolve().parents[2]
names = sys.argv[1].split(",")
res = {n: [] for n in names}
for r in range(2):
    for n in names:
        env = dict(os.environ)
        env["SRBD_QP_LIB"] = str(repo / "build" / "variants" / n / "libsrbd_qp.so") if n != "product" else ""
        out = subprocess.run([sys.executable, str(repo / "bench.py"), "--no-cpu-baseline", "--no-secondary",
                              "--no-host-path", "--steps", "5", "--warmup", "1"],
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(n, "FAILED", out.stderr[-2000:], flush=True)
            sys.exit(1)
        sp = json.loads(out.stdout.strip().splitlines()[-1])["sqp_pipeline"]
        res[n].append((sp["ms_linearize"], sp["ms_qp_solve"], sp["ms_line_search"]))
        print(n, r, res[n][-1], flush=True)
for n in names:
    print(f"{n:12s} linearize min {min(x[0] for x in res[n]):.3f}  solve {min(x[1] for x in res[n]):.3f}  "
          f"line search {min(x[2] for x in res[n]):.3f}")
