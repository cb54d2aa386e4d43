"""Dev aid: A/B the kernel time of library variants (build/variants/*/libsrbd_qp.so)
on one workload, interleaved, each run in its own process (bench.py)."""
import json
import os
import subprocess
import sys
from pathlib import Path

repo = Path(__file__).resolve().parents[2]
names = sys.argv[1].split(",")
extra = sys.argv[2:]
rounds = 2
res = {n: [] for n in names}
for r in range(rounds):
    for n in names:
        env = dict(os.environ)
        lib = repo / "build" / "variants" / n / "libsrbd_qp.so"
        env["SRBD_QP_LIB"] = str(lib) if n != "product" else ""
        out = subprocess.run([sys.executable, str(repo / "bench.py"), "--no-cpu-baseline"] + extra,
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(n, "FAILED", out.stderr[-2000:], flush=True)
            sys.exit(1)
        line = json.loads(out.stdout.strip().splitlines()[-1])
        res[n].append((line["roofline"]["kernel_avg_ms"], line["value"], line["success_rate"],
                       line["iters_mean"]))
        print(n, r, res[n][-1], flush=True)
for n in names:
    ms = [x[0] for x in res[n]]
    it = res[n][0][3]
    per_it = f"  per iteration {min(ms) / it:.3f} ms ({it:.2f} it)" if it else ""
    print(f"{n:20s} kernel ms min {min(ms):.3f}  all {['%.3f' % m for m in ms]}  value {max(x[1] for x in res[n]):.4g}{per_it}")
