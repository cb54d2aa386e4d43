"""Per-dispatch HBM traffic of one kernel across the launches of an IPM solve.

  python scripts/pmc_dispatch.py TAG WORKLOAD BATCH KERNEL_SUBSTRING [SOLVES]

Reads a scripts/profile.sh run (gpurun_out/prof_<TAG>_<WORKLOAD>/{trace,fetch,write}), picks
the dispatches of the kernel whose name contains KERNEL_SUBSTRING (the three runs launch the
same sequence, so the i-th dispatch of the name in each run is the same launch), splits them
into SOLVES equal solves (bench.py: warmup 1 + steps 5 = 6) and reports, per launch index
within a solve (= IPM iteration for RB+F1): duration, FETCH_SIZE x 2 + WRITE_SIZE (the MI355X
guide's gfx950 correction) per launch and per QP, and the achieved rate.  The full-batch
iterations are the ones before the live-QP count drops; the launch-average over a whole solve
mixes them with the near-empty tail launches."""
import csv
import glob
import json
import sys
from pathlib import Path

repo = Path(__file__).resolve().parents[1]
tag, workload, batch, sub = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
solves = int(sys.argv[5]) if len(sys.argv) > 5 else 6
src = repo / "gpurun_out" / f"prof_{tag}_{workload}"


def load(kind, pattern):
    out = []
    for f in glob.glob(str(src / kind / "**" / pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def name_of(r):
    return r.get("Kernel_Name", r.get("Name", ""))


trace = [r for r in load("trace", "*kernel_trace.csv") if sub in name_of(r)]
trace.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in trace]


def counter(kind, key):
    rows = [r for r in load(kind, "*counter_collection.csv") if sub in name_of(r) and r["Counter_Name"] == key]
    by = {}
    for r in rows:  # one row per dispatch (summed over dimensions when several)
        by.setdefault(int(r["Dispatch_Id"]), 0.0)
        by[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


fetch = [v * 2 * 1024 for v in counter("fetch", "FETCH_SIZE")]
write = [v * 1024 for v in counter("write", "WRITE_SIZE")]
n = min(len(dur), len(fetch), len(write))
per = n // solves
table = []
for i in range(per):
    idx = [s * per + i for s in range(1, solves)]  # skip the warmup solve
    d = sum(dur[j] for j in idx) / len(idx)
    f = sum(fetch[j] for j in idx) / len(idx)
    w = sum(write[j] for j in idx) / len(idx)
    table.append({"launch": i, "ms": d * 1e3, "fetch_bytes": f, "write_bytes": w,
                  "hbm_bytes_per_qp": (f + w) / batch, "tbs": (f + w) / max(d, 1e-12) / 1e12})
full = [t for t in table if t["ms"] > 0.5 * table[0]["ms"]] if table else []
out = {"workload": workload, "batch": batch, "kernel_substring": sub, "dispatches": n,
       "launches_per_solve": per, "per_launch": table,
       "full_batch_launches": len(full),
       "full_batch_mean": {k: sum(t[k] for t in full) / len(full) for k in ("ms", "hbm_bytes_per_qp", "tbs")}
       if full else None,
       "all_launch_mean": {k: sum(t[k] for t in table) / len(table) for k in ("ms", "hbm_bytes_per_qp", "tbs")}
       if table else None,
       "note": "FETCH_SIZE x2 + WRITE_SIZE per dispatch (KB x1024), matched by dispatch order across the "
               "trace / fetch / write runs; solve 0 (warmup) skipped"}
dst = repo / "profiles" / "round6"
dst.mkdir(parents=True, exist_ok=True)
(dst / f"{workload}_{sub.replace('<', '_').replace('>', '_').replace(',', '_').replace(' ', '')}_per_dispatch.json"
 ).write_text(json.dumps(out, indent=1))
print(json.dumps({k: v for k, v in out.items() if k != "per_launch"}, indent=1))
for t in table:
    print("%3d %8.3f ms %10.0f B/QP %6.2f TB/s" % (t["launch"], t["ms"], t["hbm_bytes_per_qp"], t["tbs"]))
