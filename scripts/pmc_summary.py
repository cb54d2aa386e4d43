"""Summarise a scripts/profile.sh run into profiles/<tag>/ and profiles/pmc_traffic.json.

  python scripts/pmc_summary.py TAG WORKLOAD BATCH

Reads gpurun_out/prof_<TAG>_<WORKLOAD>/{trace,fetch,write}/**.csv, keeps the
solver kernels' rows, and records per launch: average duration (kernel trace),
FETCH_SIZE x 2 (gfx950 reports half of a wide streaming read, MI355X_MICROARCH.md
HBM section) + WRITE_SIZE, in bytes."""
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

repo = Path(__file__).resolve().parents[1]
tag, workload, batch = sys.argv[1], sys.argv[2], int(sys.argv[3])
src = repo / "gpurun_out" / f"prof_{tag}_{workload}"
dst = repo / "profiles" / tag
dst.mkdir(parents=True, exist_ok=True)


def rows(kind, pattern):
    out = []
    for f in glob.glob(str(src / kind / "**" / pattern), recursive=True):
        with open(f) as fh:
            out += [r for r in csv.DictReader(fh) if "srbd::" in r.get("Kernel_Name", r.get("Name", ""))]
    return out


stats = rows("trace", "*kernel_stats.csv")
trace = rows("trace", "*kernel_trace.csv")
fetch = rows("fetch", "*counter_collection.csv")
write = rows("write", "*counter_collection.csv")
for kind, pattern, name in (("trace", "*kernel_stats.csv", "kernel_stats"),
                            ("fetch", "*counter_collection.csv", "pmc_fetch"),
                            ("write", "*counter_collection.csv", "pmc_write")):
    for f in glob.glob(str(src / kind / "**" / pattern), recursive=True):
        shutil.copy(f, dst / f"{workload}_{name}.csv")
kname = stats[0]["Name"] if stats else None
avg_ns = float(stats[0]["AverageNs"]) if stats else None
fv = [float(r["Counter_Value"]) for r in fetch if r["Counter_Name"] == "FETCH_SIZE"]
wv = [float(r["Counter_Value"]) for r in write if r["Counter_Name"] == "WRITE_SIZE"]
fetch_b = 2 * 1024 * sum(fv) / len(fv) if fv else None
write_b = 1024 * sum(wv) / len(wv) if wv else None
summary = {"workload": workload, "batch": batch, "kernel": kname, "avg_ns": avg_ns,
           "launches_traced": len(trace),
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": (fetch_b + write_b) if fv and wv else None,
           "hbm_bytes_per_qp": ((fetch_b + write_b) / batch) if fv and wv else None,
           "achieved_hbm_tbs": ((fetch_b + write_b) / (avg_ns * 1e-9) / 1e12) if fv and wv and avg_ns else None,
           "note": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads) + WRITE_SIZE; KB units x1024"}
(dst / f"{workload}_summary.json").write_text(json.dumps(summary, indent=1))
tf = repo / "profiles" / "pmc_traffic.json"
allp = json.loads(tf.read_text()) if tf.exists() else {}
allp[workload] = summary
tf.write_text(json.dumps(allp, indent=1))
print(json.dumps(summary, indent=1))
