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
# per kernel name: launches, average duration, HBM bytes per launch
per = {}
for r in stats:
    per[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                      "total_ns": float(r["TotalDurationNs"])}
for rows_, key, scale in ((fetch, "FETCH_SIZE", 2 * 1024), (write, "WRITE_SIZE", 1024)):
    acc = {}
    for r in rows_:
        if r["Counter_Name"] == key:
            acc.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * scale)
    for name, v in acc.items():
        e = per.setdefault(name, {})
        e[key.lower() + "_bytes_per_launch"] = sum(v) / len(v)
        e[key.lower() + "_launches"] = len(v)
for e in per.values():
    if "fetch_size_bytes_per_launch" in e and "write_size_bytes_per_launch" in e:
        e["hbm_bytes_per_launch"] = e["fetch_size_bytes_per_launch"] + e["write_size_bytes_per_launch"]
        if e.get("avg_ns"):
            e["achieved_hbm_tbs"] = e["hbm_bytes_per_launch"] / (e["avg_ns"] * 1e-9) / 1e12
solves = int(sys.argv[4]) if len(sys.argv) > 4 else 6  # bench: warmup 1 + steps 5
tot_ns = sum(e.get("total_ns", 0.0) for e in per.values())
tot_b = sum(e.get("hbm_bytes_per_launch", 0.0) * e.get("calls", 0) for e in per.values())
kname = stats[0]["Name"] if stats else None
dom = per.get(kname, {})
summary = {"workload": workload, "batch": batch, "profile": f"profiles/{tag}/{workload}_summary.json",
           "kernel": kname, "avg_ns": dom.get("avg_ns"),
           "launches_traced": len(trace),
           "fetch_bytes_per_launch": dom.get("fetch_size_bytes_per_launch"),
           "write_bytes_per_launch": dom.get("write_size_bytes_per_launch"),
           "hbm_bytes_per_launch": dom.get("hbm_bytes_per_launch"),
           "hbm_bytes_per_qp": (dom["hbm_bytes_per_launch"] / batch) if "hbm_bytes_per_launch" in dom else None,
           "achieved_hbm_tbs": dom.get("achieved_hbm_tbs"),
           "per_solve": {"solves": solves, "ms": tot_ns / solves * 1e-6,
                         "hbm_bytes": tot_b / solves, "hbm_bytes_per_qp": tot_b / solves / batch,
                         "achieved_hbm_tbs": tot_b / max(tot_ns, 1.0) / 1e3},
           "kernels": per,
           "note": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads) + WRITE_SIZE; KB units x1024; "
                   "per_solve sums every srbd:: kernel launch of the run / solves"}
(dst / f"{workload}_summary.json").write_text(json.dumps(summary, indent=1))
tf = repo / "profiles" / "pmc_traffic.json"
allp = json.loads(tf.read_text()) if tf.exists() else {}
allp[workload] = {k: v for k, v in summary.items() if k != "kernels"}
tf.write_text(json.dumps(allp, indent=1))
print(json.dumps(summary, indent=1))
