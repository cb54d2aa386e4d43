"""Dev aid: per-kernel averages of a scripts/profile_ipm.sh run (trace + every PMC pass).

  python scripts/dev/ipm_prof_summary.py gpurun_out/prof_<TAG>_<WORKLOAD> BATCH [out.json]

Per srbd:: kernel: launches, average ns, and each counter's average per launch (FETCH_SIZE
reported x2 and KB -> bytes, WRITE_SIZE KB -> bytes), plus derived HBM bytes per QP and TB/s.
Launches that did no work (every QP exited) are kept: the averages are per launch."""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1])
batch = int(sys.argv[2])
per = defaultdict(lambda: defaultdict(list))
for f in glob.glob(str(src / "trace" / "**" / "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "srbd::" in r["Name"]:
            per[r["Name"]]["calls"] = int(r["Calls"])
            per[r["Name"]]["avg_ns"] = float(r["AverageNs"])
for f in glob.glob(str(src / "*" / "**" / "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "srbd::" not in r["Kernel_Name"]:
            continue
        per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for name, d in per.items():
    e = {"calls": d.get("calls"), "avg_ns": d.get("avg_ns")}
    for k, v in d.items():
        if isinstance(v, list) and v:
            e[k] = sum(v) / len(v)
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
        e["hbm_bytes"] = e["FETCH_SIZE"] * 2 * 1024 + e["WRITE_SIZE"] * 1024
        e["hbm_bytes_per_qp"] = e["hbm_bytes"] / batch
        if e.get("avg_ns"):
            e["hbm_tbs"] = e["hbm_bytes"] / e["avg_ns"] / 1e3
    if "SQ_ACTIVE_INST_VALU" in e and "SQ_WAVE_CYCLES" in e:
        e["valu_frac_of_wave_cycles"] = e["SQ_ACTIVE_INST_VALU"] / max(e["SQ_WAVE_CYCLES"], 1)
        e["wait_frac_of_wave_cycles"] = e.get("SQ_WAIT_INST_ANY", 0) / max(e["SQ_WAVE_CYCLES"], 1)
    if "TCC_HIT_sum" in e:
        e["l2_hit"] = e["TCC_HIT_sum"] / max(e["TCC_HIT_sum"] + e["TCC_MISS_sum"], 1)
    short = name.split("(")[0].replace("void srbd::", "")
    out[short] = e
js = json.dumps(out, indent=1)
if len(sys.argv) > 3:
    Path(sys.argv[3]).write_text(js)
for k, e in out.items():
    print(f"{k:70s} calls {e.get('calls')} avg {e.get('avg_ns', 0) / 1e3:9.1f} us  "
          f"B/QP {e.get('hbm_bytes_per_qp', 0) / 1e3:7.1f} KB  {e.get('hbm_tbs', 0):5.2f} TB/s  "
          f"valu {e.get('valu_frac_of_wave_cycles', 0):.3f} wait {e.get('wait_frac_of_wave_cycles', 0):.3f} "
          f"l2hit {e.get('l2_hit', 0):.3f}")
