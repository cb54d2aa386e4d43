"""Dev aid: per-iteration IPM launch durations of one config-5 solve from a rocprofv3 kernel trace
(sqlite or csv under the given directory): how much of the solve is the tail."""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        rows += list(csv.DictReader(fh))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# keep the last solve: from the last init kernel on
names = [r["Kernel_Name"] for r in rows]
idx = [i for i, n in enumerate(names) if "ipm_phase_kernel" in n and ", 0, " in n]
start = idx[-1] if idx else 0
sel = rows[start:]
t0 = int(sel[0]["Start_Timestamp"])
tot = (int(sel[-1]["End_Timestamp"]) - t0) / 1e6
print(f"solve {tot:.2f} ms over {len(sel)} launches")
acc, it = 0.0, 0
cum = 0.0
for r in sel:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    n = r["Kernel_Name"]
    cum += d
    if "ipm_phase2_kernel" in n and ", 1, 2," in n:  # RB+F1 starts an iteration
        print(f"it {it:2d} start at {(int(r['Start_Timestamp']) - t0) / 1e6:8.2f} ms  RB+F1 {d:6.3f} ms")
        it += 1
