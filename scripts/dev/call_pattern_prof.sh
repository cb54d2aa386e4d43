# Dev aid: kernel + HIP API trace of the reference call pattern (one QP per solve)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import helpers
pkg = helpers.load_package()
N = 20
qp, x0 = pkg.srbd_model.generate_batch(1, N=N, seed=1003)
p = qp.packed()
vals = [np.array([float(N)])]
for k in range(N):
    for name in ("A", "B", "b", "Q", "S", "R", "q", "r"):
        vals.append(p[name][0].reshape(N + (1 if name in ("Q", "q") else 0), -1)[k])
vals += [p["Q"][0].reshape(N + 1, -1)[N], p["q"][0].reshape(N + 1, -1)[N], x0[0]]
open("/tmp/qp.bin", "wb").write(np.concatenate(vals).astype("<f8").tobytes())
PY
timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d gpurun_out/prof_call -o run -- ./build/call_pattern_bench /tmp/qp.bin 5 || exit 1
python3 - <<'PY'
import csv, glob
for kind in ("kernel_stats", "hip_api_stats"):
    fs = glob.glob(f"gpurun_out/prof_call/**/*{kind}.csv", recursive=True)
    if not fs: continue
    for x in csv.DictReader(open(fs[0])):
        print(kind, x["Name"][:60], x["Calls"], "avg %.1f us" % (float(x["AverageNs"]) / 1e3), "tot %.0f us" % (float(x["TotalDurationNs"]) / 1e3))
PY
python3 - <<'PY'
# per-call timeline (medians): launch API, launch end -> kernel start, kernel, kernel end -> the
# host's last stream query / synchronize of that call
import csv, glob, statistics as stt
kt = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in
            csv.DictReader(open(glob.glob("gpurun_out/prof_call/**/*kernel_trace.csv", recursive=True)[0])))
api = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Function"]) for x in
             csv.DictReader(open(glob.glob("gpurun_out/prof_call/**/*hip_api_trace.csv", recursive=True)[0])))
launches = [a for a in api if a[2] == "hipLaunchKernel"]
waits = [a for a in api if a[2] in ("hipStreamQuery", "hipStreamSynchronize")]
rows = []
for (ls, le, _), (ks, ke) in zip(launches, kt):
    after = [w for w in waits if w[0] >= ke]
    if not after: continue
    rows.append((le - ls, ks - le, ke - ks, after[0][1] - ke))
if len(rows) < 2:  # (the resident server: one launch serves every call)
    print("timeline: %d kernel launches for the whole run" % len(kt))
else:
    for i, name in enumerate(("launch API", "launch end -> kernel start", "kernel", "kernel end -> host sees it")):
        print("timeline %-28s median %.1f us" % (name, stt.median(r[i] for r in rows) / 1e3))
PY
