# Dev aid: kernel + HIP API trace of the reference call pattern (one QP per solve)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r4
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
timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d gpurun_out/r4/prof_call -o run -- ./build/call_pattern_bench /tmp/qp.bin 5 || exit 1
python3 - <<'PY'
import csv, glob
for kind in ("kernel_stats", "hip_api_stats"):
    fs = glob.glob(f"gpurun_out/r4/prof_call/**/*{kind}.csv", recursive=True)
    if not fs: continue
    for x in csv.DictReader(open(fs[0])):
        print(kind, x["Name"][:60], x["Calls"], "avg %.1f us" % (float(x["AverageNs"]) / 1e3), "tot %.0f us" % (float(x["TotalDurationNs"]) / 1e3))
PY
