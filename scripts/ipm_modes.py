#!/usr/bin/env python3
"""IPM cost by HPIPM mode / Riccati variant / lq_fact on SRBD QPs (N = 20): one C-ABI call per
solve on device buffers, timed wall-clock around solve + synchronize (median of REPS after one
warm-up).  Prints one JSON line {case: {ms, iters_mean, success, lq_iters_mean}}.
Usage: ipm_modes.py [BATCH] [REPS] [box_u|cone]"""
import importlib.util
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
CASES = {
    "speed_ric0": dict(mode="Speed", ric_alg=0),
    "speed_ric1": dict(mode="Speed", ric_alg=1),
    "speed_ric1_lq2": dict(mode="Speed", ric_alg=1, lq_fact=2),
    "balance_ric0": dict(mode="Balance", ric_alg=0),
    "balance_ric1_lq1": dict(mode="Balance", ric_alg=1),
    "robust_ric0": dict(mode="Robust", ric_alg=0),
    "robust_ric1_lq2": dict(mode="Robust", ric_alg=1),
}


def main():
    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    pkg = bench.import_pkg()
    import torch
    capi = pkg.capi
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cons = sys.argv[3] if len(sys.argv) > 3 else "box_u"
    ng = 24 if cons == "cone" else 0
    h = capi.Handle(20, 12, 12, ng, cons == "box_u", False, capacity=batch)
    dt, _, _, _ = bench.device_shard(pkg, h, 20, cons, batch, 0, 1003, "cuda:0")
    st, data, sol = bench.shard_buffers(capi, dt, batch, 20, "f64", "cuda:0")
    out = {}
    for name, case in CASES.items():
        s = capi.settings_struct(dict(bench.NMPC_SETTINGS, **case))
        torch.cuda.synchronize()
        ts = []
        for r in range(reps + 1):
            t0 = time.perf_counter()
            h.solve_device(batch, s, data, sol)
            h.synchronize()
            ts.append(time.perf_counter() - t0)
        it = st["iter"].cpu().numpy()
        out[name] = {"ms": float(np.median(ts[1:])) * 1e3, "iters_mean": float(it.mean()),
                     "success": float((st["status"].cpu().numpy() == 0).mean())}
        print(name, out[name], file=sys.stderr, flush=True)
    h.close()
    print(json.dumps({"batch": batch, "constraints": cons, "cases": out}), flush=True)


if __name__ == "__main__":
    main()
