#!/usr/bin/env python3
"""Small-batch IPM latency: box-u SRBD QPs, N = 20, the NMPC's
settings (iter_max 30), batches 1 / 16 / 256 / 512 / 1024, one C-ABI call per solve on device
buffers; prints one JSON line {batch: {median_ms, min_ms, iters_max, iters_mean}}.
SRBD_QP_LIB selects the library (A/B against an older build); SRBD_IPM_LATENCY_MAX=0 in the
environment keeps every batch on the batched kernels (ipm_latency.hip is the default up to 512).
Usage: ipm_small_batch.py [reps] [constraints] [mode] [ric_alg]  (mode: HPIPM's Speed / Balance /
Robust; the NMPC's Speed and classical Riccati (ric_alg 0) by default)"""
import importlib.util
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]


def main():
    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    pkg = bench.import_pkg()
    import torch
    capi = pkg.capi
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    cons = sys.argv[2] if len(sys.argv) > 2 else "box_u"
    settings = dict(bench.NMPC_SETTINGS)
    if len(sys.argv) > 3:
        settings["mode"] = sys.argv[3]
    if len(sys.argv) > 4:
        settings["ric_alg"] = int(sys.argv[4])
    out = {}
    for batch in (1, 16, 256, 512, 1024):
        qp, x0 = pkg.srbd_model.generate_batch(batch, N=20, seed=11, constraints=cons)
        h = capi.Handle(20, 12, 12, qp.ng, qp.has_box_u, qp.has_box_x, capacity=batch)
        s = capi.settings_struct(settings)
        dt, st, data, sol = capi.device_buffers(qp, x0)
        torch.cuda.synchronize()
        ts = []
        for r in range(reps + 2):
            t0 = time.perf_counter()
            h.solve_device(batch, s, data, sol)
            h.synchronize()
            ts.append(time.perf_counter() - t0)
        it = st["iter"].cpu().numpy()
        out[batch] = {"median_ms": float(np.median(ts[2:])) * 1e3, "min_ms": float(np.min(ts[2:])) * 1e3,
                      "iters_max": int(it.max()), "iters_mean": float(it.mean()),
                      "success": float((st["status"].cpu().numpy() == 0).mean())}
        h.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
