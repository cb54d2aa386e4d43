"""`bench.py --gpus 2` end to end on one GPU: the script starts its own two
ranks (no external launcher), each solves its 4096-QP shard on cuda:0, the
solutions are gathered to rank 0 over a gloo group (host-staged: one GPU cannot
host an RCCL ring of two ranks), and rank 0 prints ONE JSON line whose value is
the global batch x steps / the slowest rank's wall time."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def test_bench_gpus2_gloo_line():
    steps = 3
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--batch", "4096",
           "--dist-backend", "gloo", "--no-secondary", "--no-host-path", "--no-pipeline",
           "--steps", str(steps), "--warmup", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps
    assert d["config"]["global_batch"] == 8192 and d["config"]["batch_per_gpu"] == 4096
    assert d["config"]["dist_backend"] == "gloo"
    walls = d["config"]["rank_ms_per_step"]
    assert len(walls) == 2
    assert d["ms_per_step"] == pytest.approx(max(walls), rel=1e-9)
    assert d["value"] == pytest.approx(8192 / (max(walls) * 1e-3), rel=1e-9)
    g = d["gather"]
    assert g["ms"] > 0 and g["bytes_per_rank"] == 4096 * (2 * 21 * 12 + 20 * 12) * 8
    assert g["value_with_gather"] < d["value"]
    assert d["success_rate"] == 1.0
