"""bench.py's rank launcher on CPU (no GPU touched): `--gpus N` without an
external launcher starts N rank processes with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 set, and a WORLD_SIZE that disagrees with --gpus is
refused with a non-zero exit (--gpus was parsed and ignored)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_n_starts_n_ranks():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3", "--print-ranks"],
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ranks = [json.loads(l) for l in r.stdout.strip().splitlines()]
    assert sorted(x["rank"] for x in ranks) == [0, 1, 2]
    assert all(x["world"] == 3 and x["local_rank"] == x["rank"] for x in ranks)
    assert {x["master"][0] for x in ranks} == {"127.0.0.1"}
    assert len({x["master"][1] for x in ranks}) == 1  # one rendezvous port


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--print-ranks"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def test_single_gpu_needs_no_launcher():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--print-ranks"],
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip())["world"] == 1


def test_roofline_ceiling_derivation():
    """bench.py's roofline.ceiling: the two-sweep Riccati's minimum traffic per QP
    is the algorithmic bytes + the stage records written and read back (246 doubles) + the A, B,
    b the forward sweep reads again; at the achievable 6.3 TB/s that caps the algorithmic
    fraction of the 8 TB/s peak at 0.396 for N = 20, nx = nu = 12."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    c = bench.unconstr_ceiling(128256, 65536)
    assert c["record_round_trip_per_qp"] == 20 * 246 * 8 * 2
    assert c["forward_reread_per_qp"] == 20 * (144 + 144 + 12) * 8
    assert c["min_traffic_per_qp"] == 128256 + 78720 + 48000
    assert abs(c["ceiling"] - 128256 / 254976 * 6300 / 8000) < 1e-12
    assert 0.39 < c["ceiling"] < 0.40
