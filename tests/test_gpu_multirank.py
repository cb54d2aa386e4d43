"""BASELINE config 4 (batch 262144 over 8 GPUs, RCCL gather of the solutions)
rehearsed on one GPU: two ranks, each its own process on cuda:0, run bench.py's
own path -- shard generated from seed + global QP index (device_shard), solved
through the C-ABI (shard_buffers + solve_device), gathered to rank 0
(gather_solutions) -- at config 4's per-GPU shard of 32768 QPs.  The gather goes
through a gloo group with host-staged payloads (one GPU cannot host an RCCL ring
of two ranks); the RCCL path is the same dist.gather call on device tensors.

Rank 0 then solves the global indices [0, 65536) in one process and the gathered
x / u / pi must be bit-identical to it: sharding changes nothing about any QP."""
import importlib.util
import json
import os
import socket
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
PER_RANK = 32768  # 262144 / 8
SEED = 1003


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _solve_shard(bench, pkg, batch, rank, device):
    N = 20
    h = pkg.capi.Handle(N, 12, 12, 0, False, False, capacity=batch, device=0)
    dt, _, _, _ = bench.device_shard(pkg, h, N, "none", batch, rank, SEED, device)
    sol_t, data, sol = bench.shard_buffers(pkg.capi, dt, batch, N, "f64", device)
    h.solve_device(batch, pkg.capi.settings_struct(bench.NMPC_SETTINGS), data, sol)
    h.synchronize()
    return h, dt, sol_t


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bench = _bench()
        pkg = bench.import_pkg()
        torch.cuda.set_device(0)
        device = torch.device("cuda", 0)
        h, dt, sol_t = _solve_shard(bench, pkg, PER_RANK, rank, device)
        ok = int((sol_t["status"] == 0).sum().item())
        got = bench.gather_solutions(pkg, sol_t, world, rank, cpu_staged=True)
        t = pkg.dist.max_over_ranks(float(rank + 1), torch.device("cpu"))
        if rank == 0:
            del h, dt, sol_t
            torch.cuda.empty_cache()
            hg, _, ref = _solve_shard(bench, pkg, world * PER_RANK, 0, device)
            want = pkg.dist.solution_payload(ref["x"], ref["u"], ref["pi"]).cpu()
            allp = torch.cat(got, 0)
            res = {"shape": list(allp.shape), "want_shape": list(want.shape),
                   "bitwise_equal": bool(torch.equal(allp, want)),
                   "max_abs_diff": float((allp - want).abs().max().item()),
                   "rank0_ok": ok, "global_ok": int((ref["status"] == 0).sum().item()),
                   "t_max": t}
            (Path(out_dir) / "multirank.json").write_text(json.dumps(res))
    finally:
        dist.destroy_process_group()


def test_two_ranks_config4_shard_solve_gather(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = json.loads((tmp_path / "multirank.json").read_text())
    assert res["shape"] == res["want_shape"] == [world * PER_RANK, 21 * 12 + 20 * 12 + 21 * 12]
    assert res["rank0_ok"] == PER_RANK and res["global_ok"] == world * PER_RANK
    assert res["t_max"] == 2.0  # the slowest rank's time
    assert res["bitwise_equal"], res["max_abs_diff"]


def _rccl_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        bench = _bench()
        pkg = bench.import_pkg()
        device = torch.device("cuda", 0)
        h, dt, sol_t = _solve_shard(bench, pkg, 4096, rank, device)
        dist.barrier()
        got = bench.gather_solutions(pkg, sol_t, world, rank, cpu_staged=False)
        torch.cuda.synchronize()
        walls = [None] * world
        dist.all_gather_object(walls, 1.5)
        want = pkg.dist.solution_payload(sol_t["x"], sol_t["u"], sol_t["pi"])
        res = {"n": len(got), "device": str(got[0].device), "equal": bool(torch.equal(got[0], want)),
               "walls": walls, "backend": dist.get_backend()}
        (Path(out_dir) / "rccl.json").write_text(json.dumps(res))
    finally:
        dist.destroy_process_group()


def test_rccl_single_rank_gather(tmp_path):
    """bench.py's RCCL branch (the nccl process group, dist.gather of device tensors in
    gather_solutions, barrier, all_gather_object) executed for real with one rank on cuda:0 --
    one GPU cannot hold two RCCL ranks; the config-4 collective across 8 devices is the
    driver's run."""
    import torch.multiprocessing as mp
    mp.spawn(_rccl_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    res = json.loads((tmp_path / "rccl.json").read_text())
    assert res["backend"] == "nccl" and res["n"] == 1 and res["device"] == "cuda:0"
    assert res["equal"] and res["walls"] == [1.5]
