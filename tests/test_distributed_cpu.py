"""The N > 1 path of bench.py on CPU: world_size-2 gloo process group running
the same helpers (srbd-nmpc-solver_amd/dist.py) the GPU bench uses over RCCL:
disjoint weak-scaling shards generated per rank from seed + global index, the
max-over-ranks wall time, and the gather of (x, u, pi) to rank 0."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import helpers


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = helpers.load_package()
        D = pkg.dist
        batch, N = 6, 4
        first, last = D.shard_range(rank, batch)
        qp, x0 = pkg.srbd_model.generate_batch(batch, N=N, seed=31, constraints="none", first=first)
        # stand-in "solution" tensors that identify the QP they came from
        x = torch.from_numpy(qp.q[:, :, :].copy())            # [B, N+1, 12]
        u = torch.from_numpy(qp.r.copy())                     # [B, N, 12]
        pi = torch.from_numpy(np.repeat(x0[:, None, :], N + 1, axis=1))
        payload = D.solution_payload(x, u, pi)
        got = D.gather_to_root(payload, world, rank)
        t = D.max_over_ranks(0.1 * (rank + 1), torch.device("cpu"))
        if rank == 0:
            allp = torch.cat(got, 0)
            xs, us, pis = D.unpack_payload(allp, N, 12, 12)
            np.savez(os.path.join(out_dir, "gathered.npz"), x=xs.numpy(), u=us.numpy(),
                     pi=pis.numpy(), t=t)
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_and_gather(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = np.load(tmp_path / "gathered.npz")
    assert float(res["t"]) == pytest.approx(0.2)  # max over ranks
    pkg = helpers.load_package()
    # rank r's shard == QPs [6r, 6r+6) of one global generation
    qp, x0 = pkg.srbd_model.generate_batch(12, N=4, seed=31, constraints="none", first=0)
    np.testing.assert_array_equal(res["x"], qp.q)
    np.testing.assert_array_equal(res["u"], qp.r)
    np.testing.assert_array_equal(res["pi"][:, 0], x0)


def test_shard_ranges_disjoint_cover():
    pkg = helpers.load_package()
    rs = [pkg.dist.shard_range(r, 32768) for r in range(8)]
    assert rs[0] == (0, 32768) and rs[-1][1] == 262144
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
