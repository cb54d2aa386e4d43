"""Multi-GPU plumbing of the batched solve.

The QPs are independent, so the data path has no collective: every rank owns
a contiguous slice [rank * batch, (rank + 1) * batch) of the global batch and
generates it itself from seed + global QP index.  The only exchange is the
optional gather of the solutions (x, u, pi) to rank 0 after the solve
(BASELINE config 4), and the max-over-ranks reduction of the wall time.

Backend-agnostic: "nccl" (= RCCL over xGMI on ROCm) on the GPU box, "gloo"
in the CPU tests (tests/test_distributed_cpu.py).
"""
from __future__ import annotations

from typing import List, Optional, Tuple


def shard_range(rank: int, batch_per_rank: int) -> Tuple[int, int]:
    """Global QP indices [first, last) owned by `rank` (weak scaling)."""
    first = rank * batch_per_rank
    return first, first + batch_per_rank


def solution_payload(x, u, pi):
    """Pack per-QP x [B, N+1, nx], u [B, N, nu], pi [B, N+1, nx] into one
    contiguous [B, (N+1) nx + N nu + (N+1) nx] tensor (one message per rank)."""
    import torch
    b = x.shape[0]
    return torch.cat([x.reshape(b, -1), u.reshape(b, -1), pi.reshape(b, -1)], dim=1).contiguous()


def unpack_payload(payload, N: int, nx: int, nu: int):
    """Inverse of solution_payload."""
    b = payload.shape[0]
    nxs, nus = (N + 1) * nx, N * nu
    x = payload[:, :nxs].reshape(b, N + 1, nx)
    u = payload[:, nxs:nxs + nus].reshape(b, N, nu)
    pi = payload[:, nxs + nus:].reshape(b, N + 1, nx)
    return x, u, pi


def gather_to_root(payload, world: int, rank: int) -> Optional[List]:
    """dist.gather of every rank's payload to rank 0 (one tensor per rank);
    returns the list on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    bufs = [torch.empty_like(payload) for _ in range(world)] if rank == 0 else None
    dist.gather(payload, bufs, dst=0)
    return bufs


def max_over_ranks(seconds: float, device) -> float:
    """The slowest rank's wall time (the job's time)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
