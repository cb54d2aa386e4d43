"""Batched OCP-QP container in the C-ABI memory layout (include/srbd_qp.h).

Host-side mirror of the reference's ``hpipm::OcpQp`` stage struct
(hpipm-cpp/include/hpipm-cpp/ocp_qp.hpp:15-177), batched: every field carries a
leading batch dimension and all stages of one field are stored contiguously.

Matrices are kept here in *math orientation* (``A[b, k, i, j]`` = row i,
column j).  :meth:`OcpQpBatch.packed` returns the column-major-per-block
buffers the C-ABI expects (Eigen's default storage, which is what
``d_ocp_qp_set_all`` reads in hpipm-cpp/src/ocp_qp_ipm_solver.cpp:283-289).

Box constraints use the dense per-variable representation of the C-ABI: one
bound per variable with a 0/1 mask (a masked bound is absent).  The index-list
form of the reference (``idxbu``/``idxbx``) is converted by
:func:`dense_box_from_index`.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

__all__ = ["OcpQpBatch", "dense_box_from_index", "colmajor"]


def colmajor(m: np.ndarray) -> np.ndarray:
    """Contiguous buffer whose memory is the column-major storage of each trailing 2-D block."""
    return np.ascontiguousarray(np.swapaxes(m, -1, -2), dtype=np.float64)


def dense_box_from_index(n: int, idx, lb, ub, lb_mask=None, ub_mask=None):
    """Convert the reference's (idxb, lb, ub, masks) of one stage into dense arrays.

    Mirrors how ``d_ocp_qp_set_all`` + ``d_ocp_qp_set_l*_mask`` define box
    constraints (hpipm-cpp/src/ocp_qp_ipm_solver.cpp:283-321).  Returns
    ``(lb_d, ub_d, lb_mask_d, ub_mask_d)`` of length ``n``; variables not in
    ``idx`` get mask 0.  Duplicate indices are rejected (ValueError).
    """
    idx = list(int(i) for i in idx)
    if len(set(idx)) != len(idx):
        raise ValueError("duplicate box-constraint indices are not supported")
    lbd = np.zeros(n)
    ubd = np.zeros(n)
    lmd = np.zeros(n)
    umd = np.zeros(n)
    for c, i in enumerate(idx):
        if not 0 <= i < n:
            raise ValueError(f"box index {i} out of range [0, {n})")
        lbd[i] = lb[c]
        ubd[i] = ub[c]
        lmd[i] = 1.0 if lb_mask is None or len(lb_mask) == 0 else float(lb_mask[c])
        umd[i] = 1.0 if ub_mask is None or len(ub_mask) == 0 else float(ub_mask[c])
    return lbd, ubd, lmd, umd


@dataclass
class OcpQpBatch:
    """A batch of OCP-QPs with uniform dimensions (N, nx, nu, ng)."""

    N: int
    nx: int
    nu: int
    A: np.ndarray  # (batch, N, nx, nx)
    B: np.ndarray  # (batch, N, nx, nu)
    b: np.ndarray  # (batch, N, nx)
    Q: np.ndarray  # (batch, N+1, nx, nx)
    S: np.ndarray  # (batch, N, nu, nx)
    R: np.ndarray  # (batch, N, nu, nu)
    q: np.ndarray  # (batch, N+1, nx)
    r: np.ndarray  # (batch, N, nu)
    lbu: Optional[np.ndarray] = None  # (batch, N, nu)
    ubu: Optional[np.ndarray] = None
    lbu_mask: Optional[np.ndarray] = None
    ubu_mask: Optional[np.ndarray] = None
    lbx: Optional[np.ndarray] = None  # (batch, N+1, nx); stage 0 ignored
    ubx: Optional[np.ndarray] = None
    lbx_mask: Optional[np.ndarray] = None
    ubx_mask: Optional[np.ndarray] = None
    ng: int = 0
    C: Optional[np.ndarray] = None  # (batch, N+1, ng, nx); stage 0 ignored
    D: Optional[np.ndarray] = None  # (batch, N, ng, nu)
    lg: Optional[np.ndarray] = None  # (batch, N+1, ng)
    ug: Optional[np.ndarray] = None
    lg_mask: Optional[np.ndarray] = None
    ug_mask: Optional[np.ndarray] = None
    meta: Dict = field(default_factory=dict)

    @property
    def batch(self) -> int:
        return int(self.A.shape[0])

    @property
    def has_box_u(self) -> bool:
        return self.lbu is not None

    @property
    def has_box_x(self) -> bool:
        return self.lbx is not None

    @property
    def has_general(self) -> bool:
        return self.ng > 0 and self.lg is not None

    @property
    def num_constraints(self) -> int:
        """Number of active inequality sides per QP (max over the batch)."""
        nc = np.zeros(self.batch)
        if self.has_box_u:
            lm = np.ones_like(self.lbu) if self.lbu_mask is None else (self.lbu_mask != 0)
            um = np.ones_like(self.ubu) if self.ubu_mask is None else (self.ubu_mask != 0)
            nc += lm.reshape(self.batch, -1).sum(1) + um.reshape(self.batch, -1).sum(1)
        if self.has_box_x:
            lm = np.ones_like(self.lbx) if self.lbx_mask is None else (self.lbx_mask != 0)
            um = np.ones_like(self.ubx) if self.ubx_mask is None else (self.ubx_mask != 0)
            nc += lm[:, 1:].reshape(self.batch, -1).sum(1) + um[:, 1:].reshape(self.batch, -1).sum(1)
        if self.has_general:
            lm = np.ones_like(self.lg) if self.lg_mask is None else (self.lg_mask != 0)
            um = np.ones_like(self.ug) if self.ug_mask is None else (self.ug_mask != 0)
            nc += lm.reshape(self.batch, -1).sum(1) + um.reshape(self.batch, -1).sum(1)
        return int(nc.max()) if self.batch else 0

    def check(self) -> None:
        """Shape checks (the batched analogue of OcpQpDim::checkSize, ocp_qp_dim.cpp:59-246)."""
        bt, N, nx, nu, ng = self.batch, self.N, self.nx, self.nu, self.ng
        want = {
            "A": (bt, N, nx, nx), "B": (bt, N, nx, nu), "b": (bt, N, nx),
            "Q": (bt, N + 1, nx, nx), "S": (bt, N, nu, nx), "R": (bt, N, nu, nu),
            "q": (bt, N + 1, nx), "r": (bt, N, nu),
        }
        for name in ("lbu", "ubu", "lbu_mask", "ubu_mask"):
            want[name] = (bt, N, nu)
        for name in ("lbx", "ubx", "lbx_mask", "ubx_mask"):
            want[name] = (bt, N + 1, nx)
        for name in ("lg", "ug", "lg_mask", "ug_mask"):
            want[name] = (bt, N + 1, ng)
        want["C"] = (bt, N + 1, ng, nx)
        want["D"] = (bt, N, ng, nu)
        for name, shape in want.items():
            arr = getattr(self, name)
            if arr is None:
                continue
            if tuple(arr.shape) != shape:
                raise ValueError(f"{name}.shape must be {shape}, got {tuple(arr.shape)}")
        if (self.lbu is None) != (self.ubu is None):
            raise ValueError("lbu and ubu must be given together")
        if (self.lbx is None) != (self.ubx is None):
            raise ValueError("lbx and ubx must be given together")
        if self.ng > 0 and (self.lg is None or self.ug is None):
            raise ValueError("ng > 0 requires lg and ug")

    def packed(self) -> Dict[str, Optional[np.ndarray]]:
        """C-ABI buffers (float64, contiguous, column-major per block)."""
        self.check()
        out: Dict[str, Optional[np.ndarray]] = {}
        for name in ("A", "B", "Q", "S", "R", "C", "D"):
            m = getattr(self, name)
            out[name] = None if m is None else colmajor(m)
        for name in ("b", "q", "r", "lbu", "ubu", "lbu_mask", "ubu_mask", "lbx", "ubx",
                     "lbx_mask", "ubx_mask", "lg", "ug", "lg_mask", "ug_mask"):
            v = getattr(self, name)
            out[name] = None if v is None else np.ascontiguousarray(v, dtype=np.float64)
        if self.ng == 0:
            for name in ("C", "D", "lg", "ug", "lg_mask", "ug_mask"):
                out[name] = None
        return out

    def subset(self, idx) -> "OcpQpBatch":
        """A new batch holding QPs ``idx`` (index array or slice)."""
        kw = {}
        for name in ("A", "B", "b", "Q", "S", "R", "q", "r", "lbu", "ubu", "lbu_mask", "ubu_mask",
                     "lbx", "ubx", "lbx_mask", "ubx_mask", "C", "D", "lg", "ug", "lg_mask", "ug_mask"):
            v = getattr(self, name)
            kw[name] = None if v is None else np.ascontiguousarray(v[idx])
        return OcpQpBatch(N=self.N, nx=self.nx, nu=self.nu, ng=self.ng, meta=dict(self.meta), **kw)
