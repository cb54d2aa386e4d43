"""ctypes wrapper of the CPU parity oracle (oracle/ocp_qp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.  The product
path (libsrbd_qp.so) has no CPU fallback and does not link this library.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time
from pathlib import Path
from typing import Dict, Optional

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liboracle.so"

_dp = C.POINTER(C.c_double)


class _QP(C.Structure):
    _fields_ = [("N", C.c_int), ("nx", C.c_int), ("nu", C.c_int), ("ng", C.c_int)] + [
        (n, _dp) for n in (
            "A", "B", "b", "Q", "S", "R", "q", "r",
            "lbu", "ubu", "lbu_mask", "ubu_mask",
            "lbx", "ubx", "lbx_mask", "ubx_mask",
            "C", "D", "lg", "ug", "lg_mask", "ug_mask")
    ]


class _Settings(C.Structure):
    _fields_ = [("iter_max", C.c_int), ("alpha_min", C.c_double), ("mu0", C.c_double),
                ("tol_stat", C.c_double), ("tol_eq", C.c_double), ("tol_ineq", C.c_double),
                ("tol_comp", C.c_double), ("reg_prim", C.c_double), ("warm_start", C.c_int),
                ("pred_corr", C.c_int), ("split_step", C.c_int), ("ric_alg", C.c_int),
                ("itref_corr_max", C.c_int), ("lq_fact", C.c_int)]


class _Result(C.Structure):
    _fields_ = [("status", C.c_int), ("iter", C.c_int), ("res", C.c_double * 4), ("obj", C.c_double),
                ("lq_iters", C.c_int)]


_lib = None


def build() -> Path:
    """Compile the oracle with its Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        _lib = C.CDLL(str(LIB_PATH))
        _lib.oracle_solve.restype = C.c_int
        _lib.oracle_solve.argtypes = [C.POINTER(_QP), C.POINTER(_Settings), _dp, _dp, _dp, _dp,
                                      _dp, _dp, _dp, _dp, C.POINTER(_Result)]
        _lib.oracle_solve_batch.restype = C.c_int
        _lib.oracle_solve_batch.argtypes = [C.c_int, C.POINTER(_QP), C.POINTER(_Settings), _dp,
                                            _dp, _dp, _dp, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                            C.c_int]
    return _lib


def _ptr(a: Optional[np.ndarray]):
    if a is None:
        return _dp()
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


DEFAULT_SETTINGS = dict(iter_max=15, alpha_min=1e-8, mu0=1e2, tol_stat=1e-8, tol_eq=1e-8,
                        tol_ineq=1e-8, tol_comp=1e-8, reg_prim=1e-12, warm_start=0, pred_corr=1,
                        split_step=0, ric_alg=1, itref_corr_max=0,  # hpipm-cpp defaults (settings.hpp:26-86)
                        lq_fact=0)  # HPIPM: Balance 1, Robust 2 with the square root (MODE_LQ)


# HPIPM's mode-dependent itref_corr_max (d_ocp_qp_ipm_arg_set_default; the HIP library
# derives it from settings.mode the same way, srbd_qp_capi.hip)
MODE_ITREF = {"SpeedAbs": 0, "Speed": 0, "Balance": 2, "Robust": 4, 0: 0, 1: 0, 2: 2, 3: 4}


# and its lq_fact, with the square-root Riccati only (hpipm_d_ocp_qp_ipm.h:78); the HIP library
# derives it the same way (srbd_qp_capi.hip)
MODE_LQ = {"SpeedAbs": 0, "Speed": 0, "Balance": 1, "Robust": 2, 0: 0, 1: 0, 2: 1, 3: 2}


def _settings(s: Optional[Dict], ng: int = 0) -> _Settings:
    d = dict(DEFAULT_SETTINGS)
    if s:
        d.update({k: v for k, v in s.items() if k in d})
        if "mode" in s and "itref_corr_max" not in s:
            d["itref_corr_max"] = MODE_ITREF[s["mode"]]
        if s.get("lq_fact", -1) == -1:  # (-1: the mode's, as the C-ABI's srbd_qp_settings)
            d["lq_fact"] = MODE_LQ[s.get("mode", "Speed")] if d["ric_alg"] else 0
    return _Settings(**d)


def _make_qp(p: Dict[str, Optional[np.ndarray]], N, nx, nu, ng, keep) -> _QP:
    qp = _QP()
    qp.N, qp.nx, qp.nu, qp.ng = N, nx, nu, ng
    for name, _ in _QP._fields_[4:]:
        arr = p.get(name)
        if arr is not None:
            arr = np.ascontiguousarray(arr, dtype=np.float64)
            keep.append(arr)
        setattr(qp, name, _ptr(arr))
    return qp


def solve(batch, settings: Optional[Dict] = None, x0: Optional[np.ndarray] = None,
          x_init=None, u_init=None, riccati: bool = True):
    """Solve every QP of an OcpQpBatch one by one; returns a dict of arrays."""
    p = batch.packed()
    N, nx, nu, ng, nb = batch.N, batch.nx, batch.nu, batch.ng, batch.batch
    st = _settings(settings, batch.ng)
    out = {
        "x": np.zeros((nb, N + 1, nx)), "u": np.zeros((nb, N, nu)), "pi": np.zeros((nb, N + 1, nx)),
        "P": np.zeros((nb, N + 1, nx, nx)), "p": np.zeros((nb, N + 1, nx)),
        "K": np.zeros((nb, N, nu, nx)), "k": np.zeros((nb, N, nu)),
        "status": np.zeros(nb, dtype=np.int32), "iter": np.zeros(nb, dtype=np.int32),
        "res": np.zeros((nb, 4)), "obj": np.zeros(nb), "lq_iters": np.zeros(nb, dtype=np.int32),
    }
    if x_init is not None:
        out["x"][:] = x_init
    if u_init is not None:
        out["u"][:] = u_init
    x0 = np.zeros((nb, nx)) if x0 is None else np.asarray(x0, dtype=np.float64).reshape(nb, nx)
    L = lib()
    for i in range(nb):
        keep = []
        pi_ = {k: (None if v is None else v[i]) for k, v in p.items()}
        qp = _make_qp(pi_, N, nx, nu, ng, keep)
        x = np.ascontiguousarray(out["x"][i])
        u = np.ascontiguousarray(out["u"][i])
        pi = np.zeros((N + 1, nx))
        P = np.zeros((N + 1, nx, nx))
        pv = np.zeros((N + 1, nx))
        K = np.zeros((N, nx, nu))  # col-major nu x nx blocks
        k = np.zeros((N, nu))
        r = _Result()
        x0i = np.ascontiguousarray(x0[i])
        rc = L.oracle_solve(C.byref(qp), C.byref(st), _ptr(x0i), _ptr(x), _ptr(u), _ptr(pi),
                            _ptr(P) if riccati else _dp(), _ptr(pv) if riccati else _dp(),
                            _ptr(K) if riccati else _dp(), _ptr(k) if riccati else _dp(),
                            C.byref(r))
        if rc != 0:
            raise ValueError(f"oracle_solve failed with code {rc}")
        out["x"][i], out["u"][i], out["pi"][i] = x, u, pi
        out["P"][i] = np.swapaxes(P, -1, -2)
        out["p"][i] = pv
        out["K"][i] = np.swapaxes(K, -1, -2)
        out["k"][i] = k
        out["status"][i], out["iter"][i] = r.status, r.iter
        out["res"][i] = list(r.res)
        out["obj"][i] = r.obj
        out["lq_iters"][i] = r.lq_iters
    return out


def solve_batch_threaded(batch, settings: Optional[Dict] = None, x0=None, threads: int = 0):
    """Threaded batch solve (x, u, pi only) -- the cpu_baseline 'port'.  Returns (out, seconds)."""
    p = batch.packed()
    N, nx, nu, ng, nb = batch.N, batch.nx, batch.nu, batch.ng, batch.batch
    threads = threads or os.cpu_count() or 1
    keep = []
    qp = _make_qp(p, N, nx, nu, ng, keep)
    st = _settings(settings, batch.ng)
    x0 = np.zeros((nb, nx)) if x0 is None else np.ascontiguousarray(x0, dtype=np.float64).reshape(nb, nx)
    x = np.zeros((nb, N + 1, nx))
    u = np.zeros((nb, N, nu))
    pi = np.zeros((nb, N + 1, nx))
    status = np.zeros(nb, dtype=np.int32)
    iters = np.zeros(nb, dtype=np.int32)
    t0 = time.perf_counter()
    lib().oracle_solve_batch(nb, C.byref(qp), C.byref(st), _ptr(x0), _ptr(x), _ptr(u), _ptr(pi),
                             status.ctypes.data_as(C.POINTER(C.c_int)),
                             iters.ctypes.data_as(C.POINTER(C.c_int)), int(threads))
    dt = time.perf_counter() - t0
    return {"x": x, "u": u, "pi": pi, "status": status, "iter": iters}, dt


# ---- the cpu_baseline port of the unconstrained solve (oracle/fast_unconstr.c) ----
FAST_LIB_PATH = HERE / "build" / "libfast_unconstr.so"
_fast = None


def fast_lib():
    global _fast
    if _fast is None:
        if not FAST_LIB_PATH.exists():
            build()
        _fast = C.CDLL(str(FAST_LIB_PATH))
        _fast.fast_unconstr_solve_batch.restype = C.c_int
    return _fast


def fast_unconstr_batch(batch, x0, threads: int = 1, reg: float = 1e-12):
    """x, u, pi of an unconstrained nx = nu = 12 batch by the fixed-size CPU port.
    Returns (out, seconds)."""
    p = batch.packed()
    N, nb = batch.N, batch.batch
    assert batch.nx == 12 and batch.nu == 12 and batch.ng == 0
    arr = {k: np.ascontiguousarray(p[k], dtype=np.float64) for k in ("A", "B", "b", "Q", "S", "R", "q", "r")}
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(nb, 12)
    x = np.zeros((nb, N + 1, 12))
    u = np.zeros((nb, N, 12))
    pi = np.zeros((nb, N + 1, 12))
    t0 = time.perf_counter()
    rc = fast_lib().fast_unconstr_solve_batch(
        int(nb), int(N), *(_ptr(arr[k]) for k in ("A", "B", "b", "Q", "S", "R", "q", "r")), _ptr(x0),
        C.c_double(reg), _ptr(x), _ptr(u), _ptr(pi), int(threads))
    dt = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError("fast_unconstr_solve_batch failed")
    return {"x": x, "u": u, "pi": pi}, dt
