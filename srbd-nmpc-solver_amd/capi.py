"""ctypes binding of libsrbd_qp.so (the C-ABI declared in include/srbd_qp.h).

Device memory comes from torch (HIP tensors); every call goes through the
HIP kernels.  Importing this module on a host without the built library or
without a GPU works; calling a solve raises :class:`SrbdQpError`.
"""
from __future__ import annotations

import ctypes as C
import sys
import os
from pathlib import Path
from typing import Dict, Optional

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
# SRBD_QP_LIB: an alternative build of the same library (A/B experiments,
# scripts/dev/ab_variants.py); default the in-tree product build
LIB_PATH = Path(os.environ.get("SRBD_QP_LIB") or (PKG_DIR / "libsrbd_qp.so"))

_dp = C.c_void_p


class SrbdQpError(RuntimeError):
    pass


class Dims(C.Structure):
    _fields_ = [("N", C.c_int), ("nx", C.c_int), ("nu", C.c_int), ("ng", C.c_int),
                ("has_box_u", C.c_int), ("has_box_x", C.c_int), ("layout", C.c_int)]


class Settings(C.Structure):
    _fields_ = [("mode", C.c_int), ("iter_max", C.c_int), ("alpha_min", C.c_double),
                ("mu0", C.c_double), ("tol_stat", C.c_double), ("tol_eq", C.c_double),
                ("tol_ineq", C.c_double), ("tol_comp", C.c_double), ("reg_prim", C.c_double),
                ("warm_start", C.c_int), ("pred_corr", C.c_int), ("ric_alg", C.c_int),
                ("split_step", C.c_int), ("compute_residuals", C.c_int),
                ("f64_rescue", C.c_int), ("f32_iters", C.c_int), ("lq_fact", C.c_int)]


DATA_FIELDS = ("A", "B", "b", "Q", "S", "R", "q", "r",
               "lbu", "ubu", "lbu_mask", "ubu_mask",
               "lbx", "ubx", "lbx_mask", "ubx_mask",
               "C", "D", "lg", "ug", "lg_mask", "ug_mask", "x0")
SOL_FIELDS = ("x", "u", "pi", "P", "p", "K", "k", "status", "iter", "res", "obj", "stat")


class Data(C.Structure):
    _fields_ = [(n, _dp) for n in DATA_FIELDS]


class Solution(C.Structure):
    _fields_ = [(n, _dp) for n in SOL_FIELDS]


# srbd_qp_solve_host_cb_f64's callback: void (*)(void* ctx)
FACTORS_CB = C.CFUNCTYPE(None, C.c_void_p)


# fp32 twins (srbd_qp_data_f32 / srbd_qp_solution_f32): same field order
class Data32(C.Structure):
    _fields_ = [(n, _dp) for n in DATA_FIELDS]


class Solution32(C.Structure):
    _fields_ = [(n, _dp) for n in SOL_FIELDS]


MODES = {"SpeedAbs": 0, "Speed": 1, "Balance": 2, "Robust": 3}


class ModelParams(C.Structure):
    """srbd_model_params (include/srbd_qp.h): mpc_option.yaml / setupDynamics."""
    _fields_ = [("Q", C.c_double * 12), ("Qf", C.c_double * 12), ("R", C.c_double),
                ("dt", C.c_double), ("Lbody", C.c_double * 3), ("mu_b", C.c_double),
                ("theta_b", C.c_double), ("mass", C.c_double), ("foot_r", C.c_double * 3),
                ("foot_l", C.c_double * 3), ("mu", C.c_double), ("Lfx", C.c_double),
                ("Lfz", C.c_double), ("fmax", C.c_double), ("fmin", C.c_double),
                ("x_ref", C.c_double * 12), ("qf_scale", C.c_double),
                ("u_lo", C.c_double * 12), ("u_hi", C.c_double * 12)]


SRBD_CONSTRAINTS = {"none": 0, "box_u": 1, "cone": 2}


class LsParams(C.Structure):
    """srbd_linesearch_params (NMPC_solver.h:97-103)."""
    _fields_ = [(n, C.c_double) for n in ("theta_max", "theta_min", "eta", "beta_phi",
                                         "beta_theta", "beta_alpha", "alpha_min")]

_lib = None


def lib():
    """Load libsrbd_qp.so (raises SrbdQpError if it was not built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise SrbdQpError(f"{LIB_PATH} not built; run `make` (or __graft_entry__.build())")
        # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's).
        # Load torch first so that this library binds to the HIP runtime torch
        # already uses: one runtime per process, shared device pointers/streams.
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover - C-only consumers
            pass
        L = C.CDLL(str(LIB_PATH))
        L.srbd_qp_create.argtypes = [C.POINTER(Dims), C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        L.srbd_qp_create.restype = C.c_int
        L.srbd_qp_solve_f64.argtypes = [C.c_void_p, C.c_int, C.POINTER(Settings), C.POINTER(Data),
                                        C.POINTER(Solution), C.c_void_p]
        L.srbd_qp_solve_f64.restype = C.c_int
        L.srbd_qp_solve_host_f64.argtypes = [C.c_void_p, C.c_int, C.POINTER(Settings),
                                             C.POINTER(Data), C.POINTER(Solution)]
        L.srbd_qp_solve_host_f64.restype = C.c_int
        if hasattr(L, "srbd_qp_solve_host_cb_f64"):  # ABI 12
            L.srbd_qp_solve_host_cb_f64.argtypes = [C.c_void_p, C.c_int, C.POINTER(Settings), C.POINTER(Data),
                                                    C.POINTER(Solution), FACTORS_CB, C.c_void_p]
            L.srbd_qp_solve_host_cb_f64.restype = C.c_int
        if hasattr(L, "srbd_qp_multi_create"):  # ABI 10
            L.srbd_qp_multi_create.argtypes = [C.POINTER(Dims), C.c_int, C.POINTER(C.c_int), C.c_int,
                                               C.POINTER(C.c_void_p)]
            L.srbd_qp_multi_create.restype = C.c_int
            L.srbd_qp_multi_destroy.argtypes = [C.c_void_p]
            L.srbd_qp_multi_destroy.restype = None
            L.srbd_qp_multi_handle.argtypes = [C.c_void_p, C.c_int]
            L.srbd_qp_multi_handle.restype = C.c_void_p
            L.srbd_qp_multi_solve_f64.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(Settings),
                                                  C.POINTER(Data), C.POINTER(Solution), C.c_void_p,
                                                  C.c_void_p, C.c_void_p]
            L.srbd_qp_multi_solve_f64.restype = C.c_int
        if hasattr(L, "srbd_qp_multi_solve_f32"):  # ABI 11
            L.srbd_qp_multi_solve_f32.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(Settings),
                                                  C.POINTER(Data32), C.POINTER(Solution32), C.c_void_p,
                                                  C.c_void_p, C.c_void_p]
            L.srbd_qp_multi_solve_f32.restype = C.c_int
        if hasattr(L, "srbd_qp_host_staging_f64"):  # ABI 10 (older builds: A/B runs)
            L.srbd_qp_host_staging_f64.argtypes = [C.c_void_p, C.c_int, C.POINTER(Settings),
                                                   C.POINTER(Data), C.POINTER(Solution)]
            L.srbd_qp_host_staging_f64.restype = C.c_int
        L.srbd_qp_solve_f32.argtypes = [C.c_void_p, C.c_int, C.POINTER(Settings),
                                        C.POINTER(Data32), C.POINTER(Solution32), C.c_void_p]
        L.srbd_qp_solve_f32.restype = C.c_int
        L.srbd_qp_solve_host_f32.argtypes = [C.c_void_p, C.c_int, C.POINTER(Settings),
                                             C.POINTER(Data32), C.POINTER(Solution32)]
        L.srbd_qp_solve_host_f32.restype = C.c_int
        L.srbd_qp_destroy.argtypes = [C.c_void_p]
        L.srbd_qp_destroy.restype = None
        L.srbd_qp_synchronize.argtypes = [C.c_void_p]
        L.srbd_qp_synchronize.restype = C.c_int
        L.srbd_qp_stream.argtypes = [C.c_void_p]
        L.srbd_qp_stream.restype = C.c_void_p
        L.srbd_qp_workspace_bytes.argtypes = [C.c_void_p]
        L.srbd_qp_workspace_bytes.restype = C.c_size_t
        try:  # ABI >= 9 (older builds are still loaded by A/B scripts)
            L.srbd_qp_memory_bytes.argtypes = [C.c_void_p]
            L.srbd_qp_memory_bytes.restype = C.c_size_t
        except AttributeError:
            pass
        L.srbd_qp_default_settings.argtypes = [C.POINTER(Settings)]
        L.srbd_qp_default_settings.restype = None
        L.srbd_qp_check_settings.argtypes = [C.POINTER(Settings)]
        L.srbd_qp_check_settings.restype = C.c_int
        L.srbd_qp_status_string.argtypes = [C.c_int]
        L.srbd_qp_status_string.restype = C.c_char_p
        L.srbd_qp_error_string.argtypes = [C.c_int]
        L.srbd_qp_error_string.restype = C.c_char_p
        L.srbd_qp_last_error.argtypes = []
        L.srbd_qp_last_error.restype = C.c_char_p
        L.srbd_qp_srbd_default_params.argtypes = [C.POINTER(ModelParams)]
        L.srbd_qp_srbd_default_params.restype = None
        L.srbd_qp_srbd_linearize_f64.argtypes = [C.c_void_p, C.c_int, C.POINTER(ModelParams), C.c_int,
                                                 C.c_void_p, C.c_void_p, C.POINTER(Data), C.c_void_p]
        L.srbd_qp_srbd_linearize_f64.restype = C.c_int
        L.srbd_qp_srbd_default_linesearch.argtypes = [C.POINTER(LsParams)]
        L.srbd_qp_srbd_default_linesearch.restype = None
        L.srbd_qp_srbd_linesearch_f64.argtypes = [C.c_void_p, C.c_int, C.POINTER(ModelParams),
                                                  C.POINTER(LsParams)] + [C.c_void_p] * 8
        L.srbd_qp_srbd_linesearch_f64.restype = C.c_int
        L.srbd_qp_srbd_nmpc_f64.argtypes = [C.c_void_p, C.c_int, C.POINTER(ModelParams),
                                            C.POINTER(LsParams), C.POINTER(Settings), C.c_int,
                                            C.c_int] + [C.c_void_p] * 6
        L.srbd_qp_srbd_nmpc_f64.restype = C.c_int
        L.srbd_qp_abi_version.argtypes = []
        L.srbd_qp_abi_version.restype = C.c_int
        _lib = L
    return _lib


def exported_symbols():
    """Names the header declares (used by the CPU export test)."""
    hdr = (PKG_DIR.parent / "include" / "srbd_qp.h").read_text()
    import re
    return sorted(set(re.findall(r"\b(srbd_qp_[a-z0-9_]+)\s*\(", hdr)))


def check(rc: int, what: str = "srbd_qp") -> None:
    if rc != 0:
        L = lib()
        raise SrbdQpError(f"{what}: {L.srbd_qp_error_string(rc).decode()} ({rc}): "
                          f"{L.srbd_qp_last_error().decode()}")


def settings_struct(s: Optional[Dict] = None) -> Settings:
    st = Settings()
    lib().srbd_qp_default_settings(C.byref(st))
    if s:
        for k, v in s.items():
            if k == "mode":
                v = MODES[v] if isinstance(v, str) else int(v)
            if hasattr(st, k):
                setattr(st, k, v)
    return st


def status_string(code: int) -> str:
    return lib().srbd_qp_status_string(int(code)).decode()


class Handle:
    """Owns a srbd_qp_handle (device workspace + stream) for fixed dims."""

    def __init__(self, N: int, nx: int, nu: int, ng: int = 0, has_box_u: bool = False,
                 has_box_x: bool = False, capacity: int = 1, device: int = 0, layout: int = 0):
        self.dims = Dims(N, nx, nu, ng, int(has_box_u), int(has_box_x), int(layout))
        self.capacity = int(capacity)
        self.device = int(device)
        h = C.c_void_p()
        check(lib().srbd_qp_create(C.byref(self.dims), self.capacity, self.device, C.byref(h)),
              "srbd_qp_create")
        self._h = h

    @property
    def ptr(self):
        return self._h

    def stream(self) -> int:
        return int(lib().srbd_qp_stream(self._h) or 0)

    def workspace_bytes(self) -> int:
        return int(lib().srbd_qp_workspace_bytes(self._h))

    def memory_bytes(self) -> int:
        """Everything the handle holds (workspace + first-use buffers)."""
        return int(lib().srbd_qp_memory_bytes(self._h))

    def synchronize(self) -> None:
        check(lib().srbd_qp_synchronize(self._h), "srbd_qp_synchronize")

    def torch_stream(self):
        """The handle's HIP stream as a torch.cuda.ExternalStream (cached)."""
        import torch
        if getattr(self, "_ext", None) is None:
            self._ext = torch.cuda.ExternalStream(self.stream(), device=torch.device("cuda", self.device))
        return self._ext

    def solve_device(self, batch: int, settings: Settings, data, sol, stream: int = 0,
                     order: bool = True) -> None:
        """Launch on `stream` (0: the handle's own stream).  With order=True and no
        explicit stream, the launch is ordered like a torch op: after the work
        already queued on torch's current stream (which produced the inputs and
        zero-filled the outputs), and torch's stream waits for it in turn."""
        f = lib().srbd_qp_solve_f32 if isinstance(data, Data32) else lib().srbd_qp_solve_f64
        o = _order_before(self, stream, order)
        check(f(self._h, int(batch), C.byref(settings), C.byref(data), C.byref(sol),
                C.c_void_p(stream or None)), f.__name__)
        _order_after(o)

    def host_staging(self, batch: int, settings: Settings, data, sol) -> None:
        """srbd_qp_host_staging_f64: the non-NULL fields of data / sol (markers) become
        pointers into the handle's pinned staging buffer (in place)."""
        check(lib().srbd_qp_host_staging_f64(self._h, int(batch), C.byref(settings), C.byref(data),
                                             C.byref(sol)), "srbd_qp_host_staging_f64")

    def solve_host(self, batch: int, settings: Settings, data, sol, on_factors=None) -> None:
        """srbd_qp_solve_host_*; with `on_factors` (fp64), srbd_qp_solve_host_cb_f64: the
        callable runs once P, p, K, k are final in `sol`'s buffers."""
        if on_factors is not None:
            cb = FACTORS_CB(lambda _ctx: on_factors())
            check(lib().srbd_qp_solve_host_cb_f64(self._h, int(batch), C.byref(settings), C.byref(data),
                                                  C.byref(sol), cb, None), "srbd_qp_solve_host_cb_f64")
            return
        f = lib().srbd_qp_solve_host_f32 if isinstance(data, Data32) else lib().srbd_qp_solve_host_f64
        check(f(self._h, int(batch), C.byref(settings), C.byref(data), C.byref(sol)), f.__name__)

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().srbd_qp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """srbd_qp_multi: one solver over several devices from one thread (a handle per
    device; shards solved concurrently, x / u / pi gathered to devices[0] by peer copies)."""

    def __init__(self, N: int, nx: int, nu: int, devices, ng: int = 0, has_box_u: bool = False,
                 has_box_x: bool = False, capacity: int = 1):
        self.dims = Dims(N, nx, nu, ng, int(has_box_u), int(has_box_x), 0)
        self.devices = list(devices)
        arr = (C.c_int * len(self.devices))(*self.devices)
        m = C.c_void_p()
        check(lib().srbd_qp_multi_create(C.byref(self.dims), int(capacity), arr, len(self.devices),
                                         C.byref(m)), "srbd_qp_multi_create")
        self._m = m

    def solve(self, batches, settings: Settings, datas, sols, root_x=None, root_u=None, root_pi=None):
        """fp64 shards (Data / Solution), or fp32 ones (Data32 / Solution32: srbd_qp_multi_solve_f32)."""
        n = len(self.devices)
        b = (C.c_int * n)(*[int(x) for x in batches])
        f32 = isinstance(datas[0], Data32)
        d = ((Data32 if f32 else Data) * n)(*datas)
        s = ((Solution32 if f32 else Solution) * n)(*sols)
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        fn = "srbd_qp_multi_solve_f32" if f32 else "srbd_qp_multi_solve_f64"
        check(getattr(lib(), fn)(self._m, b, C.byref(settings), d, s, ptr(root_x), ptr(root_u),
                                 ptr(root_pi)), fn)

    def close(self) -> None:
        if getattr(self, "_m", None):
            lib().srbd_qp_multi_destroy(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _order_before(handle: "Handle", stream: int, order: bool):
    """Make the handle's stream wait for torch's current stream (inputs produced and
    outputs allocated / filled there).  No-op with an explicit stream or without an
    initialised torch CUDA context."""
    if stream or not order:
        return None
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return None
    ext = handle.torch_stream()
    cur = torch.cuda.current_stream(torch.device("cuda", handle.device))
    ext.wait_stream(cur)
    return cur, ext


def _order_after(o) -> None:
    """torch's current stream waits for the launch just queued on the handle's stream."""
    if o is not None:
        o[0].wait_stream(o[1])


def _tensor_ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def device_buffers(qp, x0: np.ndarray, device="cuda:0", want_riccati: bool = False,
                   x_init=None, u_init=None, stat_rows: int = 0, dtype=np.float64):
    """Upload an OcpQpBatch (+x0) to device tensors in the C-ABI layout.

    dtype float64 -> srbd_qp_solve_f64 structs, float32 -> the fp32 twins.
    Returns (data_tensors, sol_tensors, Data | Data32, Solution | Solution32)."""
    import torch
    np_t = np.dtype(dtype)
    p = qp.packed()
    p["x0"] = np.ascontiguousarray(x0, dtype=np.float64).reshape(qp.batch, qp.nx)
    dt = {k: (None if v is None else torch.from_numpy(np.ascontiguousarray(v, dtype=np_t)).to(device))
          for k, v in p.items()}
    nb, N, nx, nu = qp.batch, qp.N, qp.nx, qp.nu
    f64 = dict(dtype=torch.float32 if np_t == np.float32 else torch.float64, device=device)
    st = {
        "x": torch.zeros(nb, N + 1, nx, **f64) if x_init is None
        else torch.from_numpy(np.ascontiguousarray(x_init, dtype=np_t)).to(device),
        "u": torch.zeros(nb, N, nu, **f64) if u_init is None
        else torch.from_numpy(np.ascontiguousarray(u_init, dtype=np_t)).to(device),
        "pi": torch.zeros(nb, N + 1, nx, **f64),
        "status": torch.full((nb,), -1, dtype=torch.int32, device=device),
        "iter": torch.full((nb,), -1, dtype=torch.int32, device=device),
        "res": torch.zeros(nb, 4, **f64),
        "obj": torch.zeros(nb, **f64),
    }
    if stat_rows:
        st["stat"] = torch.zeros(nb, stat_rows, 18, **f64)  # HPIPM ws->stat rows
    if want_riccati:
        st["P"] = torch.zeros(nb, N + 1, nx, nx, **f64)  # col-major blocks
        st["p"] = torch.zeros(nb, N + 1, nx, **f64)
        st["K"] = torch.zeros(nb, N, nx, nu, **f64)      # col-major nu x nx blocks
        st["k"] = torch.zeros(nb, N, nu, **f64)
    DataT, SolT = (Data32, Solution32) if np_t == np.float32 else (Data, Solution)
    data = DataT(**{k: _tensor_ptr(dt.get(k)) or None for k in DATA_FIELDS})
    sol = SolT(**{k: _tensor_ptr(st.get(k)) or None for k in SOL_FIELDS})
    return dt, st, data, sol


def solve(qp, x0, settings: Optional[Dict] = None, device: str = "cuda:0", riccati: bool = False,
          x_init=None, u_init=None, handle: Optional[Handle] = None,
          stats: bool = False, dtype=np.float64) -> Dict[str, np.ndarray]:
    """Solve an OcpQpBatch on the GPU through the C-ABI; returns numpy results.

    stats=True also returns "stat" [batch][iter_max+2][18], the per-iteration
    statistics rows (alpha_aff, mu_aff, sigma, alpha_prim, alpha_dual, mu,
    res_stat, res_eq, res_ineq, res_comp, obj, 0...)."""
    import torch
    if not torch.cuda.is_available():
        raise SrbdQpError("no GPU available: libsrbd_qp has no CPU fallback")
    dev_index = torch.device(device).index or 0
    h = handle or Handle(qp.N, qp.nx, qp.nu, qp.ng, qp.has_box_u, qp.has_box_x,
                         capacity=qp.batch, device=dev_index)
    s = settings_struct(settings)
    dt, st, data, sol = device_buffers(qp, x0, device, riccati, x_init, u_init,
                                       stat_rows=(s.iter_max + 2) if stats else 0, dtype=dtype)
    h.solve_device(qp.batch, s, data, sol)
    h.synchronize()
    out = {k: v.cpu().numpy() for k, v in st.items()}
    if riccati:
        out["P"] = np.swapaxes(out["P"], -1, -2)
        out["K"] = np.swapaxes(out["K"], -1, -2)
    if handle is None:
        h.close()
    return out


def default_model_params() -> ModelParams:
    p = ModelParams()
    lib().srbd_qp_srbd_default_params(C.byref(p))
    return p


def model_params(p) -> ModelParams:
    """srbd_model_params from a srbd_model.SrbdParams (e.g. load_mpc_option's), on top
    of the library defaults (box limits, qf_scale = N)."""
    m = default_model_params()
    for name in ("Q", "Qf", "Lbody", "foot_r", "foot_l", "x_ref"):
        arr = getattr(m, name)
        for i, v in enumerate(getattr(p, name)):
            arr[i] = float(v)
    for name in ("R", "dt", "mu_b", "theta_b", "mass", "mu", "Lfx", "Lfz", "fmax", "fmin"):
        setattr(m, name, float(getattr(p, name)))
    return m


def srbd_linearize(handle: Handle, xs, us, constraints: str = "none",
                   params: Optional[ModelParams] = None, stream: int = 0, out=None):
    """Device-side prepareQpStructures: linearise SRBD trajectories xs [B][N+1][12],
    us [B][N][12] (torch fp64 device tensors) into the solver's input buffers.
    Asynchronous on the handle's stream: keep xs / us alive (and do not reuse
    their memory from another stream) until that stream has finished.
    Returns (dict of device tensors in the C-ABI layout, Data)."""
    import torch
    B, N1, _ = xs.shape
    N = N1 - 1
    dev = xs.device
    f = dict(dtype=torch.float64, device=dev)
    if out is not None:  # caller-owned buffers from a previous call (no allocation)
        t = out
        data = Data(**{k: _tensor_ptr(t.get(k)) or None for k in DATA_FIELDS})
        p = params or default_model_params()
        o = _order_before(handle, stream, True)
        check(lib().srbd_qp_srbd_linearize_f64(handle.ptr, int(B), C.byref(p),
                                               SRBD_CONSTRAINTS[constraints], C.c_void_p(xs.data_ptr()),
                                               C.c_void_p(us.data_ptr()), C.byref(data),
                                               C.c_void_p(stream or None)), "srbd_qp_srbd_linearize_f64")
        _order_after(o)
        return t, data
    t = {"A": torch.empty(B, N, 144, **f), "B": torch.empty(B, N, 144, **f),
         "b": torch.empty(B, N, 12, **f), "Q": torch.empty(B, N + 1, 144, **f),
         "S": torch.empty(B, N, 144, **f), "R": torch.empty(B, N, 144, **f),
         "q": torch.empty(B, N + 1, 12, **f), "r": torch.empty(B, N, 12, **f)}
    if constraints == "box_u":
        t["lbu"] = torch.empty(B, N, 12, **f)
        t["ubu"] = torch.empty(B, N, 12, **f)
    elif constraints == "cone":
        t["D"] = torch.empty(B, N, 24 * 12, **f)
        for k in ("lg", "ug", "lg_mask", "ug_mask"):
            t[k] = torch.empty(B, N + 1, 24, **f)
    data = Data(**{k: _tensor_ptr(t.get(k)) or None for k in DATA_FIELDS})
    p = params or default_model_params()
    o = _order_before(handle, stream, True)
    check(lib().srbd_qp_srbd_linearize_f64(handle.ptr, int(B), C.byref(p), SRBD_CONSTRAINTS[constraints],
                                           C.c_void_p(xs.data_ptr()), C.c_void_p(us.data_ptr()),
                                           C.byref(data), C.c_void_p(stream or None)),
          "srbd_qp_srbd_linearize_f64")
    _order_after(o)
    return t, data


def default_linesearch() -> LsParams:
    p = LsParams()
    lib().srbd_qp_srbd_default_linesearch(C.byref(p))
    return p


def srbd_linesearch(handle: Handle, xs, us, dx, du, alpha, params: Optional[ModelParams] = None,
                    ls: Optional[LsParams] = None, stream: int = 0):
    """Device filter line search (NMPCSolver::linearSearch) on a batch: xs/us
    (torch fp64, in place), dx/du the QP step, alpha [B] in/out.  Returns
    (merit [B,3] = phi, theta, dphi; converged [B]) device tensors."""
    import torch
    B = xs.shape[0]
    merit = torch.empty(B, 3, dtype=torch.float64, device=xs.device)
    conv = torch.empty(B, dtype=torch.int32, device=xs.device)
    p = params or default_model_params()
    lp = ls or default_linesearch()
    ptr = lambda t: C.c_void_p(t.data_ptr())
    o = _order_before(handle, stream, True)
    check(lib().srbd_qp_srbd_linesearch_f64(handle.ptr, int(B), C.byref(p), C.byref(lp), ptr(xs),
                                            ptr(us), ptr(dx), ptr(du), ptr(alpha), ptr(merit),
                                            ptr(conv), C.c_void_p(stream or None)),
          "srbd_qp_srbd_linesearch_f64")
    _order_after(o)
    return merit, conv


def srbd_nmpc(handle: Handle, xs, us, x0, alpha, constraints: str = "none",
              settings: Optional[Dict] = None, sqp_max_loop: int = 15,
              params: Optional[ModelParams] = None, ls: Optional[LsParams] = None):
    """The SQP loop of NMPCSolver::controlLoop (NMPC_solver.cpp:362-372) for a batch
    of robots on the device (srbd_qp_srbd_nmpc_f64): xs [B][N+1][12], us [B][N][12]
    (torch fp64, updated in place), x0 [B][12], alpha [B] (in place, the persistent
    alpha_ of NMPC_solver.h:104).  Returns (sqp_iter [B], converged [B]) int32
    device tensors.  Synchronous."""
    import torch
    B = xs.shape[0]
    it = torch.zeros(B, dtype=torch.int32, device=xs.device)
    conv = torch.zeros(B, dtype=torch.int32, device=xs.device)
    p = params or default_model_params()
    lp = ls or default_linesearch()
    s = settings_struct(settings)
    ptr = lambda t: C.c_void_p(t.data_ptr())
    o = _order_before(handle, 0, True)
    check(lib().srbd_qp_srbd_nmpc_f64(handle.ptr, int(B), C.byref(p), C.byref(lp), C.byref(s),
                                      SRBD_CONSTRAINTS[constraints], int(sqp_max_loop), ptr(xs),
                                      ptr(us), ptr(x0), ptr(alpha), ptr(it), ptr(conv)),
          "srbd_qp_srbd_nmpc_f64")
    _order_after(o)
    return it, conv
