"""srbd-nmpc-solver_amd -- MI355X-native batched OCP-QP Riccati/IPM solver.

Drop-in for the hot path of liwanyue123/SRBD-NMPC-Solver: the
``hpipm::OcpQpIpmSolver::solve()`` call (hpipm-cpp/src/ocp_qp_ipm_solver.cpp:181)
and the HPIPM/BLASFEO Riccati + IPM beneath it.  The product is the C-ABI
library ``libsrbd_qp.so`` (include/srbd_qp.h, HIP kernels in csrc/); this
Python package is the host-side mirror used by tests and bench.py:

* :class:`OcpQpBatch` -- batched ``hpipm::OcpQp`` in the C-ABI layout.
* :mod:`.capi` -- ctypes binding of libsrbd_qp.so (device pointers from torch).
* :mod:`.srbd_model` -- seeded SRBD QP generator (the reference's linearisation).
* :mod:`.dist` -- rank sharding / solution gather of the multi-GPU bench.

The reference's C++ interface (``hpipm::OcpQpIpmSolver`` & co.) is rebuilt in
``hpipm-cpp/`` (libhpipm-cpp.so) on top of the same C-ABI.

There is no CPU fallback: every solve runs the HIP kernels and raises if the
library or a GPU is missing.
"""
from .qp import OcpQpBatch, dense_box_from_index, colmajor  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must work on a CPU-only host (tests, build()).
    if name in ("capi", "srbd_model", "dist"):
        import importlib
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
