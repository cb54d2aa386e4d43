"""CPU-side checks of the C-ABI library: it loads, exports every entry point
include/srbd_qp.h declares, validates arguments, and fails loudly without a GPU."""
import ctypes as C
import subprocess

import numpy as np
import pytest

import helpers


def test_library_exports_every_declared_symbol(pkg):
    capi = pkg.capi
    declared = capi.exported_symbols()
    assert "srbd_qp_solve_f64" in declared and "srbd_qp_create" in declared
    out = subprocess.run(["nm", "-D", "--defined-only", str(capi.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    L = capi.lib()
    for s in declared:
        assert hasattr(L, s)


def test_abi_version_and_strings(pkg):
    L = pkg.capi.lib()
    assert L.srbd_qp_abi_version() == 12
    # hpipm::to_string (ocp_qp_ipm_solver.cpp:19-33)
    assert pkg.capi.status_string(0) == "HpipmStatus::Success"
    assert pkg.capi.status_string(1) == "HpipmStatus::MaxIterReached"
    assert pkg.capi.status_string(2) == "HpipmStatus::MinStepLengthReached"
    assert pkg.capi.status_string(3) == "HpipmStatus::NaNDetected"
    assert pkg.capi.status_string(4) == "HpipmStatus::UnknownFailure"
    assert pkg.capi.status_string(17) == "HpipmStatus::UnknownFailure"


def test_settings_struct_layout_matches_the_header(pkg):
    """The ctypes mirror of srbd_qp_settings ends where the C struct's last field ends:
    srbd_qp_default_settings writes every field, so on a sentinel-filled buffer it
    touches exactly the bytes up to the last field's end (trailing padding untouched),
    and each extension field reads back its documented default."""
    capi = pkg.capi
    buf = (C.c_ubyte * 256)(*([0xAB] * 256))
    capi.lib().srbd_qp_default_settings(C.cast(buf, C.POINTER(capi.Settings)))
    last = capi.Settings._fields_[-1][0]
    end = getattr(capi.Settings, last).offset + C.sizeof(C.c_int)
    assert all(b == 0xAB for b in bytes(buf)[end:]), "C struct is larger than the ctypes mirror"
    s = capi.Settings.from_buffer(buf)
    assert (s.compute_residuals, s.f64_rescue, s.f32_iters) == (1, 0, 0)


def test_extension_settings_are_validated(pkg):
    capi = pkg.capi
    for key in ("f64_rescue", "f32_iters"):
        s = capi.settings_struct({key: -1})
        assert capi.lib().srbd_qp_check_settings(C.byref(s)) == -6  # SRBD_QP_ESETTINGS
        assert key in capi.lib().srbd_qp_last_error().decode()


def test_default_settings_match_hpipm_cpp(pkg):
    s = pkg.capi.settings_struct()
    # hpipm-cpp/include/hpipm-cpp/ocp_qp_ipm_solver_settings.hpp:26-86
    assert s.mode == 1 and s.iter_max == 15 and s.alpha_min == 1e-8 and s.mu0 == 1e2
    assert s.tol_stat == s.tol_eq == s.tol_ineq == s.tol_comp == 1e-8
    assert s.reg_prim == 1e-12 and s.warm_start == 0 and s.pred_corr == 1
    assert s.ric_alg == 1 and s.split_step == 0


@pytest.mark.parametrize("field,value,msg", [
    ("iter_max", -1, "iter_max must be non-negative"),
    ("alpha_min", 0.0, "alpha_min must be positive"),
    ("alpha_min", 2.0, "alpha_min must be less than 1.0"),
    ("mu0", 0.0, "mu0 must be positive"),
    ("tol_stat", 0.0, "tol_stat must be positive"),
    ("tol_eq", -1.0, "tol_eq must be positive"),
    ("tol_ineq", 0.0, "tol_ineq must be positive"),
    ("tol_comp", 0.0, "tol_comp must be positive"),
    ("reg_prim", -1.0, "reg_prim must be non-negative"),
])
def test_check_settings_messages(pkg, field, value, msg):
    """Same rules and messages as OcpQpIpmSolverSettings::checkSettings (settings.cpp:7-38)."""
    L = pkg.capi.lib()
    s = pkg.capi.settings_struct({field: value})
    rc = L.srbd_qp_check_settings(C.byref(s))
    assert rc == -6
    assert msg in L.srbd_qp_last_error().decode()


def test_create_rejects_bad_dims(pkg):
    capi = pkg.capi
    with pytest.raises(capi.SrbdQpError, match="nx must be"):
        capi.Handle(10, 13, 12)
    with pytest.raises(capi.SrbdQpError, match="N must be"):
        capi.Handle(0, 12, 12)


def test_no_cpu_fallback(pkg):
    """Without a GPU the library refuses to run instead of computing on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg.capi.SrbdQpError, match="no HIP device|no GPU"):
        pkg.capi.Handle(10, 12, 12, capacity=4)
    qp, x0 = helpers.random_unconstrained(2, 5, 4, 3, 0, pkg.OcpQpBatch)
    with pytest.raises(pkg.capi.SrbdQpError):
        pkg.capi.solve(qp, x0)


def test_mode_selects_the_same_refinement_in_library_and_checker(pkg, oracle):
    """settings.mode follows hpipm::HpipmMode (SpeedAbs, Speed, Balance, Robust =
    0..3, ocp_qp_ipm_solver_settings.hpp) and selects HPIPM's itref_corr_max 0 / 0 / 2 / 4
    in the HIP library (srbd_qp_capi.hip) and in the CPU checker alike."""
    assert pkg.capi.MODES == {"SpeedAbs": 0, "Speed": 1, "Balance": 2, "Robust": 3}
    src = (helpers.REPO / "srbd-nmpc-solver_amd" / "csrc" / "srbd_qp_capi.hip").read_text()
    assert "a.itref_corr_max = st->mode == 2 ? 2 : st->mode == 3 ? 4 : 0;" in src
    for name, code in pkg.capi.MODES.items():
        want = {0: 0, 1: 0, 2: 2, 3: 4}[code]
        assert oracle.MODE_ITREF[name] == want and oracle.MODE_ITREF[code] == want
        assert oracle._settings({"mode": name}).itref_corr_max == want
    assert oracle._settings({"mode": "Balance", "itref_corr_max": 0}).itref_corr_max == 0
