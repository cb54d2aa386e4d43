"""config/mpc_option.yaml as NMPCSolver::readYaml reads it (NMPC_solver.cpp:22-46):
srbd_model.load_mpc_option and its mapping onto the C-ABI's srbd_model_params."""
import pytest

# the reference's config file layout and values (config/mpc_option.yaml:1-18)
MPC_OPTION = """
MPC:
  Q: [0,0,0,0,0,0,0,0,0,0,0,10]
  Qf: [0.5,0.5,0.5,0.01,0.01,0.01,100,100,100,0.0,0.0,100.0]
  R: 0.0001
  dt_MPC: 0.015
  horizon_MPC: 20
  sqp_max_loop: 15
Physical:
  Lbody: [0.541667, 0.516667, 1.0416667]
N_rep: 100
mu_b: 0.1
theta_b: 5.0
"""


def test_reference_config_equals_defaults(pkg, tmp_path):
    f = tmp_path / "mpc_option.yaml"
    f.write_text(MPC_OPTION)
    p, extra = pkg.srbd_model.load_mpc_option(str(f))
    assert p == pkg.srbd_model.SrbdParams()
    assert extra == {"sqp_max_loop": 15, "N_rep": 100}
    m = pkg.capi.model_params(p)
    d = pkg.capi.default_model_params()
    for name, _ in m._fields_:
        a, b = getattr(m, name), getattr(d, name)
        assert (list(a) if hasattr(a, "__len__") else a) == (list(b) if hasattr(b, "__len__") else b), name


def test_config_values_flow_through(pkg):
    text = MPC_OPTION.replace("horizon_MPC: 20", "horizon_MPC: 40").replace("R: 0.0001", "R: 0.002")
    text = text.replace("mu_b: 0.1", "mu_b: 0.25")
    p, _ = pkg.srbd_model.load_mpc_option(text)
    assert (p.N, p.R, p.mu_b) == (40, 0.002, 0.25)
    m = pkg.capi.model_params(p)
    assert (m.R, m.mu_b, m.dt) == (0.002, 0.25, 0.015)


def test_config_errors(pkg):
    with pytest.raises(KeyError):
        pkg.srbd_model.load_mpc_option(MPC_OPTION.replace("sqp_max_loop", "sqp_loops"))
    with pytest.raises(ValueError, match="MPC.Q needs 12"):
        pkg.srbd_model.load_mpc_option(MPC_OPTION.replace("Q: [0,0,0,0,0,0,0,0,0,0,0,10]", "Q: [1,2]"))
