// hpipm::OcpQpIpmSolverSettings
// (hpipm-cpp/include/hpipm-cpp/ocp_qp_ipm_solver_settings.hpp:10-86):
// same fields, same defaults, same checkSettings() messages.
#pragma once

namespace hpipm {

enum class HpipmMode { SpeedAbs, Speed, Balance, Robust };

struct OcpQpIpmSolverSettings {
 public:
  HpipmMode mode = HpipmMode::Speed;
  int iter_max = 15;
  double alpha_min = 1.0e-08;
  double mu0 = 1.0e+02;
  double tol_stat = 1.0e-08;
  double tol_eq = 1.0e-08;
  double tol_ineq = 1.0e-08;
  double tol_comp = 1.0e-08;
  double reg_prim = 1.0e-12;
  int warm_start = 0;
  int pred_corr = 1;
  int ric_alg = 1;
  int split_step = 0;
  // Extension (not in the reference; the default keeps its behaviour): the first
  // f32_iters IPM iterations of a constrained solve run in fp32, then fp64 continues
  // from that iterate to the tolerances above (srbd_qp_settings.f32_iters).
  int f32_iters = 0;

  // throws std::runtime_error on an invalid setting
  void checkSettings() const;
};

}  // namespace hpipm
