// OcpQpIpmSolverSettings::checkSettings -- the rules of
// hpipm-cpp/src/ocp_qp_ipm_solver_settings.cpp:7-38, delegated to the C-ABI's
// srbd_qp_check_settings so that host code and library agree on one rule set.
#include "hpipm-cpp/ocp_qp_ipm_solver_settings.hpp"

#include <stdexcept>
#include <string>

#include "srbd_qp.h"

namespace hpipm {

void OcpQpIpmSolverSettings::checkSettings() const {
  srbd_qp_settings s;
  srbd_qp_default_settings(&s);
  s.mode = static_cast<int>(mode);
  s.iter_max = iter_max;
  s.alpha_min = alpha_min;
  s.mu0 = mu0;
  s.tol_stat = tol_stat;
  s.tol_eq = tol_eq;
  s.tol_ineq = tol_ineq;
  s.tol_comp = tol_comp;
  s.reg_prim = reg_prim;
  s.warm_start = warm_start;
  s.pred_corr = pred_corr;
  s.ric_alg = ric_alg;
  s.split_step = split_step;
  s.f32_iters = f32_iters;
  if (srbd_qp_check_settings(&s) != SRBD_QP_OK) throw std::runtime_error(srbd_qp_last_error());
}

}  // namespace hpipm
