// hpipm::OcpQpIpmSolverStatistics
// (hpipm-cpp/include/hpipm-cpp/ocp_qp_ipm_solver_statistics.hpp:13-58).
// The per-iteration rows come from the kernel's optional `stat` output
// (include/srbd_qp.h, HPIPM ws->stat layout); lq_fact, itref_* and lin_res_*
// are always 0 (no LQ factorization or iterative refinement is run).
#pragma once

#include <cstddef>
#include <iostream>
#include <string>
#include <vector>

namespace hpipm {

struct OcpQpIpmSolverStatistics {
  int iter = 0;
  double max_res_stat = 0.0;
  double max_res_eq = 0.0;
  double max_res_ineq = 0.0;
  double max_res_comp = 0.0;
  std::vector<double> alpha_aff;
  std::vector<double> mu_aff;
  std::vector<double> sigma;
  std::vector<double> alpha_prim;
  std::vector<double> alpha_dual;
  std::vector<double> mu;
  std::vector<double> res_stat;
  std::vector<double> res_eq;
  std::vector<double> res_ineq;
  std::vector<double> res_comp;
  std::vector<double> obj;
  std::vector<double> lq_fact;
  std::vector<double> itref_pred;
  std::vector<double> itref_corr;
  std::vector<double> lin_res_stat;
  std::vector<double> lin_res_eq;
  std::vector<double> lin_res_ineq;
  std::vector<double> lin_res_comp;

  void resize(const size_t size);
  void reserve(const size_t size);
  void clear();
  void disp(std::ostream& os) const;
};

std::ostream& operator<<(std::ostream& os, const OcpQpIpmSolverStatistics& stats);

}  // namespace hpipm
