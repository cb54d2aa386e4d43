// OcpQpIpmSolverStatistics (hpipm-cpp/src/ocp_qp_ipm_solver_statistics.cpp):
// container helpers and the same disp() table.
#include "hpipm-cpp/ocp_qp_ipm_solver_statistics.hpp"

#include <iomanip>

namespace hpipm {

namespace {
template <class F>
void each_column(OcpQpIpmSolverStatistics& s, F&& f) {
  for (std::vector<double>* v :
       {&s.alpha_aff, &s.mu_aff, &s.sigma, &s.alpha_prim, &s.alpha_dual, &s.mu, &s.res_stat,
        &s.res_eq, &s.res_ineq, &s.res_comp, &s.obj, &s.lq_fact, &s.itref_pred, &s.itref_corr,
        &s.lin_res_stat, &s.lin_res_eq, &s.lin_res_ineq, &s.lin_res_comp})
    f(*v);
}
}  // namespace

void OcpQpIpmSolverStatistics::resize(const size_t size) {
  each_column(*this, [size](std::vector<double>& v) { v.resize(size); });
}

void OcpQpIpmSolverStatistics::reserve(const size_t size) {
  each_column(*this, [size](std::vector<double>& v) { v.reserve(size); });
}

void OcpQpIpmSolverStatistics::clear() {
  each_column(*this, [](std::vector<double>& v) { v.clear(); });
}

void OcpQpIpmSolverStatistics::disp(std::ostream& os) const {
  os << "================== Hpipm Solver Statistics ==================" << std::endl;
  os << "ipm iter: " << iter << std::endl;
  os << std::setprecision(5) << std::scientific;
  os << "max_res_stat: " << max_res_stat << std::endl;
  os << "max_res_eq:   " << max_res_eq << std::endl;
  os << "max_res_ineq: " << max_res_ineq << std::endl;
  os << "max_res_comp: " << max_res_comp << std::endl;
  static const char* const kHeads[] = {
      "alpha_aff", "mu_aff", "sigma", "alpha_prim", "alpha_dual", "mu",
      "res_stat", "res_eq", "res_ineq", "res_comp", "obj", "lq fact",
      "itref pred", "itref corr", "lin res stat", "lin res eq", "lin res ineq", "lin res comp"};
  for (const char* h : kHeads) os << std::left << std::setw(13) << h;
  os << std::right << std::endl;
  if (iter <= 0) return;
  const std::vector<double>* cols[] = {
      &alpha_aff, &mu_aff, &sigma, &alpha_prim, &alpha_dual, &mu, &res_stat, &res_eq, &res_ineq,
      &res_comp, &obj, &lq_fact, &itref_pred, &itref_corr, &lin_res_stat, &lin_res_eq,
      &lin_res_ineq, &lin_res_comp};
  for (int i = 0; i <= iter; ++i) {
    for (const std::vector<double>* c : cols)
      os << (static_cast<size_t>(i) < c->size() ? (*c)[i] : 0.0) << "  ";
    os << std::endl;
  }
}

std::ostream& operator<<(std::ostream& os, const OcpQpIpmSolverStatistics& stats) {
  stats.disp(os);
  return os;
}

}  // namespace hpipm
