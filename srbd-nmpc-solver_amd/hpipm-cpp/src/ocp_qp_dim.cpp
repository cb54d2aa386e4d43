// OcpQpDim: dimensions of a std::vector<OcpQp> and the size checks of
// hpipm-cpp/src/ocp_qp_dim.cpp:9-238 (same rules, same message form
// "ocp_qp[i].<field> must be <n>").
#include "hpipm-cpp/ocp_qp_dim.hpp"

#include <stdexcept>
#include <string>

namespace hpipm {

namespace {

[[noreturn]] void size_error(unsigned int stage, const char* what, const std::string& expect) {
  throw std::runtime_error("ocp_qp[" + std::to_string(stage) + "]." + what + " must be " + expect);
}

// exact size n
void need(long long got, int n, unsigned int stage, const char* what) {
  if (got != n) size_error(stage, what, std::to_string(n));
}

// empty mask or exactly n entries
void need_mask(long long got, int n, unsigned int stage, const char* what) {
  if (got != 0 && got != n) size_error(stage, what, "0 or " + std::to_string(n));
}

}  // namespace

OcpQpDim::OcpQpDim(const unsigned int N_) { resize(N_); }

OcpQpDim::OcpQpDim(const std::vector<OcpQp>& ocp_qp) { resize(ocp_qp); }

void OcpQpDim::resize(const unsigned int N_) {
  N = N_;
  for (std::vector<int>* v : {&nx, &nu, &nbx, &nbu, &ng, &nsbx, &nsbu, &nsg}) v->assign(N + 1, 0);
}

void OcpQpDim::resize(const std::vector<OcpQp>& ocp_qp) {
  if (ocp_qp.empty()) throw std::runtime_error("ocp_qp.size() must not be empty");
  resize(static_cast<unsigned int>(ocp_qp.size() - 1));
  for (unsigned int i = 0; i <= N; ++i) {
    const OcpQp& s = ocp_qp[i];
    nx[i] = static_cast<int>(s.q.size());
    nu[i] = i < N ? static_cast<int>(s.r.size()) : 0;
    nbx[i] = static_cast<int>(s.idxbx.size());
    nbu[i] = i < N ? static_cast<int>(s.idxbu.size()) : 0;
    ng[i] = static_cast<int>(s.lg.size());
    nsbx[i] = static_cast<int>(s.idxs.size());
    nsbu[i] = 0;
    nsg[i] = 0;
  }
  checkSize(ocp_qp);
}

void OcpQpDim::checkSize(const std::vector<OcpQp>& ocp_qp) const {
  if (ocp_qp.size() != N + 1)
    throw std::runtime_error("ocp_qp.size() must be " + std::to_string(N + 1));
  for (unsigned int i = 0; i <= N; ++i) {
    const OcpQp& s = ocp_qp[i];
    const bool last = i == N;
    // dynamics x+ = A x + B u + b
    if (!last) {
      need(s.A.rows(), nx[i + 1], i, "A.rows()");
      need(s.A.cols(), nx[i], i, "A.cols()");
      need(s.B.rows(), nx[i + 1], i, "B.rows()");
      need(s.B.cols(), nu[i], i, "B.cols()");
      need(s.b.size(), nx[i + 1], i, "b.size()");
    }
    // cost
    need(s.Q.rows(), nx[i], i, "Q.rows()");
    need(s.Q.cols(), nx[i], i, "Q.cols()");
    need(s.q.size(), nx[i], i, "q.size()");
    if (!last) {
      need(s.S.rows(), nu[i], i, "S.rows()");
      need(s.S.cols(), nx[i], i, "S.cols()");
      need(s.R.rows(), nu[i], i, "R.rows()");
      need(s.R.cols(), nu[i], i, "R.cols()");
      need(s.r.size(), nu[i], i, "r.size()");
    }
    // box constraints on x
    need(static_cast<long long>(s.idxbx.size()), nbx[i], i, "idxbx.size()");
    need(s.lbx.size(), nbx[i], i, "lbx.size()");
    need(s.ubx.size(), nbx[i], i, "ubx.size()");
    need_mask(s.lbx_mask.size(), nbx[i], i, "lbx_mask.size()");
    need_mask(s.ubx_mask.size(), nbx[i], i, "ubx_mask.size()");
    // box constraints on u
    if (!last) {
      need(static_cast<long long>(s.idxbu.size()), nbu[i], i, "idxbu.size()");
      need(s.lbu.size(), nbu[i], i, "lbu.size()");
      need(s.ubu.size(), nbu[i], i, "ubu.size()");
      need_mask(s.lbu_mask.size(), nbu[i], i, "lbu_mask.size()");
      need_mask(s.ubu_mask.size(), nbu[i], i, "ubu_mask.size()");
    }
    // general constraints lg <= C x + D u <= ug
    need(s.C.rows(), ng[i], i, "C.rows()");
    if (ng[i] > 0) need(s.C.cols(), nx[i], i, "C.cols()");
    if (!last) {
      need(s.D.rows(), ng[i], i, "D.rows()");
      if (ng[i] > 0) need(s.D.cols(), nu[i], i, "D.cols()");
    }
    need(s.lg.size(), ng[i], i, "lg.size()");
    need(s.ug.size(), ng[i], i, "ug.size()");
    need_mask(s.lg_mask.size(), ng[i], i, "lg_mask.size()");
    need_mask(s.ug_mask.size(), ng[i], i, "ug_mask.size()");
    // soft constraints (nsg == 0 in the reference's dims)
    if (!last) {
      need(s.Zl.rows(), nsg[i], i, "Zl.rows()");
      need(s.Zl.cols(), nsg[i], i, "Zl.cols()");
      need(s.Zu.rows(), nsg[i], i, "Zu.rows()");
      need(s.Zu.cols(), nsg[i], i, "Zu.cols()");
      need(s.zl.size(), nsg[i], i, "zl.size()");
      need(s.zu.size(), nsg[i], i, "zu.size()");
      need(static_cast<long long>(s.idxs.size()), nsg[i], i, "idxs.size()");
      need(s.lls.size(), nsg[i], i, "lls.size()");
      need(s.lus.size(), nsg[i], i, "lus.size()");
    }
  }
}

}  // namespace hpipm
