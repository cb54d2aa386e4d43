// hpipm::OcpQpDim (hpipm-cpp/include/hpipm-cpp/ocp_qp_dim.hpp:13-88):
// per-stage dimensions read off a std::vector<OcpQp>, with checkSize()
// throwing std::runtime_error messages of the same form as the reference's
// (src/ocp_qp_dim.cpp:48-238).
#pragma once

#include <vector>

#include "hpipm-cpp/ocp_qp.hpp"

namespace hpipm {

struct OcpQpDim {
 public:
  explicit OcpQpDim(const unsigned int N);
  explicit OcpQpDim(const std::vector<OcpQp>& ocp_qp);
  OcpQpDim() = default;

  unsigned int N = 0;
  std::vector<int> nx;
  std::vector<int> nu;
  std::vector<int> nbx;
  std::vector<int> nbu;
  std::vector<int> ng;
  std::vector<int> nsbx;
  std::vector<int> nsbu;
  std::vector<int> nsg;

  void resize(const unsigned int N);
  void resize(const std::vector<OcpQp>& ocp_qp);
  void checkSize(const std::vector<OcpQp>& ocp_qp) const;
};

}  // namespace hpipm
