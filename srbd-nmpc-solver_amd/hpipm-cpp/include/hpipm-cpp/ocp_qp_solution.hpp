// hpipm::OcpQpSolution (hpipm-cpp/include/hpipm-cpp/ocp_qp_solution.hpp:9-48):
// primal/dual trajectory and the Riccati quantities of one stage,
// pi[k] = P[k] x[k] + p[k],  u[k] = K[k] x[k] + k[k].
#pragma once

#include "hpipm-cpp/linalg.hpp"

namespace hpipm {

struct OcpQpSolution {
  VectorXd x;
  VectorXd u;
  VectorXd pi;
  MatrixXd P;
  VectorXd p;
  MatrixXd K;
  VectorXd k;
};

}  // namespace hpipm
