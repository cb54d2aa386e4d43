// hpipm::OcpQp -- one stage of an optimal-control QP, field for field the
// reference's struct (hpipm-cpp/include/hpipm-cpp/ocp_qp.hpp:15-177).
//
//   min  1/2 x'Q x + u'S x + 1/2 u'R u + q'x + r'u
//   s.t. x+ = A x + B u + b,  lbx <= x[idxbx] <= ubx,  lbu <= u[idxbu] <= ubu,
//        lg <= C x + D u <= ug   (optional 0/1 masks per bound).
// Soft constraints (Zl, Zu, zl, zu, idxs, lls, lus) are part of the struct for
// source compatibility; the GPU solver rejects them (see ocp_qp_ipm_solver.hpp).
#pragma once

#include <vector>

#include "hpipm-cpp/linalg.hpp"

namespace hpipm {

struct OcpQp {
  // dynamics
  MatrixXd A;
  MatrixXd B;
  VectorXd b;
  // cost
  MatrixXd Q;
  MatrixXd S;
  MatrixXd R;
  VectorXd q;
  VectorXd r;
  // box constraints on x
  std::vector<int> idxbx;
  VectorXd lbx;
  VectorXd ubx;
  VectorXd lbx_mask;
  VectorXd ubx_mask;
  // box constraints on u
  std::vector<int> idxbu;
  VectorXd lbu;
  VectorXd ubu;
  VectorXd lbu_mask;
  VectorXd ubu_mask;
  // general constraints
  MatrixXd C;
  MatrixXd D;
  VectorXd lg;
  VectorXd ug;
  VectorXd lg_mask;
  VectorXd ug_mask;
  // soft constraints
  MatrixXd Zl;
  MatrixXd Zu;
  VectorXd zl;
  VectorXd zu;
  std::vector<int> idxs;
  VectorXd lls;
  VectorXd lus;
};

}  // namespace hpipm
