// linalg.hpp -- the matrix/vector types of the hpipm-cpp interface.
//
// With Eigen on the include path (the reference's NMPC build) OcpQp and
// OcpQpSolution hold Eigen::MatrixXd / Eigen::VectorXd exactly like
// hpipm-cpp/include/hpipm-cpp/ocp_qp.hpp:8-9, so existing callers compile
// unchanged.  Without Eigen (this image) the column-major dense types of
// dense.hpp stand in; define HPIPM_CPP_NO_EIGEN to force them.
#pragma once

#if !defined(HPIPM_CPP_NO_EIGEN) && __has_include(<Eigen/Core>)
#include <Eigen/Core>
namespace hpipm {
using MatrixXd = Eigen::MatrixXd;
using VectorXd = Eigen::VectorXd;
}  // namespace hpipm
#define HPIPM_CPP_HAS_EIGEN 1
#else
#include "hpipm-cpp/dense.hpp"
namespace hpipm {
using MatrixXd = dense::Matrix;
using VectorXd = dense::Vector;
}  // namespace hpipm
#define HPIPM_CPP_HAS_EIGEN 0
#endif
