// dense.hpp -- minimal column-major dense matrix/vector used by the hpipm-cpp
// interface when Eigen is not available (this image ships no Eigen).
//
// Only what the OcpQp / OcpQpSolution marshalling needs (rows/cols/size,
// contiguous column-major data(), resize, element access) plus a handful of
// arithmetic helpers for host-side glue code and tests.  Storage order and
// data() semantics match Eigen::MatrixXd / Eigen::VectorXd, so the solver
// source compiles unchanged against either (see linalg.hpp).
#pragma once

#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstddef>
#include <initializer_list>
#include <stdexcept>
#include <vector>

namespace hpipm {
namespace dense {

using Index = std::ptrdiff_t;

class Matrix {
 public:
  Matrix() = default;
  Matrix(Index rows, Index cols) { resize(rows, cols); }

  Index rows() const { return rows_; }
  Index cols() const { return cols_; }
  Index size() const { return rows_ * cols_; }
  double* data() { return v_.empty() ? nullptr : v_.data(); }
  const double* data() const { return v_.empty() ? nullptr : v_.data(); }

  void resize(Index rows, Index cols) {
    if (rows < 0 || cols < 0) throw std::invalid_argument("negative matrix size");
    rows_ = rows;
    cols_ = cols;
    v_.assign(static_cast<size_t>(rows * cols), 0.0);
  }

  double& operator()(Index i, Index j) { return v_[static_cast<size_t>(j * rows_ + i)]; }
  double operator()(Index i, Index j) const { return v_[static_cast<size_t>(j * rows_ + i)]; }

  Matrix& setZero() { return setConstant(0.0); }
  Matrix& setConstant(double c) {
    std::fill(v_.begin(), v_.end(), c);
    return *this;
  }
  Matrix& setIdentity() {
    setZero();
    for (Index i = 0; i < std::min(rows_, cols_); ++i) (*this)(i, i) = 1.0;
    return *this;
  }

  static Matrix Zero(Index r, Index c) { return Matrix(r, c); }
  static Matrix Constant(Index r, Index c, double v) { return Matrix(r, c).setConstant(v); }
  static Matrix Identity(Index r, Index c) { return Matrix(r, c).setIdentity(); }

  Matrix transpose() const {
    Matrix t(cols_, rows_);
    for (Index j = 0; j < cols_; ++j)
      for (Index i = 0; i < rows_; ++i) t(j, i) = (*this)(i, j);
    return t;
  }

  double squaredNorm() const {
    double s = 0.0;
    for (double x : v_) s += x * x;
    return s;
  }
  double norm() const { return std::sqrt(squaredNorm()); }
  double maxAbs() const {
    double m = 0.0;
    for (double x : v_) m = std::max(m, std::fabs(x));
    return m;
  }

  // Eigen's isApprox: ||a - b|| <= prec * min(||a||, ||b||)
  bool isApprox(const Matrix& o, double prec = 1e-12) const {
    if (rows_ != o.rows_ || cols_ != o.cols_) return false;
    double d = 0.0;
    for (size_t i = 0; i < v_.size(); ++i) d += (v_[i] - o.v_[i]) * (v_[i] - o.v_[i]);
    return std::sqrt(d) <= prec * std::min(norm(), o.norm());
  }

  Matrix& operator+=(const Matrix& o) {
    check_same(o);
    for (size_t i = 0; i < v_.size(); ++i) v_[i] += o.v_[i];
    return *this;
  }
  Matrix& operator-=(const Matrix& o) {
    check_same(o);
    for (size_t i = 0; i < v_.size(); ++i) v_[i] -= o.v_[i];
    return *this;
  }
  Matrix& operator*=(double s) {
    for (double& x : v_) x *= s;
    return *this;
  }

 protected:
  void check_same(const Matrix& o) const {
    if (rows_ != o.rows_ || cols_ != o.cols_) throw std::invalid_argument("matrix size mismatch");
  }
  Index rows_ = 0, cols_ = 0;
  std::vector<double> v_;
};

class Vector : public Matrix {
 public:
  Vector() : Matrix(0, 1) {}
  explicit Vector(Index n) : Matrix(n, 1) {}
  Vector(std::initializer_list<double> l) : Matrix(static_cast<Index>(l.size()), 1) {
    std::copy(l.begin(), l.end(), v_.begin());
  }
  // a single-column matrix converts implicitly, like Eigen expressions do
  Vector(const Matrix& m) : Matrix(m) {  // NOLINT
    if (m.cols() != 1 && m.size() != 0) throw std::invalid_argument("Vector from non-column matrix");
    rows_ = m.size();
    cols_ = 1;
  }

  void resize(Index n) { Matrix::resize(n, 1); }
  double& operator()(Index i) { return v_[static_cast<size_t>(i)]; }
  double operator()(Index i) const { return v_[static_cast<size_t>(i)]; }
  double& operator[](Index i) { return v_[static_cast<size_t>(i)]; }
  double operator[](Index i) const { return v_[static_cast<size_t>(i)]; }

  static Vector Zero(Index n) { return Vector(n); }
  static Vector Constant(Index n, double v) {
    Vector r(n);
    r.setConstant(v);
    return r;
  }
  double dot(const Vector& o) const {
    check_same(o);
    double s = 0.0;
    for (size_t i = 0; i < v_.size(); ++i) s += v_[i] * o.v_[i];
    return s;
  }
};

inline Matrix operator+(Matrix a, const Matrix& b) { return a += b; }
inline Matrix operator-(Matrix a, const Matrix& b) { return a -= b; }
inline Matrix operator-(Matrix a) { return a *= -1.0; }
inline Matrix operator*(double s, Matrix a) { return a *= s; }
inline Matrix operator*(Matrix a, double s) { return a *= s; }
inline Matrix operator*(const Matrix& a, const Matrix& b) {
  if (a.cols() != b.rows()) throw std::invalid_argument("matrix product size mismatch");
  Matrix c(a.rows(), b.cols());
  for (Index j = 0; j < b.cols(); ++j)
    for (Index k = 0; k < a.cols(); ++k) {
      const double bkj = b(k, j);
      for (Index i = 0; i < a.rows(); ++i) c(i, j) += a(i, k) * bkj;
    }
  return c;
}

}  // namespace dense
}  // namespace hpipm
