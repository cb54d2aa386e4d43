// Minimal test harness + dense helpers for the hpipm-cpp interface tests
// (the image has neither gtest nor Eigen).  TEST(name, needs_gpu) registers a
// case; main() runs the cases selected on the command line:
//   hpipm_cpp_test [--cpu-only] [--golden DIR] [name ...]
#pragma once

#include <cmath>
#include <cstdio>
#include <functional>
#include <iostream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "hpipm-cpp/hpipm-cpp.hpp"

namespace test {

struct Case {
  const char* name;
  bool gpu;
  std::function<void()> fn;
};

inline std::vector<Case>& registry() {
  static std::vector<Case> r;
  return r;
}

struct Registrar {
  Registrar(const char* n, bool gpu, std::function<void()> f) {
    registry().push_back({n, gpu, std::move(f)});
  }
};

inline int& failures() {
  static int f = 0;
  return f;
}

inline std::string& golden_dir() {
  static std::string d = "tests/golden";
  return d;
}

#define TEST(NAME, GPU)                                             \
  static void test_##NAME();                                        \
  static ::test::Registrar reg_##NAME(#NAME, GPU, &test_##NAME);    \
  static void test_##NAME()

#define EXPECT_TRUE(c)                                                             \
  do {                                                                             \
    if (!(c)) {                                                                    \
      ++::test::failures();                                                        \
      std::fprintf(stderr, "  FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);        \
    }                                                                              \
  } while (0)

#define EXPECT_EQ(a, b) EXPECT_TRUE((a) == (b))

#define EXPECT_THROW_MSG(stmt, msg)                                                      \
  do {                                                                                   \
    bool thrown_ = false;                                                                \
    try {                                                                                \
      stmt;                                                                              \
    } catch (const std::exception& e_) {                                                 \
      thrown_ = true;                                                                    \
      if (std::string(e_.what()).find(msg) == std::string::npos) {                       \
        ++::test::failures();                                                            \
        std::fprintf(stderr, "  FAILED %s:%d: message '%s' lacks '%s'\n", __FILE__,      \
                     __LINE__, e_.what(), msg);                                          \
      }                                                                                  \
    }                                                                                    \
    if (!thrown_) {                                                                      \
      ++::test::failures();                                                              \
      std::fprintf(stderr, "  FAILED %s:%d: %s did not throw\n", __FILE__, __LINE__, #stmt); \
    }                                                                                    \
  } while (0)

using hpipm::MatrixXd;
using hpipm::VectorXd;

inline std::mt19937& rng() {
  static std::mt19937 g(20240611u);
  return g;
}

// uniform in [-1, 1] like Eigen::MatrixXd::Random
inline MatrixXd Random(long r, long c) {
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  MatrixXd m(r, c);
  for (long j = 0; j < c; ++j)
    for (long i = 0; i < r; ++i) m(i, j) = u(rng());
  return m;
}
inline VectorXd RandomVec(long n) { return VectorXd(Random(n, 1)); }
inline VectorXd AbsRandomVec(long n) {
  VectorXd v = RandomVec(n);
  for (long i = 0; i < n; ++i) v(i) = std::fabs(v(i));
  return v;
}

inline MatrixXd block(const MatrixXd& m, long r0, long c0, long nr, long nc) {
  MatrixXd b(nr, nc);
  for (long j = 0; j < nc; ++j)
    for (long i = 0; i < nr; ++i) b(i, j) = m(r0 + i, c0 + j);
  return b;
}

// Gauss-Jordan with partial pivoting (test-side only)
inline MatrixXd inverse(const MatrixXd& a) {
  const long n = a.rows();
  MatrixXd m = a, inv = MatrixXd::Identity(n, n);
  for (long c = 0; c < n; ++c) {
    long piv = c;
    for (long r = c + 1; r < n; ++r)
      if (std::fabs(m(r, c)) > std::fabs(m(piv, c))) piv = r;
    if (m(piv, c) == 0.0) throw std::runtime_error("singular matrix");
    for (long j = 0; j < n; ++j) {
      std::swap(m(c, j), m(piv, j));
      std::swap(inv(c, j), inv(piv, j));
    }
    const double d = 1.0 / m(c, c);
    for (long j = 0; j < n; ++j) {
      m(c, j) *= d;
      inv(c, j) *= d;
    }
    for (long r = 0; r < n; ++r) {
      if (r == c) continue;
      const double f = m(r, c);
      if (f == 0.0) continue;
      for (long j = 0; j < n; ++j) {
        m(r, j) -= f * m(c, j);
        inv(r, j) -= f * inv(c, j);
      }
    }
  }
  return inv;
}

inline bool approx(const MatrixXd& a, const MatrixXd& b, double prec) { return a.isApprox(b, prec); }

}  // namespace test
