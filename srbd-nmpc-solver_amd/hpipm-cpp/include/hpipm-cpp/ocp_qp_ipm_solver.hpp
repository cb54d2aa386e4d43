// hpipm::OcpQpIpmSolver on MI355X
// (interface of hpipm-cpp/include/hpipm-cpp/ocp_qp_ipm_solver.hpp:19-147).
//
// Same names, argument meaning and error behaviour as the reference: solve()
// takes x0 and the N+1 stages, fills qp_sol[0..N] (x, u, pi, P, p, K, k) with
// x[0] == x0 and the stage-0 Riccati terms rebuilt, updates the statistics and
// returns the HPIPM status.  Underneath, every solve is one launch of the
// batched HIP kernels through the C-ABI in include/srbd_qp.h; there is no CPU
// solver behind this class (no GPU -> std::runtime_error).
//
// MI355X extension: solveBatch() hands B independent QPs of identical
// dimensions to one launch (one 16-lane group per QP), which is how the GPU
// earns its throughput; solve() is solveBatch() with B = 1.
//
// Restrictions of this build (each reported as std::runtime_error):
//   * nx, nu uniform over the stages (nu[N] = 0), 1 <= nx, nu <= 12, N <= 1024;
//   * general constraints: ng <= 64 per stage (fewer rows are padded with
//     masked rows);
//   * soft constraints (idxs / Zl / Zu / zl / zu / lls / lus) unsupported.
// Like the reference (ocp_qp_ipm_solver.cpp:128-130) the stage-0 state is
// eliminated: idxbx / lbx / ubx and C of stage 0 are accepted and ignored.
#pragma once

#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "hpipm-cpp/linalg.hpp"
#include "hpipm-cpp/ocp_qp.hpp"
#include "hpipm-cpp/ocp_qp_dim.hpp"
#include "hpipm-cpp/ocp_qp_ipm_solver_settings.hpp"
#include "hpipm-cpp/ocp_qp_ipm_solver_statistics.hpp"
#include "hpipm-cpp/ocp_qp_solution.hpp"

namespace hpipm {

enum class HpipmStatus {
  Success = 0,
  MaxIterReached = 1,
  MinStepLengthReached = 2,
  NaNDetected = 3,
  UnknownFailure = 4,
};

std::string to_string(const HpipmStatus& hpipm_status);
std::ostream& operator<<(std::ostream& os, const HpipmStatus& hpipm_status);

class OcpQpIpmSolver {
 public:
  OcpQpIpmSolver(const std::vector<OcpQp>& ocp_qp,
                 const OcpQpIpmSolverSettings& solver_settings = OcpQpIpmSolverSettings());
  OcpQpIpmSolver(const OcpQpIpmSolverSettings& solver_settings = OcpQpIpmSolverSettings());
  ~OcpQpIpmSolver();

  OcpQpIpmSolver(const OcpQpIpmSolver&) = delete;
  OcpQpIpmSolver& operator=(const OcpQpIpmSolver&) = delete;
  OcpQpIpmSolver(OcpQpIpmSolver&&) noexcept;
  OcpQpIpmSolver& operator=(OcpQpIpmSolver&&) noexcept;

  // store, unchecked like the reference (ocp_qp_ipm_solver.cpp:83-117); solve() checks
  void setSolverSettings(const OcpQpIpmSolverSettings& solver_settings);

  // dimension check + device workspace for these dimensions (:120-178)
  void resize(const std::vector<OcpQp>& ocp_qp);

  // one QP (:181-414)
  HpipmStatus solve(const VectorXd& x0, std::vector<OcpQp>& ocp_qp,
                    std::vector<OcpQpSolution>& qp_sol);

  // B independent QPs with identical dimensions, one kernel launch.
  // qp_sol is resized to B x (N+1); statistics per QP via getBatchStatistics().
  std::vector<HpipmStatus> solveBatch(const std::vector<VectorXd>& x0,
                                      std::vector<std::vector<OcpQp>>& ocp_qp,
                                      std::vector<std::vector<OcpQpSolution>>& qp_sol);

  const OcpQpIpmSolverSettings& getIpmSolverSettings() const;
  // statistics of the last solve() (of QP 0 after solveBatch())
  const OcpQpIpmSolverStatistics& getSolverStatistics() const;
  const std::vector<OcpQpIpmSolverStatistics>& getBatchStatistics() const;

  // HIP device the solver runs on (default 0); takes effect at the next resize
  void setDevice(int device);
  int device() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace hpipm
