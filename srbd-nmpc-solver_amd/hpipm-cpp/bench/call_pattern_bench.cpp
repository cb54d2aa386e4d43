// The reference caller's solve pattern, timed through the hpipm-cpp interface:
// NMPCSolver::solveQpProblems (NMPC_solver.cpp:316-330) constructs a fresh
// OcpQpIpmSolver for every SQP iteration, solves ONE QP from host (Eigen-layout)
// buffers and destroys the solver; controlLoop does that up to sqp_max_loop = 15
// times per NMPC step (NMPC_solver.cpp:362-372).
//
//   call_pattern_bench QP_FILE [reps]
//
// QP_FILE: raw little-endian doubles, nx = nu = 12: N, then per stage k < N
// A, B, b, Q, S, R, q, r (column-major blocks), then Q_N, q_N, then x0.
// Prints one JSON line: per-solve wall times (us) of
//   "construct_solve_destruct": the reference pattern, 15 per NMPC step;
//   "persistent_solver":        one solver reused for every solve.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "hpipm-cpp/hpipm-cpp.hpp"

namespace {

using Clock = std::chrono::steady_clock;

struct Reader {
  std::vector<double> v;
  size_t pos = 0;
  double next() {
    if (pos >= v.size()) throw std::runtime_error("QP file too short");
    return v[pos++];
  }
  void fill(hpipm::MatrixXd& m, int r, int c) {
    m.resize(r, c);
    for (int i = 0; i < r * c; ++i) m.data()[i] = next();
  }
  void fill(hpipm::VectorXd& x, int n) {
    x.resize(n);
    for (int i = 0; i < n; ++i) x.data()[i] = next();
  }
};

double median(std::vector<double> t) {
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s QP_FILE [reps]\n", argv[0]);
    return 2;
  }
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  const int sqp_max_loop = 15;  // config/mpc_option.yaml
  Reader rd;
  {
    std::ifstream f(argv[1], std::ios::binary);
    if (!f) throw std::runtime_error(std::string("cannot open ") + argv[1]);
    f.seekg(0, std::ios::end);
    rd.v.resize(static_cast<size_t>(f.tellg()) / sizeof(double));
    f.seekg(0);
    f.read(reinterpret_cast<char*>(rd.v.data()), static_cast<std::streamsize>(rd.v.size() * sizeof(double)));
  }
  const int N = static_cast<int>(rd.next()), nx = 12, nu = 12;
  std::vector<hpipm::OcpQp> qp(N + 1);
  for (int k = 0; k < N; ++k) {
    rd.fill(qp[k].A, nx, nx);
    rd.fill(qp[k].B, nx, nu);
    rd.fill(qp[k].b, nx);
    rd.fill(qp[k].Q, nx, nx);
    rd.fill(qp[k].S, nu, nx);
    rd.fill(qp[k].R, nu, nu);
    rd.fill(qp[k].q, nx);
    rd.fill(qp[k].r, nu);
  }
  rd.fill(qp[N].Q, nx, nx);
  rd.fill(qp[N].q, nx);
  hpipm::VectorXd x0;
  rd.fill(x0, nx);

  // NMPC_solver.cpp:70-82
  hpipm::OcpQpIpmSolverSettings st;
  st.mode = hpipm::HpipmMode::Speed;
  st.iter_max = 30;
  st.alpha_min = 1e-8;
  st.mu0 = 1e2;
  st.tol_stat = st.tol_eq = st.tol_ineq = st.tol_comp = 1e-4;
  st.reg_prim = 1e-12;
  st.warm_start = 0;
  st.pred_corr = 1;
  st.ric_alg = 0;
  st.split_step = 1;

  std::vector<hpipm::OcpQpSolution> sol(N + 1);
  int bad = 0;
  // warm-up: first solver of this shape (handle, staging and pinned buffers created)
  {
    hpipm::OcpQpIpmSolver s(qp, st);
    bad += s.solve(x0, qp, sol) != hpipm::HpipmStatus::Success;
  }
  std::vector<double> t_ref, t_step, t_pers;
  for (int r = 0; r < reps; ++r) {
    const auto s0 = Clock::now();
    for (int i = 0; i < sqp_max_loop; ++i) {
      const auto t0 = Clock::now();
      hpipm::OcpQpIpmSolver solver(qp, st);  // NMPC_solver.cpp:319
      bad += solver.solve(x0, qp, sol) != hpipm::HpipmStatus::Success;
      t_ref.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    t_step.push_back(std::chrono::duration<double, std::micro>(Clock::now() - s0).count());
  }
  {
    hpipm::OcpQpIpmSolver solver(qp, st);
    for (int r = 0; r < reps * sqp_max_loop; ++r) {
      const auto t0 = Clock::now();
      bad += solver.solve(x0, qp, sol) != hpipm::HpipmStatus::Success;
      t_pers.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
  }
  std::printf(
      "{\"N\": %d, \"solves\": %zu, \"construct_solve_destruct_us\": {\"median\": %.2f, \"min\": %.2f}, "
      "\"nmpc_step_15_solves_us\": {\"median\": %.2f, \"min\": %.2f}, "
      "\"persistent_solver_us\": {\"median\": %.2f, \"min\": %.2f}, \"failed\": %d, \"u0\": [%.17g, %.17g]}\n",
      N, t_ref.size(), median(t_ref), *std::min_element(t_ref.begin(), t_ref.end()), median(t_step),
      *std::min_element(t_step.begin(), t_step.end()), median(t_pers),
      *std::min_element(t_pers.begin(), t_pers.end()), bad, sol[0].u.data()[0], sol[0].u.data()[1]);
  return bad ? 1 : 0;
}
