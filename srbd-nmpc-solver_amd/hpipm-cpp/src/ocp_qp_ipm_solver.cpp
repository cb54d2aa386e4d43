// hpipm::OcpQpIpmSolver over the MI355X C-ABI (include/srbd_qp.h).
//
// The reference (hpipm-cpp/src/ocp_qp_ipm_solver.cpp:181-414) hands per-stage
// Eigen pointers to HPIPM, calls d_ocp_qp_ipm_solve, reads the solution and
// Riccati factors back and rebuilds stage 0 on the host.  Here the stages of
// every QP of the batch are packed into the C-ABI's batch/stage-major
// buffers, one srbd_qp_solve_host_f64 call runs the whole batch on the GPU
// (x0 elimination and the stage-0 rebuild happen inside the kernel), and the
// results are unpacked into OcpQpSolution / OcpQpIpmSolverStatistics.
#include "hpipm-cpp/ocp_qp_ipm_solver.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#include "srbd_qp.h"

namespace {
// SRBD_SHIM_PROFILE=1: host time of the staged one-QP path by piece (staging pointers, packing,
// the C-ABI solve, unpacking), summed over the process and printed to stderr at exit.
struct ShimProfile {
  bool on = std::getenv("SRBD_SHIM_PROFILE") != nullptr;
  double t[4] = {0, 0, 0, 0};
  long n = 0;
  ~ShimProfile() {
    if (on && n)
      std::fprintf(stderr, "{\"shim_profile_us\": {\"calls\": %ld, \"staging\": %.2f, \"pack\": %.2f, "
                           "\"solve_host\": %.2f, \"unpack\": %.2f}}\n",
                   n, t[0] / n, t[1] / n, t[2] / n, t[3] / n);
  }
};
ShimProfile g_prof;
using PClock = std::chrono::steady_clock;
inline double us_since(PClock::time_point t0) {
  return std::chrono::duration<double, std::micro>(PClock::now() - t0).count();
}
}  // namespace

namespace hpipm {

std::string to_string(const HpipmStatus& hpipm_status) {
  switch (hpipm_status) {
    case HpipmStatus::Success:
      return "HpipmStatus::Success";
    case HpipmStatus::MaxIterReached:
      return "HpipmStatus::MaxIterReached";
    case HpipmStatus::MinStepLengthReached:
      return "HpipmStatus::MinStepLengthReached";
    case HpipmStatus::NaNDetected:
      return "HpipmStatus::NaNDetected";
    default:
      return "HpipmStatus::UnknownFailure";
  }
}

std::ostream& operator<<(std::ostream& os, const HpipmStatus& hpipm_status) {
  return os << to_string(hpipm_status);
}

namespace {

[[noreturn]] void abi_error(const char* what) {
  throw std::runtime_error(std::string(what) + ": " + srbd_qp_last_error());
}

void copy_block(double* dst, size_t off, const double* src, size_t n) {
  if (n) std::memcpy(dst + off, src, n * sizeof(double));
}

// rows x cols column-major src (ld = rows) into dst at off with leading dimension ld
void copy_mat(double* dst, size_t off, size_t ld, const double* src, size_t rows, size_t cols) {
  if (rows == ld) {  // contiguous columns: one copy
    if (rows && cols) std::memcpy(dst + off, src, rows * cols * sizeof(double));
    return;
  }
  for (size_t c = 0; c < cols; ++c)
    if (rows) std::memcpy(dst + off + c * ld, src + c * rows, rows * sizeof(double));
}
void copy_mat(std::vector<double>& dst, size_t off, size_t ld, const double* src, size_t rows,
              size_t cols) {
  copy_mat(dst.data(), off, ld, src, rows, cols);
}
// the leading rows x cols block of a column-major ld x * src into dst (ld = rows)
void take_mat(double* dst, const double* src, size_t ld, size_t rows, size_t cols) {
  if (rows == ld) {  // the whole block: one copy (the one-QP call's unpack is bound by these
                     // reads of the pinned buffer the kernel wrote)
    if (rows && cols) std::memcpy(dst, src, rows * cols * sizeof(double));
    return;
  }
  for (size_t c = 0; c < cols; ++c)
    if (rows) std::memcpy(dst + c * rows, src + c * ld, rows * sizeof(double));
}

// Stage dimensions of the C-ABI problem: nx, nu are the largest over the stages.
// hpipm-cpp lets nx[i], nu[i] vary per stage (ocp_qp_dim.cpp:37-53); the C-ABI takes
// uniform dimensions, so a stage with fewer states or inputs is embedded in the uniform
// one (pack): its A, B rows / columns beyond its dimensions are zero, so those states stay
// 0 and cost nothing, and its extra inputs get R = 1 on the diagonal (u = 0 there) -- the
// same embedding pad.hip applies below 12 x 12.  The solution is cut back per stage
// (unpack).
struct Shape {
  int N = 0, nx = 0, nu = 0, ng = 0;
  bool box_u = false, box_x = false;
  bool operator==(const Shape& o) const {
    return N == o.N && nx == o.nx && nu == o.nu && ng == o.ng && box_u == o.box_u &&
           box_x == o.box_x;
  }
  bool operator!=(const Shape& o) const { return !(*this == o); }
};

Shape shape_of(const OcpQpDim& d) {
  Shape s;
  s.N = static_cast<int>(d.N);
  for (unsigned int i = 0; i <= d.N; ++i) {
    s.nx = std::max(s.nx, d.nx[i]);
    if (i < d.N) s.nu = std::max(s.nu, d.nu[i]);
    if (d.nsbx[i] != 0 || d.nsbu[i] != 0 || d.nsg[i] != 0)
      throw std::runtime_error("OcpQpIpmSolver: soft constraints are not supported");
    s.ng = std::max(s.ng, d.ng[i]);
    if (i < d.N && d.nbu[i] > 0) s.box_u = true;
    if (i > 0 && d.nbx[i] > 0) s.box_x = true;  // stage-0 x bounds: eliminated with x0
  }
  return s;
}

// Process-wide pool of C-ABI handles.  The reference's caller builds a new
// OcpQpIpmSolver for every SQP iteration (NMPC_solver.cpp:318-319); a handle owns a
// HIP stream and a device workspace, so creating one per solver would put a stream
// create, hipMallocs and a stream destroy around every single QP solve.  A solver
// takes a handle of its shape from the pool (or creates one) and gives it back when it
// is destroyed or resized; the next solver of the same shape reuses it.  A handle is
// used by one solver at a time, so concurrent solvers on different threads stay
// independent, as HPIPM instances with separate memory are.
class HandlePool {
 public:
  static HandlePool& get() {
    // never destroyed: handles still pooled at exit are reclaimed with the process
    // (freeing them from a static destructor would race the HIP runtime's teardown)
    static HandlePool* pool = new HandlePool();
    return *pool;
  }
  srbd_qp_handle acquire(int device, const Shape& s, int batch, int* capacity) {
    {
      std::lock_guard<std::mutex> lk(m_);
      size_t best = free_.size();
      for (size_t i = 0; i < free_.size(); ++i) {
        const Entry& e = free_[i];
        if (e.device == device && e.shape == s && e.capacity >= batch &&
            (best == free_.size() || e.capacity < free_[best].capacity))
          best = i;
      }
      if (best != free_.size()) {
        Entry e = free_[best];
        free_.erase(free_.begin() + static_cast<long>(best));
        parked_bytes_ -= e.bytes;
        *capacity = e.capacity;
        return e.h;
      }
    }
    srbd_qp_dims d{s.N, s.nx, s.nu, s.ng, s.box_u ? 1 : 0, s.box_x ? 1 : 0, SRBD_QP_LAYOUT_QP_MAJOR};
    srbd_qp_handle h = nullptr;
    if (srbd_qp_create(&d, batch, device, &h) != SRBD_QP_OK) abi_error("OcpQpIpmSolver::resize");
    *capacity = batch;
    return h;
  }
  void release(int device, const Shape& s, int capacity, srbd_qp_handle h) {
    if (!h) return;
    // big handles (batched solves) are freed, not parked; the count covers everything a
    // handle holds (workspace, staging, pinned mirror, padding / rescue buffers), and the
    // parked handles together stay under kMaxPooledBytes
    const size_t bytes = srbd_qp_memory_bytes(h);
    {
      std::lock_guard<std::mutex> lk(m_);
      if (free_.size() < kMaxPooled && parked_bytes_ + bytes <= kMaxPooledBytes) {
        free_.push_back(Entry{device, s, capacity, h, bytes});
        parked_bytes_ += bytes;
        return;
      }
    }
    srbd_qp_destroy(h);
  }

 private:
  struct Entry {
    int device;
    Shape shape;
    int capacity;
    srbd_qp_handle h;
    size_t bytes;  // srbd_qp_memory_bytes when parked
  };
  static constexpr size_t kMaxPooled = 16;
  static constexpr size_t kMaxPooledBytes = size_t(256) << 20;  // all parked handles together
  std::mutex m_;
  std::vector<Entry> free_;
  size_t parked_bytes_ = 0;
};

}  // namespace

struct OcpQpIpmSolver::Impl {
  OcpQpIpmSolverSettings settings;
  OcpQpIpmSolverStatistics stats;
  std::vector<OcpQpIpmSolverStatistics> batch_stats;
  OcpQpDim dim;
  int device = 0;
  srbd_qp_handle handle = nullptr;
  Shape shape;
  int capacity = 0;
  // host staging (batch/stage-major, column-major blocks)
  std::vector<double> A, B, b, Q, S, R, q, r, x0;
  std::vector<double> lbu, ubu, lbu_m, ubu_m, lbx, ubx, lbx_m, ubx_m;
  std::vector<double> C, D, lg, ug, lg_m, ug_m;
  std::vector<double> x, u, pi, P, p, K, k, res, obj, stat;
  std::vector<int> status, iter;

  ~Impl() { release(); }
  void release() {
    if (handle) HandlePool::get().release(device, shape, capacity, handle);
    handle = nullptr;
    capacity = 0;
  }

  void ensure_handle(const Shape& s, int batch) {
    if (handle && s == shape && batch <= capacity) return;
    release();
    handle = HandlePool::get().acquire(device, s, std::max(batch, 1), &capacity);
    shape = s;
  }

  srbd_qp_settings abi_settings() const {
    srbd_qp_settings s;
    srbd_qp_default_settings(&s);
    s.mode = static_cast<int>(settings.mode);
    s.iter_max = settings.iter_max;
    s.alpha_min = settings.alpha_min;
    s.mu0 = settings.mu0;
    s.tol_stat = settings.tol_stat;
    s.tol_eq = settings.tol_eq;
    s.tol_ineq = settings.tol_ineq;
    s.tol_comp = settings.tol_comp;
    s.reg_prim = settings.reg_prim;
    s.warm_start = settings.warm_start;
    s.pred_corr = settings.pred_corr;
    s.ric_alg = settings.ric_alg;
    s.split_step = settings.split_step;
    s.f32_iters = settings.f32_iters;
    return s;
  }

  // Where pack() writes the unconstrained fields and unpack() reads the outputs: the vectors
  // above, or the C-ABI's pinned staging buffer (srbd_qp_host_staging_f64), which the kernel
  // then reads and writes in place -- no staging copies on the reference's one-QP path.
  struct Bufs {
    double *A = nullptr, *B = nullptr, *b = nullptr, *Q = nullptr, *S = nullptr, *R = nullptr,
           *q = nullptr, *r = nullptr, *x0 = nullptr;
    double *x = nullptr, *u = nullptr, *pi = nullptr, *P = nullptr, *p = nullptr, *K = nullptr,
           *k = nullptr, *res = nullptr, *obj = nullptr, *stat = nullptr;
    int *status = nullptr, *iter = nullptr;
  };
  Bufs buf;  // bound by pack()

  void pack(const std::vector<VectorXd>& x0s, const std::vector<std::vector<OcpQp>>& qps,
            const std::vector<std::vector<OcpQpSolution>>* warm, const Bufs* staged = nullptr);
  // parts: kFactors (P, p, K, k), kRest (x, u, pi, statistics), or both
  static constexpr int kFactors = 1, kRest = 2;
  std::vector<HpipmStatus> unpack(std::vector<std::vector<OcpQpSolution>>& sols, int parts = kFactors | kRest);
};

void OcpQpIpmSolver::Impl::pack(const std::vector<VectorXd>& x0s,
                                const std::vector<std::vector<OcpQp>>& qps,
                                const std::vector<std::vector<OcpQpSolution>>* warm,
                                const Bufs* staged) {
  const size_t nb = qps.size(), N = shape.N, nx = shape.nx, nu = shape.nu, ng = shape.ng;
  auto sized = [](std::vector<double>& v, size_t n) { v.assign(n, 0.0); };
  // every stage at the uniform dims: each input element is written below, no zero fill needed
  bool uniform = true;
  for (unsigned int i = 0; i <= dim.N; ++i)
    uniform = uniform && static_cast<size_t>(dim.nx[i]) == nx && (i == dim.N || static_cast<size_t>(dim.nu[i]) == nu);
  if (staged) {
    buf = *staged;
    if (!uniform) {
      auto zero = [](double* p, size_t n) { std::memset(p, 0, n * sizeof(double)); };
      zero(buf.A, nb * N * nx * nx);
      zero(buf.B, nb * N * nx * nu);
      zero(buf.b, nb * N * nx);
      zero(buf.Q, nb * (N + 1) * nx * nx);
      zero(buf.S, nb * N * nu * nx);
      zero(buf.R, nb * N * nu * nu);
      zero(buf.q, nb * (N + 1) * nx);
      zero(buf.r, nb * N * nu);
      zero(buf.x0, nb * nx);
    }
  } else {
    sized(A, nb * N * nx * nx);
    sized(B, nb * N * nx * nu);
    sized(b, nb * N * nx);
    sized(Q, nb * (N + 1) * nx * nx);
    sized(S, nb * N * nu * nx);
    sized(R, nb * N * nu * nu);
    sized(q, nb * (N + 1) * nx);
    sized(r, nb * N * nu);
    sized(x0, nb * nx);
    buf = Bufs{};
    buf.A = A.data(); buf.B = B.data(); buf.b = b.data(); buf.Q = Q.data(); buf.S = S.data();
    buf.R = R.data(); buf.q = q.data(); buf.r = r.data(); buf.x0 = x0.data();
  }
  if (shape.box_u) {
    for (auto* v : {&lbu, &ubu, &lbu_m, &ubu_m}) sized(*v, nb * N * nu);
  }
  if (shape.box_x) {
    for (auto* v : {&lbx, &ubx, &lbx_m, &ubx_m}) sized(*v, nb * (N + 1) * nx);
  }
  if (ng) {
    sized(C, nb * (N + 1) * ng * nx);
    sized(D, nb * N * ng * nu);
    for (auto* v : {&lg, &ug, &lg_m, &ug_m}) sized(*v, nb * (N + 1) * ng);
  }
  const size_t nx0 = static_cast<size_t>(dim.nx[0]);
  for (size_t bi = 0; bi < nb; ++bi) {
    const std::vector<OcpQp>& qp = qps[bi];
    if (static_cast<size_t>(x0s[bi].size()) != nx0)
      throw std::runtime_error("x0.size() must be " + std::to_string(nx0));
    copy_block(buf.x0, bi * nx, x0s[bi].data(), nx0);
    for (size_t k = 0; k <= N; ++k) {
      const OcpQp& s = qp[k];
      const size_t sk = bi * (N + 1) + k;  // stage index, N+1 stages
      const size_t xk = static_cast<size_t>(dim.nx[k]);  // this stage's dimensions
      copy_mat(buf.Q, sk * nx * nx, nx, s.Q.data(), xk, xk);
      copy_block(buf.q, sk * nx, s.q.data(), xk);
      if (k < N) {
        const size_t si = bi * N + k;  // stage index, N stages
        const size_t uk = static_cast<size_t>(dim.nu[k]), xn = static_cast<size_t>(dim.nx[k + 1]);
        copy_mat(buf.A, si * nx * nx, nx, s.A.data(), xn, xk);
        copy_mat(buf.B, si * nx * nu, nx, s.B.data(), xn, uk);
        copy_block(buf.b, si * nx, s.b.data(), xn);
        copy_mat(buf.S, si * nu * nx, nu, s.S.data(), uk, xk);
        copy_mat(buf.R, si * nu * nu, nu, s.R.data(), uk, uk);
        for (size_t j = uk; j < nu; ++j) buf.R[si * nu * nu + j * nu + j] = 1.0;  // embedded inputs
        copy_block(buf.r, si * nu, s.r.data(), uk);
        if (shape.box_u) {
          // index form -> dense per-variable bounds + masks (include/srbd_qp.h)
          for (size_t j = 0; j < s.idxbu.size(); ++j) {
            const int v = s.idxbu[j];
            if (v < 0 || static_cast<size_t>(v) >= uk)
              throw std::runtime_error("ocp_qp[" + std::to_string(k) + "].idxbu[" +
                                       std::to_string(j) + "] out of range");
            const size_t o = si * nu + v;
            lbu[o] = s.lbu[j];
            ubu[o] = s.ubu[j];
            lbu_m[o] = s.lbu_mask.size() ? s.lbu_mask[j] : 1.0;
            ubu_m[o] = s.ubu_mask.size() ? s.ubu_mask[j] : 1.0;
          }
        }
        if (ng && s.D.size()) {
          // pad to ng rows: column-major ng x nu block, extra rows stay 0
          copy_mat(D, si * ng * nu, ng, s.D.data(), static_cast<size_t>(s.D.rows()), uk);
        }
      }
      if (shape.box_x && k > 0) {
        for (size_t j = 0; j < s.idxbx.size(); ++j) {
          const int v = s.idxbx[j];
          if (v < 0 || static_cast<size_t>(v) >= xk)
            throw std::runtime_error("ocp_qp[" + std::to_string(k) + "].idxbx[" +
                                     std::to_string(j) + "] out of range");
          const size_t o = sk * nx + v;
          lbx[o] = s.lbx[j];
          ubx[o] = s.ubx[j];
          lbx_m[o] = s.lbx_mask.size() ? s.lbx_mask[j] : 1.0;
          ubx_m[o] = s.ubx_mask.size() ? s.ubx_mask[j] : 1.0;
        }
      }
      if (ng) {
        const size_t rows = s.lg.size();
        if (rows && s.C.size()) copy_mat(C, sk * ng * nx, ng, s.C.data(), rows, xk);
        for (size_t rr = 0; rr < rows; ++rr) {
          const size_t o = sk * ng + rr;
          lg[o] = s.lg[rr];
          ug[o] = s.ug[rr];
          lg_m[o] = s.lg_mask.size() ? s.lg_mask[rr] : 1.0;
          ug_m[o] = s.ug_mask.size() ? s.ug_mask[rr] : 1.0;
        }
      }
    }
  }
  // outputs (x/u double as the warm start when settings.warm_start); the staged ones are
  // written whole by the solve
  if (!staged) {
    sized(x, nb * (N + 1) * nx);
    sized(u, nb * N * nu);
    sized(pi, nb * (N + 1) * nx);
    sized(P, nb * (N + 1) * nx * nx);
    sized(p, nb * (N + 1) * nx);
    sized(K, nb * N * nu * nx);
    sized(k, nb * N * nu);
    sized(res, nb * 4);
    sized(obj, nb);
    sized(stat, nb * (settings.iter_max + 2) * 18);
    status.assign(nb, -1);
    iter.assign(nb, 0);
    buf.x = x.data(); buf.u = u.data(); buf.pi = pi.data(); buf.P = P.data(); buf.p = p.data();
    buf.K = K.data(); buf.k = k.data(); buf.res = res.data(); buf.obj = obj.data();
    buf.stat = stat.data(); buf.status = status.data(); buf.iter = iter.data();
  }
  if (warm) {
    if (staged && !uniform) {
      std::memset(buf.x, 0, nb * (N + 1) * nx * sizeof(double));
      std::memset(buf.u, 0, nb * N * nu * sizeof(double));
    }
    for (size_t bi = 0; bi < nb; ++bi) {
      const std::vector<OcpQpSolution>& w = (*warm)[bi];
      for (size_t kk = 0; kk < N; ++kk) {
        copy_block(buf.x, (bi * (N + 1) + kk + 1) * nx, w[kk + 1].x.data(), static_cast<size_t>(dim.nx[kk + 1]));
        copy_block(buf.u, (bi * N + kk) * nu, w[kk].u.data(), static_cast<size_t>(dim.nu[kk]));
      }
    }
  }
}

std::vector<HpipmStatus> OcpQpIpmSolver::Impl::unpack(
    std::vector<std::vector<OcpQpSolution>>& sols, int parts) {
  const size_t nb = sols.size(), N = shape.N, nx = shape.nx, nu = shape.nu;
  const size_t rows = static_cast<size_t>(settings.iter_max) + 2;
  std::vector<HpipmStatus> out;
  if (parts & kFactors) {
    for (size_t bi = 0; bi < nb; ++bi) {
      std::vector<OcpQpSolution>& sol = sols[bi];
      for (size_t kk = 0; kk <= N; ++kk) {
        OcpQpSolution& s = sol[kk];
        const size_t sk = bi * (N + 1) + kk;
        const size_t xk = static_cast<size_t>(dim.nx[kk]);  // the stage's own dimensions
        s.P.resize(xk, xk);
        s.p.resize(xk);
        take_mat(s.P.data(), buf.P + sk * nx * nx, nx, xk, xk);
        std::memcpy(s.p.data(), buf.p + sk * nx, xk * sizeof(double));
        if (kk < N) {
          const size_t si = bi * N + kk, uk = static_cast<size_t>(dim.nu[kk]);
          s.K.resize(uk, xk);
          s.k.resize(uk);
          take_mat(s.K.data(), buf.K + si * nu * nx, nu, uk, xk);
          std::memcpy(s.k.data(), buf.k + si * nu, uk * sizeof(double));
        } else {
          s.k.resize(0);  // nu[N] = 0 (ocp_qp_ipm_solver.cpp:221-223)
        }
      }
    }
  }
  if (!(parts & kRest)) return out;
  out.resize(nb);
  batch_stats.resize(nb);
  for (size_t bi = 0; bi < nb; ++bi) {
    std::vector<OcpQpSolution>& sol = sols[bi];
    for (size_t kk = 0; kk <= N; ++kk) {
      OcpQpSolution& s = sol[kk];
      const size_t sk = bi * (N + 1) + kk;
      const size_t xk = static_cast<size_t>(dim.nx[kk]);
      s.x.resize(xk);
      s.pi.resize(xk);
      std::memcpy(s.x.data(), buf.x + sk * nx, xk * sizeof(double));
      std::memcpy(s.pi.data(), buf.pi + sk * nx, xk * sizeof(double));
      if (kk < N) {
        const size_t si = bi * N + kk, uk = static_cast<size_t>(dim.nu[kk]);
        s.u.resize(uk);
        std::memcpy(s.u.data(), buf.u + si * nu, uk * sizeof(double));
      }
    }
    OcpQpIpmSolverStatistics& st = batch_stats[bi];
    st.iter = buf.iter[bi];
    st.max_res_stat = buf.res[bi * 4 + 0];
    st.max_res_eq = buf.res[bi * 4 + 1];
    st.max_res_ineq = buf.res[bi * 4 + 2];
    st.max_res_comp = buf.res[bi * 4 + 3];
    st.clear();
    const size_t nrow = std::min(rows, static_cast<size_t>(st.iter) + 2);
    st.reserve(nrow);
    std::vector<double>* cols[] = {
        &st.alpha_aff, &st.mu_aff, &st.sigma, &st.alpha_prim, &st.alpha_dual, &st.mu,
        &st.res_stat, &st.res_eq, &st.res_ineq, &st.res_comp, &st.obj, &st.lq_fact,
        &st.itref_pred, &st.itref_corr, &st.lin_res_stat, &st.lin_res_eq, &st.lin_res_ineq,
        &st.lin_res_comp};
    for (size_t i = 0; i < nrow; ++i)
      for (size_t c = 0; c < 18; ++c) cols[c]->push_back(buf.stat[(bi * rows + i) * 18 + c]);
    const int code = buf.status[bi];
    out[bi] = (code >= 0 && code <= 3) ? static_cast<HpipmStatus>(code) : HpipmStatus::UnknownFailure;
  }
  if (nb) stats = batch_stats[0];
  return out;
}

OcpQpIpmSolver::OcpQpIpmSolver(const std::vector<OcpQp>& ocp_qp,
                               const OcpQpIpmSolverSettings& solver_settings)
    : impl_(new Impl()) {
  setSolverSettings(solver_settings);
  resize(ocp_qp);
}

OcpQpIpmSolver::OcpQpIpmSolver(const OcpQpIpmSolverSettings& solver_settings) : impl_(new Impl()) {
  setSolverSettings(solver_settings);
}

OcpQpIpmSolver::~OcpQpIpmSolver() = default;
OcpQpIpmSolver::OcpQpIpmSolver(OcpQpIpmSolver&&) noexcept = default;
OcpQpIpmSolver& OcpQpIpmSolver::operator=(OcpQpIpmSolver&&) noexcept = default;

// Stores the settings as the reference does (ocp_qp_ipm_solver.cpp:83-117: no
// checkSettings() there); an invalid value is reported by solve(), whose C-ABI call
// runs srbd_qp_check_settings.
void OcpQpIpmSolver::setSolverSettings(const OcpQpIpmSolverSettings& solver_settings) {
  impl_->settings = solver_settings;
}

void OcpQpIpmSolver::resize(const std::vector<OcpQp>& ocp_qp) {
  impl_->dim.resize(ocp_qp);
  impl_->ensure_handle(shape_of(impl_->dim), std::max(impl_->capacity, 1));
}

HpipmStatus OcpQpIpmSolver::solve(const VectorXd& x0, std::vector<OcpQp>& ocp_qp,
                                  std::vector<OcpQpSolution>& qp_sol) {
  std::vector<VectorXd> x0s{x0};
  std::vector<std::vector<OcpQp>> qps(1);
  qps[0].swap(ocp_qp);
  std::vector<std::vector<OcpQpSolution>> sols(1);
  sols[0].swap(qp_sol);
  struct Restore {  // hand the caller's vectors back even when solveBatch throws
    std::vector<OcpQp>& a;
    std::vector<OcpQpSolution>& b;
    std::vector<std::vector<OcpQp>>& qa;
    std::vector<std::vector<OcpQpSolution>>& qb;
    ~Restore() {
      a.swap(qa[0]);
      b.swap(qb[0]);
    }
  } restore{ocp_qp, qp_sol, qps, sols};
  return solveBatch(x0s, qps, sols)[0];
}

std::vector<HpipmStatus> OcpQpIpmSolver::solveBatch(
    const std::vector<VectorXd>& x0, std::vector<std::vector<OcpQp>>& ocp_qp,
    std::vector<std::vector<OcpQpSolution>>& qp_sol) {
  Impl& m = *impl_;
  if (ocp_qp.empty()) throw std::runtime_error("ocp_qp must hold at least one QP");
  if (x0.size() != ocp_qp.size())
    throw std::runtime_error("x0.size() must be " + std::to_string(ocp_qp.size()));
  // dimensions: the first QP sets them, every other QP must match
  m.dim.resize(ocp_qp[0]);
  const Shape s0 = shape_of(m.dim);
  Shape s = s0;
  for (size_t bi = 1; bi < ocp_qp.size(); ++bi) {
    OcpQpDim d(ocp_qp[bi]);
    Shape si = shape_of(d);
    if (d.N != m.dim.N || d.nx != m.dim.nx || d.nu != m.dim.nu)
      throw std::runtime_error("ocp_qp[" + std::to_string(bi) +
                               "]: every QP of a batch must have the same N, nx[i], nu[i]");
    s.ng = std::max(s.ng, si.ng);
    s.box_u = s.box_u || si.box_u;
    s.box_x = s.box_x || si.box_x;
  }
  const int nb = static_cast<int>(ocp_qp.size());
  m.ensure_handle(s, nb);
  // solution containers (ocp_qp_ipm_solver.cpp:186-223)
  if (qp_sol.size() != ocp_qp.size()) qp_sol.resize(ocp_qp.size());
  for (size_t bi = 0; bi < qp_sol.size(); ++bi) {
    std::vector<OcpQpSolution>& sol = qp_sol[bi];
    if (sol.size() != static_cast<size_t>(s.N) + 1) sol.resize(s.N + 1);
    if (m.settings.warm_start) {
      for (int i = 0; i <= s.N; ++i)
        if (sol[i].x.size() != m.dim.nx[i])
          throw std::runtime_error("qp_sol[" + std::to_string(i) + "].x.size() must be " +
                                   std::to_string(m.dim.nx[i]));
      for (int i = 0; i < s.N; ++i)
        if (sol[i].u.size() != m.dim.nu[i])
          throw std::runtime_error("qp_sol[" + std::to_string(i) + "].u.size() must be " +
                                   std::to_string(m.dim.nu[i]));
    }
  }
  const srbd_qp_settings st = m.abi_settings();
  // Unconstrained QPs (the reference's NMPC QP) are packed straight into the C-ABI's pinned
  // staging buffer: the solve then makes no staging copy (and, for up to 256 QPs, the kernel
  // reads and writes that buffer in place).
  srbd_qp_data_f64 d{};
  srbd_qp_solution_f64 o{};
  bool staged = false;
  if (!s.ng && !s.box_u && !s.box_x) {
    const double* mk = reinterpret_cast<const double*>(16);  // "wanted" markers
    double* mo = const_cast<double*>(mk);
    d.A = d.B = d.b = d.Q = d.S = d.R = d.q = d.r = d.x0 = mk;
    o.x = o.u = o.pi = o.P = o.p = o.K = o.k = o.res = o.obj = o.stat = mo;
    o.status = o.iter = reinterpret_cast<int*>(16);
    auto tp = PClock::now();
    staged = srbd_qp_host_staging_f64(m.handle, nb, &st, &d, &o) == SRBD_QP_OK;
    if (g_prof.on) g_prof.t[0] += us_since(tp);
    if (staged) {
      Impl::Bufs bs;
      bs.A = const_cast<double*>(d.A); bs.B = const_cast<double*>(d.B); bs.b = const_cast<double*>(d.b);
      bs.Q = const_cast<double*>(d.Q); bs.S = const_cast<double*>(d.S); bs.R = const_cast<double*>(d.R);
      bs.q = const_cast<double*>(d.q); bs.r = const_cast<double*>(d.r); bs.x0 = const_cast<double*>(d.x0);
      bs.x = o.x; bs.u = o.u; bs.pi = o.pi; bs.P = o.P; bs.p = o.p; bs.K = o.K; bs.k = o.k;
      bs.res = o.res; bs.obj = o.obj; bs.stat = o.stat; bs.status = o.status; bs.iter = o.iter;
      tp = PClock::now();
      m.pack(x0, ocp_qp, m.settings.warm_start ? &qp_sol : nullptr, &bs);
      if (g_prof.on) g_prof.t[1] += us_since(tp);
      // the factors (P, p, K, k: most of the outputs) are unpacked by the callback, while
      // the kernel still runs its forward sweep (srbd_qp_solve_host_cb_f64)
      struct Ctx {
        Impl* m;
        std::vector<std::vector<OcpQpSolution>>* sol;
      } cx{&m, &qp_sol};
      auto on_factors = [](void* p) {
        Ctx* c = static_cast<Ctx*>(p);
        c->m->unpack(*c->sol, Impl::kFactors);
      };
      tp = PClock::now();
      if (srbd_qp_solve_host_cb_f64(m.handle, nb, &st, &d, &o, on_factors, &cx) != SRBD_QP_OK)
        abi_error("OcpQpIpmSolver::solve");
      if (g_prof.on) g_prof.t[2] += us_since(tp);
      tp = PClock::now();
      std::vector<HpipmStatus> res = m.unpack(qp_sol, Impl::kRest);
      if (g_prof.on) {
        g_prof.t[3] += us_since(tp);
        ++g_prof.n;
      }
      return res;
    }
    d = srbd_qp_data_f64{};
    o = srbd_qp_solution_f64{};
  }
  m.pack(x0, ocp_qp, m.settings.warm_start ? &qp_sol : nullptr);
  auto ptr = [](std::vector<double>& v) -> double* { return v.empty() ? nullptr : v.data(); };
  d.A = m.A.data(); d.B = m.B.data(); d.b = m.b.data();
  d.Q = m.Q.data(); d.S = m.S.data(); d.R = m.R.data();
  d.q = m.q.data(); d.r = m.r.data(); d.x0 = m.x0.data();
  if (s.box_u) {
    d.lbu = ptr(m.lbu); d.ubu = ptr(m.ubu); d.lbu_mask = ptr(m.lbu_m); d.ubu_mask = ptr(m.ubu_m);
  }
  if (s.box_x) {
    d.lbx = ptr(m.lbx); d.ubx = ptr(m.ubx); d.lbx_mask = ptr(m.lbx_m); d.ubx_mask = ptr(m.ubx_m);
  }
  if (s.ng) {
    // an all-zero C (e.g. the friction cone, which constrains u only) goes in as
    // NULL: the kernel then skips the C products instead of multiplying zeros
    const bool c_zero = std::all_of(m.C.begin(), m.C.end(), [](double v) { return v == 0.0; });
    d.C = c_zero ? nullptr : ptr(m.C);
    d.D = ptr(m.D); d.lg = ptr(m.lg); d.ug = ptr(m.ug);
    d.lg_mask = ptr(m.lg_m); d.ug_mask = ptr(m.ug_m);
  }
  o.x = m.x.data(); o.u = m.u.data(); o.pi = m.pi.data();
  o.P = m.P.data(); o.p = m.p.data(); o.K = m.K.data(); o.k = m.k.data();
  o.status = m.status.data(); o.iter = m.iter.data(); o.res = m.res.data(); o.obj = m.obj.data();
  o.stat = m.stat.data();
  if (srbd_qp_solve_host_f64(m.handle, nb, &st, &d, &o) != SRBD_QP_OK)
    abi_error("OcpQpIpmSolver::solve");
  return m.unpack(qp_sol);
}

const OcpQpIpmSolverSettings& OcpQpIpmSolver::getIpmSolverSettings() const {
  return impl_->settings;
}

const OcpQpIpmSolverStatistics& OcpQpIpmSolver::getSolverStatistics() const {
  return impl_->stats;
}

const std::vector<OcpQpIpmSolverStatistics>& OcpQpIpmSolver::getBatchStatistics() const {
  return impl_->batch_stats;
}

void OcpQpIpmSolver::setDevice(int device) {
  if (device != impl_->device) impl_->release();
  impl_->device = device;
}

int OcpQpIpmSolver::device() const { return impl_->device; }

}  // namespace hpipm
