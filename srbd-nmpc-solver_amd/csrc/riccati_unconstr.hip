// riccati_unconstr.hip -- batched unconstrained OCP-QP solve (nc == 0).
//
// Replaces, for a batch of QPs, HPIPM's nc == 0 branch of d_ocp_qp_ipm_solve:
// one d_ocp_qp_fact_solve_kkt_unconstr (hpipm_d_ocp_qp_kkt.h:54) and
// iter = 0 (pinned by hpipm-cpp/test/ocp_qp_ipm_solver.cpp:55-56), plus the
// getters and stage-0 rebuild of hpipm-cpp/src/ocp_qp_ipm_solver.cpp:337-373.
//
// One kernel, two sweeps per QP group (see qp_group.h):
//   backward k = N-1..0 : riccati_step on the stage's column-owned blocks,
//                         then write the forward record {K, P, k, p} to the
//                         per-QP workspace;
//   forward  k = 0..N   : row-owned u = K x + k, pi = P x + p,
//                         x+ = A x + B u + b, with x, u broadcast by DPP.
// The forward sweep reads the records in LIFO order (stage 0 was written
// last), so the most recent records are still in L2 / Infinity Cache.
//
// The stage-0 block is factorized in full with x_0 = x0 fixed, which gives
// exactly the values of the reference's x0-eliminated solve + stage-0
// rebuild (K0 = -G0^-1 H0, P0 = Q0 - H0'G0^-1 H0 + A0'P1 A0, ...).
#include "kernels.h"
#include "riccati.h"
#include "mfma_lat.h"

#define SRBD_REAL double
#define SRBD_NS ric_f64
#define SRBD_WITH_LATENCY 1  // the fp64 matrix-core single-QP kernel (riccati_latency_impl.h)
#include "riccati_unconstr_impl.h"
#undef SRBD_WITH_LATENCY
#undef SRBD_REAL
#undef SRBD_NS
#define SRBD_WITH_LATENCY 0
#define SRBD_REAL float
#define SRBD_NS ric_f32
#include "riccati_unconstr_impl.h"
#undef SRBD_REAL
#undef SRBD_NS

namespace srbd {

size_t ws_doubles_unconstr(int N) { return (size_t)(N + 1) * kWsStage; }

hipError_t prepare_riccati_device() {
  hipError_t e = ric_f64::prepare_device();
  return e == hipSuccess ? ric_f32::prepare_device() : e;
}

template <>
hipError_t launch_riccati_unconstr<double>(const ProblemArgsT<double>& a, hipStream_t stream) {
  return ric_f64::launch(a, stream);
}
template <>
hipError_t launch_riccati_unconstr<float>(const ProblemArgsT<float>& a, hipStream_t stream) {
  return ric_f32::launch(a, stream);
}
template <>
hipError_t launch_unconstr_residuals<double>(const ProblemArgsT<double>& a, hipStream_t stream) {
  return ric_f64::launch_residuals(a, stream);
}
template <>
hipError_t launch_unconstr_residuals<float>(const ProblemArgsT<float>& a, hipStream_t stream) {
  return ric_f32::launch_residuals(a, stream);
}
template <>
bool unconstr_fused_residuals<double>(const ProblemArgsT<double>& a) {
  return ric_f64::fused_residuals(a);
}
template <>
bool unconstr_fused_residuals<float>(const ProblemArgsT<float>& a) {
  return ric_f32::fused_residuals(a);
}
template <>
bool unconstr_reads_once<double>(const ProblemArgsT<double>& a) {
  return ric_f64::reads_once(a);
}
template <>
bool unconstr_reads_once<float>(const ProblemArgsT<float>& a) {
  return ric_f32::reads_once(a);
}
bool latency_server_ok(const ProblemArgsT<double>& a) { return ric_f64::server_ok(a); }
hipError_t launch_latency_server(const ProblemArgsT<double>& a, LatMailbox* mb, int epoch, int last_done,
                                 long long idle_ticks, long long life_ticks, hipStream_t stream) {
  return ric_f64::launch_server(a, mb, epoch, last_done, idle_ticks, life_ticks, stream);
}

}  // namespace srbd

#if SRBD_TSTAMP
// Diagnostic builds only (not part of include/srbd_qp.h): copy the (id, cycle) pairs the
// last launches appended (this translation unit's buffer: the unconstrained kernels) and
// reset the buffer; returns the number of pairs.
extern "C" int srbd_qp_diag_tstamps(unsigned long long* out, int cap) {
  unsigned n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(srbd::g_tstamp_n), sizeof n) != hipSuccess) return -1;
  if (n > (unsigned)srbd::kTstampCap) n = srbd::kTstampCap;
  if ((int)n > cap) n = (unsigned)cap;
  if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(srbd::g_tstamp), 2 * sizeof(unsigned long long) * n) != hipSuccess)
    return -1;
  const unsigned zero = 0;
  hipMemcpyToSymbol(HIP_SYMBOL(srbd::g_tstamp_n), &zero, sizeof zero);
  return (int)n;
}
#endif
