// ipm_box.hip -- batched box-constrained OCP-QP interior-point solve.
//
// Replaces, for a batch of QPs, HPIPM's d_ocp_qp_ipm_solve (hpipm_d_ocp_qp_ipm.h:238)
// in its relative formulation: Mehrotra predictor-corrector with the
// residuals of hpipm_d_ocp_qp_res.h:57-67 and the core ops of
// hpipm_d_core_qp_ipm_aux.h:44-62 (Gamma/gamma, alpha, mu_aff, centering
// correction, update), the KKT factorization of d_ocp_qp_fact_solve_kkt_step
// (hpipm_d_ocp_qp_kkt.h:56) and the corrector solve d_ocp_qp_solve_kkt_step
// (:60).  The arithmetic is restated in oracle/ocp_qp_oracle.c (ipm loop), the
// parity reference.
//
// One 16-lane group per QP runs the whole IPM; a wavefront advances four QPs.
// The iteration is host-driven, one launch per pair of sweeps over the horizon
// (k = stage), with per-QP state in the workspace (a QP that has exited returns
// at the top of every later launch):
//   RB  k = N..0  apply the previous step to stage k, its residuals res_g /
//                 res_b / res_d / res_m (norms, mu, obj), Gamma / gamma, and the
//                 barrier-augmented factorization (riccati_step) writing the
//                 stage record {L, K, P, 1/diag L, k, p}.  Every QP
//                 block is read from global memory once per iteration; the
//                 row-owned residual products go through LDS.  After the sweep:
//                 exit test (NaN, converged, iter_max, min step).
//   F1  k = 0..N  predictor step (row-owned from the record), dt / dlam,
//                 alpha_aff and the mu_aff sums -> sigma = (mu_aff / mu)^3
//   B2  k = N..0  corrector right-hand side, vector-only Riccati recursion
//                 reusing the record (element-owned)
//   F2  k = 0..N  corrector step, dt / dlam, alpha_prim / alpha_dual
// RB + F1 and B2 + F2 run as one launch each (ipm_phase2_kernel).
// Box bounds are dense per variable (include/srbd_qp.h), so bound i of u_k /
// x_k lives on lane i next to u_k[i] / x_k[i]: every constraint operation is
// lane-local and the barrier Hessian only touches the diagonals of R and Q.
// General rows (D u + C x, ng <= 64) go in 12-row chunks, lane i = row i.
#include "kernels.h"

#include <cstdlib>
#include "riccati.h"

#define SRBD_REAL double
#define SRBD_NS ipm_f64
#include "ipm_box_impl.h"
#undef SRBD_REAL
#undef SRBD_NS
#define SRBD_REAL float
#define SRBD_NS ipm_f32
#include "ipm_box_impl.h"
#undef SRBD_REAL
#undef SRBD_NS

namespace srbd {

size_t ws_doubles_ipm(int N, int ng) {
  const int nch = (ng + kMaxDim - 1) / kMaxDim;
  return ipm_f64::kQsSize +
         (size_t)(N + 1) * ((size_t)kIpmStage + (size_t)nch * kGenChunk + (nch ? kGenVec : 0));
}

namespace {
__global__ void gather_warm_bars_kernel(const float* __restrict__ ws32, size_t ws_qp, int N,
                                        size_t stride, int nch, const int* __restrict__ idx, int rows,
                                        double* __restrict__ dst) {
  const size_t W = 96 + (size_t)nch * 48, per_qp = (size_t)(N + 1) * W;
  const size_t total = (size_t)rows * per_qp;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t r = t / per_qp, rem = t - r * per_qp, k = rem / W, j = rem - k * W;
    const size_t off = j < 96 ? kStLam + j : kIpmStage + ((j - 96) / 48) * kGenChunk + (j - 96) % 48;
    const size_t q = idx ? (size_t)idx[r] : r;
    dst[t] = (double)ws32[q * ws_qp + ipm_f32::kQsSize + k * stride + off];
  }
}
// f32_iters: one thread per (QP, stage, value); exp = ((c + 2) & 3) * 12 maps a bar component
// (ll, lu, tl, tu) to its step (dll at 24, dlu at 36, dtl at 0, dtu at 12)
__global__ void gather_warm_apply_kernel(const float* __restrict__ ws32, size_t ws_qp, int N,
                                         size_t stride, int nch, int batch, double* __restrict__ dst) {
  const size_t W = 96 + (size_t)nch * 48, per_qp = (size_t)(N + 1) * W;
  const size_t total = (size_t)batch * per_qp;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t q = t / per_qp, rem = t - q * per_qp, k = rem / W, j = rem - k * W;
    const float* qs = ws32 + q * ws_qp;
    const float* st = qs + ipm_f32::kQsSize + k * stride;
    const bool pending = qs[ipm_f32::kQsStatus] < 0.0f;
    const size_t f = j < 96 ? j / 48 : 0, c = ((j < 96 ? j : j - 96) % 48) / 12, i = j % 12;
    const float* bar = j < 96 ? st + kStLam + j
                              : st + kIpmStage + ((j - 96) / 48) * kGenChunk + (j - 96) % 48;
    const float* stp = j < 96 ? st + kStDlt + f * 48 + ((c + 2) & 3) * 12 + i
                              : st + kIpmStage + ((j - 96) / 48) * kGenChunk + 48 + ((c + 2) & 3) * 12 + i;
    const float a = pending ? qs[c < 2 ? ipm_f32::kQsAlphaD : ipm_f32::kQsAlphaP] : 0.0f;
    double v = (double)*bar;
    if (a != 0.0f) v += (double)a * (double)*stp;
    dst[t] = v;
  }
}

__global__ void gather_warm_iterate_kernel(const float* __restrict__ ws32, size_t ws_qp, int N,
                                           size_t stride, int batch, const float* __restrict__ x32,
                                           const float* __restrict__ u32, const float* __restrict__ pi32,
                                           double* __restrict__ x, double* __restrict__ u,
                                           double* __restrict__ pi) {
  const size_t ex = (size_t)(N + 1) * 12, eu = (size_t)N * 12, per_qp = 2 * ex + eu;
  const size_t total = (size_t)batch * per_qp;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t q = t / per_qp, rem = t - q * per_qp;
    const float* qs = ws32 + q * ws_qp;
    const bool pending = qs[ipm_f32::kQsStatus] < 0.0f;
    const float ap = pending ? qs[ipm_f32::kQsAlphaP] : 0.0f, ad = pending ? qs[ipm_f32::kQsAlphaD] : 0.0f;
    if (rem < ex) {  // x (x_0 is never stepped)
      const size_t k = rem / 12, i = rem % 12;
      double v = (double)x32[q * ex + rem];
      if (k > 0 && ap != 0.0f)
        v += (double)ap * (double)qs[ipm_f32::kQsSize + k * stride + kStStep + 12 + i];
      x[q * ex + rem] = v;
    } else if (rem < ex + eu) {
      const size_t e = rem - ex, k = e / 12, i = e % 12;
      double v = (double)u32[q * eu + e];
      if (ap != 0.0f) v += (double)ap * (double)qs[ipm_f32::kQsSize + k * stride + kStStep + i];
      u[q * eu + e] = v;
    } else {
      const size_t e = rem - ex - eu, k = e / 12, i = e % 12;
      double v = (double)pi32[q * ex + e];
      if (k > 0 && ad != 0.0f)
        v += (double)ad * (double)qs[ipm_f32::kQsSize + k * stride + kStStep + 24 + i];
      pi[q * ex + e] = v;
    }
  }
}
}  // namespace

hipError_t launch_gather_warm_apply(const float* ws32, size_t ws_qp, int N, int ng, int batch,
                                    const float* x32, const float* u32, const float* pi32, double* x,
                                    double* u, double* pi, double* bars, hipStream_t s) {
  if (batch <= 0) return hipSuccess;
  const int nch = (ng + kMaxDim - 1) / kMaxDim;
  const size_t stride = (size_t)kIpmStage + (size_t)nch * kGenChunk + (nch ? kGenVec : 0);
  auto grid = [](size_t total) {
    const size_t blocks = (total + 255) / 256;
    return dim3((unsigned)(blocks < 8192 ? blocks : 8192));
  };
  const size_t tb = (size_t)batch * (N + 1) * (96 + (size_t)nch * 48);
  hipLaunchKernelGGL(gather_warm_apply_kernel, grid(tb), dim3(256), 0, s, ws32, ws_qp, N, stride, nch,
                     batch, bars);
  const size_t ti = (size_t)batch * ((size_t)(N + 1) * 24 + (size_t)N * 12);
  hipLaunchKernelGGL(gather_warm_iterate_kernel, grid(ti), dim3(256), 0, s, ws32, ws_qp, N, stride, batch,
                     x32, u32, pi32, x, u, pi);
  return hipGetLastError();
}

hipError_t launch_gather_warm_bars(const float* ws32, size_t ws_qp, int N, int ng, const int* idx,
                                   int rows, double* dst, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  const int nch = (ng + kMaxDim - 1) / kMaxDim;
  const size_t stride = (size_t)kIpmStage + (size_t)nch * kGenChunk + (nch ? kGenVec : 0);
  const size_t total = (size_t)rows * (N + 1) * (96 + (size_t)nch * 48);
  const size_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(gather_warm_bars_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256),
                     0, s, ws32, ws_qp, N, stride, nch, idx, rows, dst);
  return hipGetLastError();
}

// Small fp64 batches of the classical-Riccati Speed solve go to the one-launch latency IPM
// (ipm_latency.hip); SRBD_IPM_LATENCY_MAX (QPs, default kIpmLatencyMaxBatch, 0 = off) moves the
// switch point (read at every launch, so a test can run one problem through both paths).
int ipm_latency_max_batch() {
  const char* e = std::getenv("SRBD_IPM_LATENCY_MAX");
  return e ? std::atoi(e) : kIpmLatencyMaxBatch;
}

template <>
hipError_t launch_ipm_box<double>(const ProblemArgsT<double>& a, hipStream_t stream) {
  if (ipm_latency_ok(a, ipm_latency_max_batch())) return launch_ipm_latency(a, stream);
  return ipm_f64::launch(a, stream);
}
hipError_t launch_ipm_box_batched(const ProblemArgsT<double>& a, hipStream_t stream) {
  return ipm_f64::launch(a, stream);
}
template <>
hipError_t launch_ipm_box<float>(const ProblemArgsT<float>& a, hipStream_t stream) {
  return ipm_f32::launch(a, stream);
}

}  // namespace srbd

#if SRBD_TSTAMP
// Diagnostic builds only: this translation unit's stamp buffer (the IPM kernels), as
// srbd_qp_diag_tstamps does for the unconstrained ones.
extern "C" int srbd_qp_diag_tstamps_ipm(unsigned long long* out, int cap) {
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
