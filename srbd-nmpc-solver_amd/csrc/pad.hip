// pad.hip -- problems with nx < 12 or nu < 12 run through the 12 x 12 kernels.
//
// HPIPM sizes every stage to its own nx / nu (hpipm_d_ocp_qp_dim.h); here the
// solver kernels exist for the 12 x 12 stage only, so a smaller problem is
// embedded in it before the solve and cut out of it afterwards:
//   * padded states: zero rows / columns of A, B (rows), Q, S, C, zero b, q, x0
//     -> they stay 0 and contribute nothing;
//   * padded inputs: zero columns of B, S (rows), D, zero r, R = 1 on the
//     padded diagonal -> u_pad = 0, and the Cholesky of R + B'PB stays defined;
//   * padded bounds are masked (mask 0), i.e. absent, exactly like an index
//     not listed in idxbu / idxbx (d_ocp_qp_set_lbu_mask semantics).
// The embedded QP has the same KKT system plus decoupled identity rows, so the
// solution, the residual norms and the iteration trace are those of the
// original one.  lg / ug (and their masks) keep their shape and are not copied.
#include "kernels.h"

#include <hip/hip_runtime.h>

namespace srbd {
namespace {

// dst: nblk blocks of dr x dc (column-major); src: nblk blocks of sr x sc (or
// NULL: every in-range element is `dflt`).  Out-of-range elements are `fill`,
// `diag` on the diagonal.
template <typename T>
__global__ void __launch_bounds__(256) pad_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                  long long nblk, int sr, int sc, int dr, int dc,
                                                  T fill, T diag, T dflt) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)dr * dc;
  if (t >= nblk * per) return;
  const long long blk = t / per;
  const int e = (int)(t - blk * per);
  const int i = e % dr, j = e / dr;
  T v;
  if (i < sr && j < sc)
    v = src ? src[blk * ((long long)sr * sc) + (long long)j * sr + i] : dflt;
  else
    v = i == j ? diag : fill;
  dst[t] = v;
}

// dst: nblk blocks of sr x sc cut out of src's dr x dc blocks
template <typename T>
__global__ void __launch_bounds__(256) unpad_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                    long long nblk, int sr, int sc, int dr, int dc) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)sr * sc;
  if (t >= nblk * per) return;
  const long long blk = t / per;
  const int e = (int)(t - blk * per);
  const int i = e % sr, j = e / sr;
  dst[t] = src[blk * ((long long)dr * dc) + (long long)j * dr + i];
}

template <typename T>
hipError_t pad(const T* src, T* dst, long long nblk, int sr, int sc, int dr, int dc, T fill, T diag,
               T dflt, hipStream_t s) {
  const long long n = nblk * dr * dc;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(pad_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, nblk,
                     sr, sc, dr, dc, fill, diag, dflt);
  return hipGetLastError();
}

template <typename T>
hipError_t unpad(const T* src, T* dst, long long nblk, int sr, int sc, int dr, int dc, hipStream_t s) {
  const long long n = nblk * sr * sc;
  if (n <= 0 || !dst) return hipSuccess;
  hipLaunchKernelGGL(unpad_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst,
                     nblk, sr, sc, dr, dc);
  return hipGetLastError();
}

// Element offsets of the padded arrays inside the pad buffer (per `batch` QPs).
struct PadLayout {
  size_t A, B, b, Q, S, R, q, r, x0, lbu, ubu, lbum, ubum, lbx, ubx, lbxm, ubxm, C, D;
  size_t x, u, pi, P, p, K, k, total;
  PadLayout(size_t batch, size_t N, size_t ng) {
    size_t o = 0;
    auto take = [&](size_t n) {
      const size_t at = o;
      o += (n + 31) / 32 * 32;  // 256-byte aligned in fp64
      return at;
    };
    const size_t M = 144, V = 12;
    A = take(batch * N * M); B = take(batch * N * M); b = take(batch * N * V);
    Q = take(batch * (N + 1) * M); S = take(batch * N * M); R = take(batch * N * M);
    q = take(batch * (N + 1) * V); r = take(batch * N * V); x0 = take(batch * V);
    lbu = take(batch * N * V); ubu = take(batch * N * V); lbum = take(batch * N * V); ubum = take(batch * N * V);
    lbx = take(batch * (N + 1) * V); ubx = take(batch * (N + 1) * V);
    lbxm = take(batch * (N + 1) * V); ubxm = take(batch * (N + 1) * V);
    C = take(batch * (N + 1) * ng * V); D = take(batch * N * ng * V);
    x = take(batch * (N + 1) * V); u = take(batch * N * V); pi = take(batch * (N + 1) * V);
    P = take(batch * (N + 1) * M); p = take(batch * (N + 1) * V); K = take(batch * N * M); k = take(batch * N * V);
    total = o;
  }
};

}  // namespace

size_t pad_elems(int batch, int N, int ng) { return PadLayout(batch, N, ng).total; }

template <typename T>
hipError_t pad_problem(const ProblemArgsT<T>& a, T* buf, ProblemArgsT<T>& o, hipStream_t s) {
  const PadLayout L(a.batch, a.N, a.ng);
  const long long Bq = a.batch, N = a.N;
  const int nx = a.nx, nu = a.nu, ng = a.ng;
  const T z = T(0), one = T(1);
  o = a;
  o.nx = 12;
  o.nu = 12;
  hipError_t e = hipSuccess;
  auto P = [&](const T* src, size_t off, long long nblk, int sr, int sc, int dr, int dc, T diag, T dflt,
               const T*& field) {
    if (e != hipSuccess) return;
    T* dst = buf + off;
    e = pad<T>(src, dst, nblk, sr, sc, dr, dc, z, diag, dflt, s);
    field = dst;
  };
  P(a.A, L.A, Bq * N, nx, nx, 12, 12, z, z, o.A);
  P(a.B, L.B, Bq * N, nx, nu, 12, 12, z, z, o.B);
  P(a.b, L.b, Bq * N, nx, 1, 12, 1, z, z, o.b);
  P(a.Q, L.Q, Bq * (N + 1), nx, nx, 12, 12, z, z, o.Q);
  P(a.S, L.S, Bq * N, nu, nx, 12, 12, z, z, o.S);
  P(a.R, L.R, Bq * N, nu, nu, 12, 12, one, z, o.R);  // padded inputs: R = 1
  P(a.q, L.q, Bq * (N + 1), nx, 1, 12, 1, z, z, o.q);
  P(a.r, L.r, Bq * N, nu, 1, 12, 1, z, z, o.r);
  P(a.x0, L.x0, Bq, nx, 1, 12, 1, z, z, o.x0);
  if (a.lbu) {  // padded bounds: value 0, mask 0 (absent); a NULL mask means all active
    P(a.lbu, L.lbu, Bq * N, nu, 1, 12, 1, z, z, o.lbu);
    P(a.ubu, L.ubu, Bq * N, nu, 1, 12, 1, z, z, o.ubu);
    P(a.lbu_mask, L.lbum, Bq * N, nu, 1, 12, 1, z, one, o.lbu_mask);
    P(a.ubu_mask, L.ubum, Bq * N, nu, 1, 12, 1, z, one, o.ubu_mask);
  }
  if (a.lbx) {
    P(a.lbx, L.lbx, Bq * (N + 1), nx, 1, 12, 1, z, z, o.lbx);
    P(a.ubx, L.ubx, Bq * (N + 1), nx, 1, 12, 1, z, z, o.ubx);
    P(a.lbx_mask, L.lbxm, Bq * (N + 1), nx, 1, 12, 1, z, one, o.lbx_mask);
    P(a.ubx_mask, L.ubxm, Bq * (N + 1), nx, 1, 12, 1, z, one, o.ubx_mask);
  }
  if (ng > 0 && a.C) P(a.C, L.C, Bq * (N + 1), ng, nx, ng, 12, z, z, o.C);
  if (ng > 0 && a.D) P(a.D, L.D, Bq * N, ng, nu, ng, 12, z, z, o.D);
  // solution buffers (x, u are also the warm start)
  T* const X = buf + L.x;
  T* const U = buf + L.u;
  if (e == hipSuccess) {
    if (a.warm_start) {
      e = pad<T>(a.x, X, Bq * (N + 1), nx, 1, 12, 1, z, z, z, s);
      if (e == hipSuccess) e = pad<T>(a.u, U, Bq * N, nu, 1, 12, 1, z, z, z, s);
    }
  }
  o.x = X;
  o.u = U;
  o.pi = buf + L.pi;
  o.P = a.P ? buf + L.P : nullptr;
  o.p = a.p ? buf + L.p : nullptr;
  o.K = a.K ? buf + L.K : nullptr;
  o.k = a.k ? buf + L.k : nullptr;
  return e;
}

template <typename T>
hipError_t unpad_solution(const ProblemArgsT<T>& a, const ProblemArgsT<T>& o, hipStream_t s) {
  const long long Bq = a.batch, N = a.N;
  const int nx = a.nx, nu = a.nu;
  hipError_t e = unpad<T>(o.x, a.x, Bq * (N + 1), nx, 1, 12, 1, s);
  if (e == hipSuccess) e = unpad<T>(o.u, a.u, Bq * N, nu, 1, 12, 1, s);
  if (e == hipSuccess) e = unpad<T>(o.pi, a.pi, Bq * (N + 1), nx, 1, 12, 1, s);
  if (e == hipSuccess && a.P) e = unpad<T>(o.P, a.P, Bq * (N + 1), nx, nx, 12, 12, s);
  if (e == hipSuccess && a.p) e = unpad<T>(o.p, a.p, Bq * (N + 1), nx, 1, 12, 1, s);
  if (e == hipSuccess && a.K) e = unpad<T>(o.K, a.K, Bq * N, nu, nx, 12, 12, s);
  if (e == hipSuccess && a.k) e = unpad<T>(o.k, a.k, Bq * N, nu, 1, 12, 1, s);
  return e;
}

template hipError_t pad_problem<double>(const ProblemArgsT<double>&, double*, ProblemArgsT<double>&,
                                        hipStream_t);
template hipError_t pad_problem<float>(const ProblemArgsT<float>&, float*, ProblemArgsT<float>&,
                                       hipStream_t);
template hipError_t unpad_solution<double>(const ProblemArgsT<double>&, const ProblemArgsT<double>&,
                                           hipStream_t);
template hipError_t unpad_solution<float>(const ProblemArgsT<float>&, const ProblemArgsT<float>&,
                                          hipStream_t);

}  // namespace srbd
