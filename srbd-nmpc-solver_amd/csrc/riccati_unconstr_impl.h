// riccati_unconstr_impl.h -- body of the unconstrained batched solve, instantiated
// per precision by riccati_unconstr.hip (SRBD_REAL, SRBD_NS).  No include guard.

#ifndef SRBD_EARLY_LOADS
#define SRBD_EARLY_LOADS 0
#endif
#ifndef SRBD_PREFETCH_AB
#define SRBD_PREFETCH_AB 0
#endif
#ifndef SRBD_NT_REC
#define SRBD_NT_REC 0
#endif
#ifndef SRBD_NT_INPUTS
#define SRBD_NT_INPUTS 0
#endif
namespace srbd {
namespace SRBD_NS {

using real = SRBD_REAL;


// out[i] = v[i] for i < n (static register indices, predicated stores)
__device__ __forceinline__ void store_n(real* out, int n, const real (&v)[12]) {
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    if (I < n) out[I] = v[I];
  });
}

template <bool FULL>
struct StageLoader {
  int nx, nu;
  // column `col` of an (rows x ncols) column-major block, zero-padded
  __device__ __forceinline__ void col(const real* blk, int rows, int ld, int c, bool ok,
                                      real (&v)[12]) const {
    if constexpr (FULL) {
#if SRBD_NT_INPUTS == 2
      load12_nt(blk + c * 12, v);
#elif SRBD_NT_INPUTS
      // streamed once: non-temporal, so the records keep the caches
      const real* q = blk + c * 12;
      sfor<0, 12>([&](auto i) {
        constexpr int I = decltype(i)::value;
        v[I] = __builtin_nontemporal_load(q + I);
      });
#else
      load12(blk + c * 12, v);
#endif
    } else {
      load_col_pad(blk + (size_t)c * ld, rows, ok, v);
    }
  }
};

template <bool FULL>
__global__ void __launch_bounds__(256, 2) riccati_unconstr_kernel(ProblemArgsT<real> a) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int qp = gid >> 4;
  const int lane = threadIdx.x & (kGroup - 1);
  if (qp >= a.batch) return;
  const int N = a.N;
  const int nx = FULL ? 12 : a.nx;
  const int nu = FULL ? 12 : a.nu;
  const bool isv = lane == kVecLane;
  const int col = lane < kMaxDim ? lane : kMaxDim - 1;
  const real reg = a.reg;

  const size_t nxx = (size_t)nx * nx, nxu = (size_t)nx * nu, nuu = (size_t)nu * nu;
#ifdef SRBD_DIAG_SHARED_INPUT  // diagnostic build only: every QP reads QP (qp & 63)'s data
  const int qin = qp & 63;
#else
  const int qin = qp;
#endif
  // input block of stage k: QP-major ([batch][stage][blk], Eigen order) or
  // stage-major ([stage][batch][blk]: a wavefront's QPs adjacent in memory)
  const bool smaj = a.layout == 1;
  auto at = [&](const real* base, int nstage, size_t blk, int k) -> const real* {
    return smaj ? base + ((size_t)k * a.batch + qin) * blk : base + ((size_t)qin * nstage + k) * blk;
  };
  // forward records, stage-major: stage k of QP q at ws[(k * batch + q) * kWsStage], so the
  // four QPs of a wavefront write / read one contiguous 15 KB block per stage
  auto rec_at = [&](int k) -> real* {
#if SRBD_WS_STAGE_MAJOR
    return a.ws + ((size_t)k * a.batch + qp) * kWsStage;
#else
    return a.ws + (size_t)qp * a.ws_qp + (size_t)k * kWsStage;
#endif
  };

  StageLoader<FULL> ld{nx, nu};
  const bool xcol = lane < nx;  // lane owns a real state column
  const bool ucol = lane < nu;  // lane owns a real input column

  // ---------------- terminal stage: P_N = Q_N, p_N = q_N ----------------
  real P[12];
  if (isv) {
    ld.col(at(a.q, N + 1, nx, N), nx, nx, 0, true, P);
  } else {
    ld.col(at(a.Q, N + 1, nxx, N), nx, nx, col, xcol, P);
  }
  {
    real* rec = rec_at(N);
    if (lane < kMaxDim) store_packed_col(rec + kWsP, lane, P);
    if (isv) store12(rec + kWsp, P);
    if (a.P && xcol) store_n(a.P + ((size_t)qp * (N + 1) + N) * nxx + (size_t)lane * nx, nx, P);
    if (a.p && isv) store_n(a.p + ((size_t)qp * (N + 1) + N) * nx, nx, P);
  }

  // ---------------- backward sweep ----------------
  real A_[12], B_[12];
  // A, B (VL: b) of stage k: column-owned
  auto loadAB = [&](int k, real (&Av)[12], real (&Bv)[12]) {
    if (isv) {
      ld.col(at(a.b, N, nx, k), nx, nx, 0, true, Av);
      sfor<0, 12>([&](auto i) { Bv[decltype(i)::value] = real(0.0); });
    } else {
      ld.col(at(a.A, N, nxx, k), nx, nx, col, xcol, Av);
      ld.col(at(a.B, N, nxu, k), nx, nx, col, ucol, Bv);
    }
  };
#if SRBD_PREFETCH_AB == 3
  // B of stage k only (VL: zeros)
  auto loadB = [&](int k, real (&Bv)[12]) {
    if (isv) {
      sfor<0, 12>([&](auto i) { Bv[decltype(i)::value] = real(0.0); });
    } else {
      ld.col(at(a.B, N, nxu, k), nx, nx, col, ucol, Bv);
    }
  };
  auto loadA = [&](int k, real (&Av)[12]) {
    if (isv) {
      ld.col(at(a.b, N, nx, k), nx, nx, 0, true, Av);
    } else {
      ld.col(at(a.A, N, nxx, k), nx, nx, col, xcol, Av);
    }
  };
  if (N > 0) loadB(N - 1, B_);
#elif SRBD_PREFETCH_AB
  if (N > 0) loadAB(N - 1, A_, B_);
#endif
#pragma unroll 1
  for (int k = N - 1; k >= 0; --k) {
#if SRBD_PREFETCH_AB == 3
    loadA(k, A_);
#elif !SRBD_PREFETCH_AB
    loadAB(k, A_, B_);
#endif
    auto loadR = [&](real (&Rc)[12]) {
      if (isv) {
        sfor<0, 12>([&](auto i) { Rc[decltype(i)::value] = real(0.0); });
      } else {
        ld.col(at(a.R, N, nuu, k), nu, nu, col, ucol, Rc);
        if constexpr (!FULL) {
          // padded inputs: R = 1 on the diagonal keeps G positive definite
          sfor<0, 12>([&](auto i) {
            constexpr int I = decltype(i)::value;
            if (lane == I && lane >= nu) Rc[I] = real(1.0);
          });
        }
      }
    };
    auto loadSQ = [&](real (&Sc)[12], real (&Qc)[12]) {
      if (isv) {
        ld.col(at(a.r, N, nu, k), nu, nu, 0, true, Sc);
        ld.col(at(a.q, N + 1, nx, k), nx, nx, 0, true, Qc);
      } else {
        ld.col(at(a.S, N, nxu, k), nu, nu, col, xcol, Sc);
        ld.col(at(a.Q, N + 1, nxx, k), nx, nx, col, xcol, Qc);
      }
    };
    StageFactor<real> f;
#if SRBD_PREFETCH_AB
    // the next stage's A, B are requested half-way through this stage (after the
    // products, before the triangular solves), so their latency hides behind
    // the solves, the P update and the record stores
    real An[12], Bn[12];
#if SRBD_PREFETCH_AB == 3
    // B only (24 VGPRs): A is requested at the top of the stage and hides
    // behind P B, G and the Cholesky
    riccati_step<1>(P, A_, B_, loadR, loadSQ, lane, reg, f, [&]() {
      if (k > 0) loadB(k - 1, Bn);
    });
#else
    riccati_step<SRBD_PREFETCH_AB>(P, A_, B_, loadR, loadSQ, lane, reg, f, [&]() {
      if (k > 0) loadAB(k - 1, An, Bn);
    });
#endif
#elif SRBD_EARLY_LOADS
    // all five blocks of the stage requested up front: one memory latency per
    // stage instead of three (R, then S/Q, behind the phase fences)
    real Re[12], Se[12], Qe[12];
    loadR(Re);
    loadSQ(Se, Qe);
    riccati_step(
        P, A_, B_,
        [&](real (&Rc)[12]) {
          sfor<0, 12>([&](auto i) { Rc[decltype(i)::value] = Re[decltype(i)::value]; });
        },
        [&](real (&Sc)[12], real (&Qc)[12]) {
          sfor<0, 12>([&](auto i) {
            Sc[decltype(i)::value] = Se[decltype(i)::value];
            Qc[decltype(i)::value] = Qe[decltype(i)::value];
          });
        },
        lane, reg, f);
#else
    riccati_step(P, A_, B_, loadR, loadSQ, lane, reg, f);
#endif

    real* rec = rec_at(k);
#ifdef SRBD_DIAG_NO_RECORD  // diagnostic build only: no record traffic
    if (k == -7) {
#else
    if (lane < kMaxDim) {
#endif
      sfor<0, 12>([&](auto m) {
        constexpr int M = decltype(m)::value;
        rec[kWsK + M * 12 + lane] = f.Kc[M];
        rec[kWsAcl + M * 12 + lane] = A_[M];
      });
      store_packed_col(rec + kWsP, lane, f.F);
    }
    if (isv) {
      store12(rec + kWsk, f.Kc);
      store12(rec + kWsbcl, A_);
      store12(rec + kWsp, f.F);
    }
    if (a.P && xcol) store_n(a.P + ((size_t)qp * (N + 1) + k) * nxx + (size_t)lane * nx, nx, f.F);
    if (a.p && isv) store_n(a.p + ((size_t)qp * (N + 1) + k) * nx, nx, f.F);
    if (a.K && xcol) store_n(a.K + ((size_t)qp * N + k) * nxu + (size_t)lane * nu, nu, f.Kc);
    if (a.k && isv) store_n(a.k + ((size_t)qp * N + k) * nu, nu, f.Kc);
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      P[I] = f.F[I];
    });
#if SRBD_PREFETCH_AB == 3
    sfor<0, 12>([&](auto i) { B_[decltype(i)::value] = Bn[decltype(i)::value]; });
#elif SRBD_PREFETCH_AB
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      A_[I] = An[I];
      B_[I] = Bn[I];
    });
#endif
  }

  // ---------------- forward sweep (row-owned) ----------------
  // The record rows of stage k+1 are loaded while stage k computes (the loads
  // do not depend on x), so each stage pays one memory latency less.
  const int row = lane < kMaxDim ? lane : kMaxDim - 1;
  real xv = (lane < nx) ? a.x0[(size_t)qp * nx + lane] : real(0.0);
  bool bad = false;
  real* xo = a.x + (size_t)qp * (N + 1) * nx;
  real* uo = a.u + (size_t)qp * N * nu;
  real* po = a.pi + (size_t)qp * (N + 1) * nx;
  real Pr[12], Kr[12], Ar[12], pv, kv, bv;
  auto load_rows = [&](int k, real (&P_)[12], real (&K_)[12], real (&A__)[12], real& p_,
                       real& k_, real& b_) {
    const real* rec = rec_at(k);
    load_packed_sym(rec + kWsP, row, P_);
    p_ = rec[kWsp + row];
    if (k < N) {
#if SRBD_NT_REC
      load12_nt(rec + kWsK + row * 12, K_);
      load12_nt(rec + kWsAcl + row * 12, A__);
#else
      load12(rec + kWsK + row * 12, K_);
      load12(rec + kWsAcl + row * 12, A__);
#endif
      k_ = rec[kWsk + row];
      b_ = rec[kWsbcl + row];
    }
  };
  load_rows(0, Pr, Kr, Ar, pv, kv, bv);
#ifdef SRBD_DIAG_NO_FWD  // diagnostic build only
  if (N > 0) return;
#endif
#pragma unroll 1
  for (int k = 0; k <= N; ++k) {
    real Pn[12], Kn[12], An[12], pvn = real(0.0), kvn = real(0.0), bvn = real(0.0);
    if (k < N) load_rows(k + 1, Pn, Kn, An, pvn, kvn, bvn);
    real bx[12];
    sfor<0, 12>([&](auto j) {
      constexpr int J = decltype(j)::value;
      bx[J] = bc<J>(xv);
    });
    real pp = pv;
    sfor<0, 12>([&](auto j) {
      constexpr int J = decltype(j)::value;
      pp = fmadd(Pr[J], bx[J], pp);
    });
    if (lane < nx) {
      xo[(size_t)k * nx + lane] = xv;
      po[(size_t)k * nx + lane] = pp;
    }
    if (k == N) break;
    real uu = kv, xn = bv;
    sfor<0, 12>([&](auto j) {
      constexpr int J = decltype(j)::value;
      uu = fmadd(Kr[J], bx[J], uu);
      xn = fmadd(Ar[J], bx[J], xn);
    });
    if (lane < nu) uo[(size_t)k * nu + lane] = uu;
    bad |= (lane < nu && !(uu == uu)) || (lane < nx && !(xn == xn));
    xv = xn;
    sfor<0, 12>([&](auto j) {
      constexpr int J = decltype(j)::value;
      Pr[J] = Pn[J];
      Kr[J] = Kn[J];
      Ar[J] = An[J];
    });
    pv = pvn;
    kv = kvn;
    bv = bvn;
  }
  if (a.status || a.iter) {
    const unsigned long long m = __ballot(bad);
    const int shift = (threadIdx.x & 63) & ~(kGroup - 1);
    const bool any_bad = ((m >> shift) & 0xffffull) != 0;
    if (lane == 0) {
      if (a.status) a.status[qp] = any_bad ? 3 : 0;
      if (a.iter) a.iter[qp] = 0;
    }
  }
}


// KKT residuals and objective of an unconstrained solution: HPIPM's
// d_ocp_qp_res_compute (hpipm_d_ocp_qp_res.h:57-67) for nc = 0, as the oracle's
// compute_residuals states it (oracle/ocp_qp_oracle.c):
//   res_stat = max( |R u + S x + r + B'pi_{k+1}| (k < N), |Q x + S'u + q + A'pi_{k+1} - pi_k| (k >= 1) )
//   res_eq   = max |A x + B u + b - x_{k+1}|,   res_ineq = res_comp = 0,
//   obj      = sum_k u'(R u / 2 + r) + x'(Q x / 2 + q) (k >= 1) + u'S x.
// Run only when the caller asks for res / obj.  One 32-lane group per QP, lane l
// takes stages l, l + 32, ...; any dims (padded problems are checked unpadded).
constexpr int kResGroup = 32;
__global__ void __launch_bounds__(256) unconstr_residuals_kernel(ProblemArgsT<real> a) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int qp = gid / kResGroup, lane = gid % kResGroup;
  if (qp >= a.batch) return;
  const int N = a.N, nx = a.nx, nu = a.nu;
  const bool smaj = a.layout == 1;
  auto at = [&](const real* base, int nstage, size_t blk, int k) -> const real* {
    return smaj ? base + ((size_t)k * a.batch + qp) * blk : base + ((size_t)qp * nstage + k) * blk;
  };
  const size_t nxx = (size_t)nx * nx, nxu = (size_t)nx * nu, nuu = (size_t)nu * nu;
  const real* x = a.x + (size_t)qp * (N + 1) * nx;
  const real* u = a.u + (size_t)qp * N * nu;
  const real* pi = a.pi + (size_t)qp * (N + 1) * nx;
  auto upd = [](real& m, real v) {
    v = v < real(0) ? -v : v;
    if (v > m || v != v) m = v;  // NaN propagates
  };
  real mg = real(0), mb = real(0), ob = real(0);
  for (int k = lane; k <= N; k += kResGroup) {
    const real* xk = x + (size_t)k * nx;
    const real* Q = at(a.Q, N + 1, nxx, k);
    const real* q = at(a.q, N + 1, nx, k);
    real Sx[12];
    for (int i = 0; i < 12; ++i) Sx[i] = real(0);
    if (k < N) {
      const real* uk = u + (size_t)k * nu;
      const real* xn = x + (size_t)(k + 1) * nx;
      const real* pn = pi + (size_t)(k + 1) * nx;
      const real* A = at(a.A, N, nxx, k);
      const real* B = at(a.B, N, nxu, k);
      const real* b = at(a.b, N, nx, k);
      const real* S = at(a.S, N, nxu, k);
      const real* R = at(a.R, N, nuu, k);
      const real* r = at(a.r, N, nu, k);
      for (int i = 0; i < nu; ++i) {  // column-major blocks: M[i][j] = M[j * rows + i]
        real ru = real(0), sx = real(0), bp = real(0);
        for (int j = 0; j < nu; ++j) ru += R[(size_t)j * nu + i] * uk[j];
        for (int j = 0; j < nx; ++j) sx += S[(size_t)j * nu + i] * xk[j];
        for (int j = 0; j < nx; ++j) bp += B[(size_t)i * nx + j] * pn[j];
        Sx[i] = sx;
        upd(mg, ru + sx + r[i] + bp);
        ob += uk[i] * (real(0.5) * ru + r[i]) + (k == 0 ? uk[i] * sx : real(0));
      }
      for (int i = 0; i < nx; ++i) {
        real v = b[i] - xn[i];
        for (int j = 0; j < nx; ++j) v += A[(size_t)j * nx + i] * xk[j];
        for (int j = 0; j < nu; ++j) v += B[(size_t)j * nx + i] * uk[j];
        upd(mb, v);
      }
    }
    if (k > 0) {
      const real* uk = u + (size_t)k * nu;
      const real* pn = pi + (size_t)(k + 1) * nx;
      const real* A = k < N ? at(a.A, N, nxx, k) : nullptr;
      const real* S = k < N ? at(a.S, N, nxu, k) : nullptr;
      for (int i = 0; i < nx; ++i) {
        real qx = real(0), g = q[i] - pi[(size_t)k * nx + i];
        for (int j = 0; j < nx; ++j) qx += Q[(size_t)j * nx + i] * xk[j];
        g += qx;
        if (k < N) {
          for (int j = 0; j < nu; ++j) g += S[(size_t)i * nu + j] * uk[j];
          for (int j = 0; j < nx; ++j) g += A[(size_t)i * nx + j] * pn[j];
        }
        upd(mg, g);
        ob += xk[i] * (real(0.5) * qx + q[i]);
      }
      if (k < N)
        for (int i = 0; i < nu; ++i) ob += uk[i] * Sx[i];
    }
  }
  for (int m = kResGroup / 2; m >= 1; m >>= 1) {
    const real og = __shfl_xor(mg, m, kResGroup), obb = __shfl_xor(mb, m, kResGroup);
    if (og > mg || og != og) mg = og;
    if (obb > mb || obb != obb) mb = obb;
    ob += __shfl_xor(ob, m, kResGroup);
  }
  if (lane == 0) {
    if (a.res) {
      a.res[(size_t)qp * 4 + 0] = mg;
      a.res[(size_t)qp * 4 + 1] = mb;
      a.res[(size_t)qp * 4 + 2] = real(0);
      a.res[(size_t)qp * 4 + 3] = real(0);
    }
    if (a.obj) a.obj[qp] = ob;
    if (a.stat) {  // row 0 (iteration 0): mu = 0, res_stat, res_eq, res_ineq, res_comp, obj
      real* row = a.stat + (size_t)qp * a.stat_rows * kStatCols;
      row[6] = mg;
      row[7] = mb;
      row[10] = ob;
    }
    if (a.status && (mg != mg || mb != mb)) a.status[qp] = 3;  // NaNDetected
  }
}

hipError_t launch_residuals(const ProblemArgsT<real>& a, hipStream_t stream) {
  if (a.batch <= 0) return hipSuccess;
  const long long n = (long long)a.batch * kResGroup;
  hipLaunchKernelGGL(unconstr_residuals_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     stream, a);
  return hipGetLastError();
}

hipError_t launch(const ProblemArgsT<real>& a, hipStream_t stream) {
  if (a.batch <= 0) return hipSuccess;
  const int threads = 256;
  const long long lanes = (long long)a.batch * kGroup;
  const int blocks = (int)((lanes + threads - 1) / threads);
  // 12 x 12 stages only: smaller problems arrive embedded by pad.hip
  if (a.nx != 12 || a.nu != 12) return hipErrorInvalidValue;
#ifndef SRBD_UNC_DYN_LDS
#define SRBD_UNC_DYN_LDS 0
#endif
  // (A/B knob) dynamic LDS the kernel does not use, to cap workgroups per CU
  hipLaunchKernelGGL(riccati_unconstr_kernel<true>, dim3(blocks), dim3(threads), SRBD_UNC_DYN_LDS, stream, a);
  return hipGetLastError();
}

}  // namespace SRBD_NS
}  // namespace srbd
