// riccati.h -- per-stage Riccati building blocks on a 16-lane QP group.
//
// Math (classical Riccati, ric_alg = 0, as pinned by the reference test
// hpipm-cpp/test/ocp_qp_ipm_solver.cpp:67-90, with p = -s):
//   WB = P B,  G = R + B'WB,  L = chol(G + reg I)
//   W  = P [A | b] + [0 | p]
//   H  = S + B'W_A,  g = r + B'w,  F = Q + A'W_A,  f = q + A'w
//   Y  = L^-1 H,  y = L^-1 g,  K = -L^-T Y,  k = -L^-T y
//   P- = F - Y'Y,  p- = f - Y'y
// (the forward passes step x+ = A x + B u + b with the QP's own blocks)
// This is HPIPM's d_ocp_qp_fact_solve_kkt_unconstr (hpipm_d_ocp_qp_kkt.h:54)
// i.e. the BLASFEO dgemm_nt / dsyrk_ln / dpotrf_l / dtrsv chain, re-blocked
// for one-column-per-lane.  A non-positive pivot zeroes its direction like
// BLASFEO's dpotrf_l instead of producing NaN.
//
// Square-root Riccati (ric_alg = 1, hpipm-cpp's default,
// ocp_qp_ipm_solver_settings.hpp:81; HPIPM's square_root_alg): the cost-to-go
// travels as its Cholesky factor, P = Lp Lp', p = Lp s, so every Hessian term of
// the stage is a sum of squares (riccati_step_sqrt below).
//
// The phases are ordered to keep the live register set at ~6 column arrays
// (the arch-VGPR file is 256 x 32 bit per lane = 128 doubles): P is
// broadcast twice (for WB, then for W) and B twice (for G, then for H)
// rather than holding WA, WB, G, H and F at once.
//
// Register conventions inside a group (lane l, VL = 15):
//   P[i]  : lane l < 12 -> P[i][l] (= P[l][i]); VL -> p[i]
//           (square root: lane l -> Lp[i][l], zero above the diagonal; VL -> s[i])
//   A_[i] : lane l < 12 -> A[i][l];             VL -> b[i]
//   B_[i] : lane l < 12 -> B[i][l]              (VL: zeros)
//   Rc[i] : R[i][l];  Sc[i]: S[i][l] (VL: r[i]);  Qc[i]: Q[i][l] (VL: q[i])
#pragma once

#include "qp_group.h"

// Keeps the machine scheduler from hoisting one phase's broadcasts/loads into
// the previous phase (which blows the 256-VGPR budget).
#define SRBD_PHASE_FENCE() __builtin_amdgcn_sched_barrier(0)

namespace srbd {

// Diagnostic phase timestamps (builds with -DSRBD_TSTAMP=1 only, read back by
// srbd_qp_diag_tstamps in such a build): lane 0 of workgroup 0 appends (id, cycle counter)
// at the phase boundaries of a stage -- the critical path of a single-QP solve.
#ifndef SRBD_TSTAMP
#define SRBD_TSTAMP 0
#endif
constexpr int kTstampCap = 4096;
#if SRBD_TSTAMP
static __device__ unsigned long long g_tstamp[2 * kTstampCap];
static __device__ unsigned int g_tstamp_n;
#endif
__device__ __forceinline__ void tstamp(int id) {
#if SRBD_TSTAMP
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const unsigned i = g_tstamp_n;
    if (i < kTstampCap) {
      g_tstamp[2 * i] = (unsigned long long)id;
      g_tstamp[2 * i + 1] = __builtin_readcyclecounter();
      g_tstamp_n = i + 1;
    }
  }
#else
  (void)id;
#endif
}

// C[:,l] += P M[:,l]: P symmetric & column-owned, M column-owned (fused
// v_fmac_*_dpp blocks of qp_group.h: the broadcast rides on the FMA).
template <typename T>
__device__ __forceinline__ void sym_mul_col(const T (&P)[12], const T (&M)[12], T (&C)[12]) {
  sfor<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    fma_bcast_src<K>(C, P, M[K]);
  });
}

// C[i][l] += X[:,i]' Y[:,l] for i < 12 (X, Y column-owned)
template <typename T>
__device__ __forceinline__ void tmul_acc(const T (&X)[12], const T (&Y)[12], T (&C)[12]) {
  sfor<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    fma_bcast_lanes(C, X[K], Y[K]);
  });
}

// A triangular solve applies a diagonal entry of L as rs = 1 / L_ll (0 for a zeroed pivot).
template <typename T>
__device__ __forceinline__ T apply_rs(T x, T rs) {
  return x * rs;
}
// rs of a pivot d (> 0, else the zeroed direction) and 1 / L_ll for scaling L's column
template <typename T>
__device__ __forceinline__ void pivot_rs(T d, T& rs, T& inv_l) {
  rs = d > T(0) ? T(1) / __builtin_sqrt(d) : T(0);
  inv_l = rs;
}

// Right-looking Cholesky of the column-owned symmetric G (lane l holds
// G[:,l]); `reg` is added to each pivot.  On exit Lc holds column l of L
// (rows > l meaningful) and rs = 1 / L[l][l] (0 for a non-positive pivot).
// A lane past the last column (VL) is eliminated as a border column: with G
// holding a vector v there, Lc[i] * bc<i>(rs) = (L^-1 v)[i] on exit.
template <typename T>
__device__ __forceinline__ void chol_cols(T (&G)[12], const int lane, const T reg, T (&Lc)[12],
                                          T& rs) {
  T dmine = T(1);
  sfor<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    const T dk = bc<K>(G[K]) + reg;
    const T inv = dk > T(0) ? T(1) / dk : T(0);
    const T s = lane > K ? G[K] * inv : T(0);
    sfor<K + 1, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      G[I] = fmadd(-bc<K>(G[I]), s, G[I]);
    });
    dmine = lane == K ? dk : dmine;
  });
  T inv_l;
  pivot_rs(dmine, rs, inv_l);
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    Lc[I] = G[I] * inv_l;
  });
}

// H <- L^-1 H (column-owned right-hand sides), forward substitution.
template <typename T>
__device__ __forceinline__ void trsv_lower(const T (&Lc)[12], const T rs, T (&H)[12]) {
  sfor<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    const T y = apply_rs(H[K], bc<K>(rs));
    H[K] = y;
    sfor<K + 1, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      H[I] = fmadd(-bc<K>(Lc[I]), y, H[I]);
    });
  });
}

// Kc = -L^-T y by column sweeps: for K = 11..0: z_K = y_K / L_KK, then
// y_I -= L_KI z_K for I < K (L_KI = lane I's column, row K): 12 independent
// updates per step instead of a serial dot-product chain.  y is kept.
template <typename T>
__device__ __forceinline__ void trsv_upper_t_neg_axpy(const T (&Lc)[12], const T rs,
                                                      const T (&y)[12], T (&Kc)[12]) {
  T w[12];
  sfor<0, 12>([&](auto i) { w[decltype(i)::value] = y[decltype(i)::value]; });
  sfor_down<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    w[K] = apply_rs(w[K], bc<K>(rs));
    const T nz = -w[K];
    sfor<0, K>([&](auto i) {
      constexpr int I = decltype(i)::value;
      w[I] = fmadd(bc<I>(Lc[K]), nz, w[I]);
    });
  });
  sfor<0, 12>([&](auto i) { Kc[decltype(i)::value] = -w[decltype(i)::value]; });
}

template <typename T>
struct StageFactor {
  T F[12];   // on exit: P_k column (VL: p_k)
  T H[12];   // on exit: Y = L^-1 H column (VL: y)
  T Lc[12];  // L column (rows > l meaningful)
  T rs;      // 1 / L[l][l]
  T Kc[12];  // K column (VL: k)
};

template <typename TO, typename TI>
__device__ __forceinline__ void convert12(const TI (&in)[12], TO (&out)[12]) {
  sfor<0, 12>([&](auto i) { out[decltype(i)::value] = TO(in[decltype(i)::value]); });
}

// G (in TG) -> the stage's factor L (o.Lc, o.rs, in T).  TG = double in the fp32 IPM
// with general rows: with the friction cone's Gamma of 1e8-1e10 on active rows, R (1e-2)
// is below the fp32 rounding of D'Gamma D, and G must be formed and factorized in fp64
// to keep it; the triangular solves with the rounded factor are
// backward stable entry by entry and stay in fp32.
template <typename TG, typename T>
__device__ __forceinline__ void chol_g(TG (&G)[12], const int lane, const T reg, StageFactor<T>& o) {
  if constexpr (std::is_same_v<TG, T>) {
    chol_cols(G, lane, reg, o.Lc, o.rs);
  } else {
    TG rsg;
    chol_cols(G, lane, TG(reg), G, rsg);  // (in place)
    convert12(G, o.Lc);
    o.rs = T(rsg);
  }
}

// C += X'Y with C in TG and X, Y in T (widened first when the precisions differ)
template <typename TG, typename T>
__device__ __forceinline__ void tmul_acc_g(const T (&X)[12], const T (&Y)[12], TG (&C)[12]) {
  if constexpr (std::is_same_v<TG, T>) {
    tmul_acc(X, Y, C);
  } else {
    sfor<0, 12>([&](auto kk) {
      constexpr int K = decltype(kk)::value;
      fma_bcast_lanes(C, TG(X[K]), TG(Y[K]));
    });
  }
}

struct NoMid {
  __device__ __forceinline__ void operator()() const {}
};

// Column-owned M (lane l holds M[:, l]) made exactly symmetric from its lower triangle:
// lane l's entries above the diagonal (rows I < l) are replaced by lane I's entry of row l
// (only lanes J > I change M[I], so no source is overwritten before it is read).
template <typename T>
__device__ __forceinline__ void symmetrize_lower(T (&M)[12], const int lane) {
  sfor<1, 12>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    sfor<0, J>([&](auto ii) {
      constexpr int I = decltype(ii)::value;
      const T v = bc<I>(M[J]);
      M[I] = lane == J ? v : M[I];
    });
    SRBD_PHASE_FENCE();
  });
}

// Column-owned M made exactly symmetric as (M + M')/2: the pair (I, J) of entries is
// averaged from both lanes' broadcasts, so lane J's M[I] and lane I's M[J] receive the same
// value (each pair is touched once, no source is read after it changed).
template <typename T>
__device__ __forceinline__ void symmetrize_avg(T (&M)[12], const int lane) {
  sfor<1, 12>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    sfor<0, J>([&](auto ii) {
      constexpr int I = decltype(ii)::value;
      const T lo = bc<I>(M[J]);  // M[J][I] (lane I's column, row J)
      const T up = bc<J>(M[I]);  // M[I][J]
      const T v = T(0.5) * (lo + up);
      M[I] = lane == J ? v : M[I];
      M[J] = lane == I ? v : M[J];
    });
    SRBD_PHASE_FENCE();
  });
}


// The common tail of both step variants: given L = chol(G) and the column-owned
// H (VL: g) and F (VL: f) of the stage,
//   Y = L^-1 H, K = -L^-T Y, P_k = F - Y'Y (VL: p_k = f - Y'y).
// `mid` runs before the triangular solves (MidAt = 1) or after them (MidAt = 2).
// SYMP (the IPM's factorizations): P_k leaves exactly symmetric.  The stage record keeps P's
// lower triangle only, and with the IPM's barrier Hessians of ~1e12 the next stage's
// factorization (register P) and the sweeps that read the record P then solve systems that
// differ far above the factorization's own error.  fp64: P_k in the textbook form F + K'H
// (VL: f + K'g, as the oracle's riccati_factor / riccati_vectors form it), averaged with its
// transpose.  Of the forms measured on the degenerate endgame family of DESIGN.md 4.4 (Speed,
// 64 copies, ric_alg 0) F - Y'Y with its lower triangle converged on 58, F - Y'Y averaged on
// 62, F + K'H with its lower triangle on 49 and F + K'H averaged on 64 (the oracle's 63-64).
// H waits for the product in `hstash` (12 reals per lane, e.g. the caller's dead LDS block) or
// in registers.  fp32 (the config-5 kernels, at fp32 tolerances): F - Y'Y, lower triangle
// copied up (the fp64 form measured +0.8% on config 5 for no change in its iterates' reach).
template <int MidAt, bool SYMP, typename T, typename Mid>
__device__ __forceinline__ void riccati_tail(const int lane, StageFactor<T>& o, Mid&& mid, T* hstash) {
  if constexpr (MidAt == 1) {
    mid();
    SRBD_PHASE_FENCE();
  }
  constexpr bool kHK = SYMP && sizeof(T) == 8;
  T Hs[kHK ? 12 : 1];
  if constexpr (kHK) {
    if (hstash) {
      store12(hstash, o.H);
    } else {
      sfor<0, 12>([&](auto i) { Hs[decltype(i)::value] = o.H[decltype(i)::value]; });
    }
  }
  // ---- Y = L^-1 H, K = -L^-T Y
  trsv_lower(o.Lc, o.rs, o.H);
  SRBD_PHASE_FENCE();
  tstamp(7);
  launder(o.Lc);
  trsv_upper_t_neg_axpy(o.Lc, o.rs, o.H, o.Kc);
  SRBD_PHASE_FENCE();
  tstamp(8);
  if constexpr (MidAt == 2) {
    mid();
    SRBD_PHASE_FENCE();
  }
  if constexpr (kHK) {
    // ---- P_k = F + K'H (VL: p_k = f + K'g), averaged with its transpose
    if (hstash) load12(hstash, Hs);
    tmul_acc(o.Kc, Hs, o.F);
    SRBD_PHASE_FENCE();
    symmetrize_avg(o.F, lane);
  } else {
    // ---- P_k = F - Y'Y (VL: p_k = f - Y'y)
    T Hn[12];
    sfor<0, 12>([&](auto i) { Hn[decltype(i)::value] = -o.H[decltype(i)::value]; });
    tmul_acc(o.H, Hn, o.F);
    if constexpr (SYMP) {
      SRBD_PHASE_FENCE();
      symmetrize_lower(o.F, lane);
    }
  }
  SRBD_PHASE_FENCE();
  tstamp(9);
  tstamp(10);
}

// One backward Riccati step.  `P` holds P_{k+1} (VL: p_{k+1}) on entry.
// The S/Q/R columns are fetched through the callables so that their loads
// are issued late (short live ranges).
// `mid` runs between the products and the triangular solves (MidAt = 1: P is
// dead there) or after the solves (MidAt = 2: L is dead too): the caller may
// issue the next stage's loads into registers of its own.
template <int MidAt = 1, bool SYMP = false, typename TGin = void, typename T, typename LoadR,
          typename LoadSQ, typename Mid = NoMid>
__device__ __forceinline__ void riccati_step(const T (&P)[12], T (&A_)[12], T (&B_)[12],
                                             LoadR&& loadR, LoadSQ&& loadSQ, const int lane,
                                             const T reg, StageFactor<T>& o, Mid&& mid = Mid{},
                                             T* hstash = nullptr) {
  using TG = std::conditional_t<std::is_void_v<TGin>, T, TGin>;
  const bool isv = lane == kVecLane;
  // ---- G = R + B'(P B), L = chol(G)  (loadR fills a TG column)
  {
    T WB[12];
    sfor<0, 12>([&](auto i) { WB[decltype(i)::value] = T(0); });
    sym_mul_col(P, B_, WB);
    SRBD_PHASE_FENCE();
    tstamp(1);
    TG G[12];
    loadR(G);
    tmul_acc_g(B_, WB, G);
    SRBD_PHASE_FENCE();
    tstamp(2);
    chol_g(G, lane, reg, o);
  }
  SRBD_PHASE_FENCE();
  tstamp(3);
  // ---- W = P [A | b] (+ p on VL); H = S + B'W; F = Q + A'W
  {
    T Pl[12], Bl[12];
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      Pl[I] = P[I];
      Bl[I] = B_[I];
    });
    launder(Pl);
    launder(Bl);
    T W[12];
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      W[I] = isv ? Pl[I] : T(0);
    });
    sym_mul_col(Pl, A_, W);
    SRBD_PHASE_FENCE();
    tstamp(4);
    loadSQ(o.H, o.F);
    tmul_acc(Bl, W, o.H);
    SRBD_PHASE_FENCE();
    tstamp(5);
    tmul_acc(A_, W, o.F);
  }
  SRBD_PHASE_FENCE();
  tstamp(6);
  riccati_tail<MidAt, SYMP>(lane, o, mid, hstash);
}

// Square-root step (ric_alg = 1).  `Lp` holds the factor of P_{k+1} (lane l: column l,
// zero above the diagonal; VL: s_{k+1} with p_{k+1} = Lp s_{k+1}) on entry:
//   MB = Lp'B,  MA = Lp'A,  m = Lp'b + s
//   G = R + MB'MB,  H = S + MB'MA,  F = Q + MA'MA,  g = r + MB'm,  f = q + MA'm
// -- in exact arithmetic the classical B'PB, B'PA, A'PA, B'(Pb + p), A'(Pb + p) --
// then the common tail.  The caller continues the recursion with sqrt_factor(P_k).
template <int MidAt = 1, bool SYMP = false, typename TGin = void, typename T, typename LoadR,
          typename LoadSQ, typename Mid = NoMid>
__device__ __forceinline__ void riccati_step_sqrt(const T (&Lp)[12], T (&A_)[12], T (&B_)[12],
                                                  LoadR&& loadR, LoadSQ&& loadSQ, const int lane,
                                                  const T reg, StageFactor<T>& o,
                                                  Mid&& mid = Mid{}, T* hstash = nullptr) {
  using TG = std::conditional_t<std::is_void_v<TGin>, T, TGin>;
  const bool isv = lane == kVecLane;
  // ---- MB = Lp'B (VL: 0, its B_ column is 0); G = R + MB'MB, L = chol(G)
  T MB[12];
  sfor<0, 12>([&](auto i) { MB[decltype(i)::value] = T(0); });
  tmul_acc(Lp, B_, MB);
  SRBD_PHASE_FENCE();
  {
    TG G[12];
    loadR(G);
    tmul_acc_g(MB, MB, G);
    SRBD_PHASE_FENCE();
    chol_g(G, lane, reg, o);
  }
  SRBD_PHASE_FENCE();
  // ---- MA = Lp'[A | b] + [0 | s]; H = S + MB'MA; F = Q + MA'MA
  {
    T MA[12];
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      MA[I] = isv ? Lp[I] : T(0);
    });
    tmul_acc(Lp, A_, MA);
    SRBD_PHASE_FENCE();
    loadSQ(o.H, o.F);
    tmul_acc(MB, MA, o.H);
    SRBD_PHASE_FENCE();
    tmul_acc(MA, MA, o.F);
  }
  SRBD_PHASE_FENCE();
  riccati_tail<MidAt, SYMP>(lane, o, mid, hstash);
}

// ---------------------------------------------------------------------------
// HPIPM's LQ factorization of the stage (lq_fact, hpipm_d_ocp_qp_ipm.h:78; its
// d_ocp_qp_fact_lq_solve_kkt_step, hpipm_d_ocp_qp_kkt.h:58, restated): the stage factor
// L = [Lu 0; Lxu Lx] (24 x 24, [u; x] order) is updated by Householder reflections from the
// right that absorb dense columns, L L' <- L L' + [Au; Ax][Au; Ax]', without ever forming
// the product (the barrier Hessians of ~1e13 never meet the O(1) data in a sum).
// Row-owned: lane j < 12 holds u-row j (Lu row j, entries 0..j) and x-row j (Lxu row j; Lx
// row j, entries 0..j) of L and the two rows' entries of the 12 columns being absorbed.
// One reflection per row i = 0..23 maps row i's entries (pivot, its 12 column entries) to
// (||.||, 0, ..., 0) with a positive diagonal (LAPACK dlarfgp's choice, BLASFEO dgelqf_pd);
// the pivot row is broadcast to the group, every row below it updated.  Lanes 12..15 hold
// zeros throughout.
template <typename T>
struct LqRows {
  T Lu[12], Lxu[12], Lx[12];
};

// reflection data of a pivot row held by lane I: alpha = its diagonal, sigma = its squared
// column entries; returns false when the row has nothing to absorb (a negative diagonal is
// then flipped by the caller, as dlarfgp returns beta >= 0)
template <int I, typename T>
__device__ __forceinline__ bool lq_reflector(T al_own, T sig_own, T& nrm, T& v0, T& inv) {
  const T al = bc<I>(al_own), sig = bc<I>(sig_own);
  if (!(sig > T(0))) {
    nrm = al;
    return false;
  }
  nrm = __builtin_sqrt(al * al + sig);
  v0 = al <= T(0) ? al - nrm : -sig / (al + nrm);
  inv = T(2) / (v0 * v0 + sig);
  return true;
}

template <typename T>
__device__ __forceinline__ void lq_absorb(LqRows<T>& L, T (&Au)[12], T (&Ax)[12], const int lane) {
  // ---- u rows (pivot row I on lane I, column I) ----
  sfor<0, 12>([&](auto ii) {
    constexpr int I = decltype(ii)::value;
    T sig = T(0);
    sfor<0, 12>([&](auto c) { sig = fmadd(Au[decltype(c)::value], Au[decltype(c)::value], sig); });
    T nrm, v0, inv;
    if (lq_reflector<I>(L.Lu[I], sig, nrm, v0, inv)) {
      T vb[12];
      sfor<0, 12>([&](auto c) { vb[decltype(c)::value] = bc<I>(Au[decltype(c)::value]); });
      T du = L.Lu[I] * v0, dx = L.Lxu[I] * v0;
      sfor<0, 12>([&](auto c) {
        constexpr int C = decltype(c)::value;
        du = fmadd(Au[C], vb[C], du);
        dx = fmadd(Ax[C], vb[C], dx);
      });
      const T fu = lane > I ? du * inv : T(0);  // u rows below the pivot
      const T fx = dx * inv;                    // every x row
      L.Lu[I] = fmadd(-fu, v0, L.Lu[I]);
      L.Lxu[I] = fmadd(-fx, v0, L.Lxu[I]);
      sfor<0, 12>([&](auto c) {
        constexpr int C = decltype(c)::value;
        Au[C] = fmadd(-fu, vb[C], Au[C]);
        Ax[C] = fmadd(-fx, vb[C], Ax[C]);
      });
      if (lane == I) {
        L.Lu[I] = nrm;
        sfor<0, 12>([&](auto c) { Au[decltype(c)::value] = T(0); });
      }
    } else if (nrm < T(0)) {  // nothing to absorb, negative diagonal: flip column I
      if (lane >= I) L.Lu[I] = -L.Lu[I];
      L.Lxu[I] = -L.Lxu[I];
    }
    SRBD_PHASE_FENCE();
  });
  // ---- x rows (pivot row 12 + I on lane I, column 12 + I; the u rows are done) ----
  sfor<0, 12>([&](auto ii) {
    constexpr int I = decltype(ii)::value;
    T sig = T(0);
    sfor<0, 12>([&](auto c) { sig = fmadd(Ax[decltype(c)::value], Ax[decltype(c)::value], sig); });
    T nrm, v0, inv;
    if (lq_reflector<I>(L.Lx[I], sig, nrm, v0, inv)) {
      T vb[12];
      sfor<0, 12>([&](auto c) { vb[decltype(c)::value] = bc<I>(Ax[decltype(c)::value]); });
      T dx = L.Lx[I] * v0;
      sfor<0, 12>([&](auto c) { dx = fmadd(Ax[decltype(c)::value], vb[decltype(c)::value], dx); });
      const T fx = lane > I ? dx * inv : T(0);
      L.Lx[I] = fmadd(-fx, v0, L.Lx[I]);
      sfor<0, 12>([&](auto c) { Ax[decltype(c)::value] = fmadd(-fx, vb[decltype(c)::value], Ax[decltype(c)::value]); });
      if (lane == I) {
        L.Lx[I] = nrm;
        sfor<0, 12>([&](auto c) { Ax[decltype(c)::value] = T(0); });
      }
    } else if (nrm < T(0)) {
      if (lane >= I) L.Lx[I] = -L.Lx[I];
    }
    SRBD_PHASE_FENCE();
  });
}

// Transpose of a 12 x 12 block between row- and column-owned through the group's LDS block
// `blk` (144 reals): lane j's v (a row or a column) in, lane j's transposed vector out.
// `keep` masks the result to entries I >= lane (lower: column-owned from row-owned) or I <=
// lane (rows from a column-owned lower factor), 0 = full.
template <typename T>
__device__ __forceinline__ void group_transpose(T* blk, const int lane, T (&v)[12], int keep) {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  if (lane < 12) {
    sfor<0, 6>([&](auto i) {
      constexpr int I = decltype(i)::value;
      blk[lane * 12 + 2 * I] = v[2 * I];
      blk[lane * 12 + 2 * I + 1] = v[2 * I + 1];
    });
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int r = lane < 12 ? lane : 0;
  sfor<0, 12>([&](auto j) {
    constexpr int J = decltype(j)::value;
    const T x = blk[J * 12 + r];
    const bool ok = lane < 12 && (keep > 0 ? J >= lane : keep < 0 ? J <= lane : true);
    v[J] = ok ? x : T(0);
  });
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// One backward step by LQ (lq_fact), ric_alg 1's recursion otherwise (riccati_step_sqrt):
//   Lh = chol([R~ S'; S Q~])       R~ = R + box Gamma_u (+ reg on the pivots), Q~ = Q + box Gamma_x
//   L  = LQ([Lh | [B'; A'] Lp | dense columns of `extra`])
// `loadR` / `loadSQ` fill R~ and S, Q~ (VL: r~, q~) as for riccati_step_sqrt, without the dense
// general-row terms; `extra(L, lane)` absorbs those (lq_absorb per 12-row chunk).  HPIPM keeps
// the box Gamma as a diagonal block beside Lh ([L | L | A], dgelqf_pd_lla); here it is added to
// the Hessian's diagonal before its Cholesky -- a diagonal addition, nothing can cancel -- and
// only the dense terms (the cost-to-go [B'; A'] Lp and the general rows sqrt(Gamma) [D'; C'])
// are absorbed by reflections.  On exit o holds Lu (o.Lc, o.rs), K | k (o.Kc), Y (o.H) and, on VL,
// p_k (o.F); Lp holds the next factor Lx (column-owned, zeros above the diagonal) and on VL
// s_k = Lx^-1 p_k.  `blk`: the group's 144-real LDS block (free here).
template <typename T, typename LoadR, typename LoadSQ, typename Extra>
__device__ __forceinline__ void riccati_step_lq(T (&Lp)[12], T (&A_)[12], T (&B_)[12], LoadR&& loadR,
                                                LoadSQ&& loadSQ, const int lane, const T reg,
                                                StageFactor<T>& o, T* blk, Extra&& extra) {
  const bool isv = lane == kVecLane, own = lane < kMaxDim;
  // ---- MB = Lp'B, MA = Lp'[A | b] + [0 | s] (VL: m), as riccati_step_sqrt
  T MB[12], MA[12];
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    MB[I] = T(0);
    MA[I] = isv ? Lp[I] : T(0);
  });
  tmul_acc(Lp, B_, MB);
  tmul_acc(Lp, A_, MA);
  SRBD_PHASE_FENCE();
  // ---- vectors on the element owners: g_i = (MB'm)_i, f_i = (MA'm)_i (m on VL)
  T gi = T(0), fi = T(0);
  sfor<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    const T mk = bc<kVecLane>(MA[K]);
    gi = fmadd(MB[K], mk, gi);
    fi = fmadd(MA[K], mk, fi);
  });
  SRBD_PHASE_FENCE();
  // ---- Lh: Lu_h = chol(R~), Y_h = Lu_h^-1 S, Lx_h = chol(Q~ - Y_h'Y_h)
  LqRows<T> L;
  T Sc[12], Qc[12], rs_h;
  {
    T G[12];
    loadR(G);
    chol_cols(G, lane, reg, L.Lu, rs_h);
  }
  loadSQ(Sc, Qc);  // (VL: r~, q~)
  // g_i = r~_i + (MB'm)_i, f_i = q~_i + (MA'm)_i on their element owners
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    const T r = bc<kVecLane>(Sc[I]), q = bc<kVecLane>(Qc[I]);
    if (lane == I) {
      gi += r;
      fi += q;
    }
  });
  trsv_lower(L.Lu, rs_h, Sc);  // lane l: Y_h[:, l] = row l of Lxu_h
  {
    T Yn[12];
    sfor<0, 12>([&](auto i) { Yn[decltype(i)::value] = -Sc[decltype(i)::value]; });
    tmul_acc(Sc, Yn, Qc);
  }
  T rs_x;
  chol_cols(Qc, lane, T(0), L.Lx, rs_x);
  sfor<0, 12>([&](auto i) { L.Lxu[decltype(i)::value] = own ? Sc[decltype(i)::value] : T(0); });
  SRBD_PHASE_FENCE();
  // column-owned lower factors (rows >= l meaningful) -> rows
  group_transpose(blk, lane, L.Lu, -1);
  group_transpose(blk, lane, L.Lx, -1);
  // ---- absorb [B'; A'] Lp (u row j: MB[:, j], x row j: MA[:, j]) and the dense rows
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    if (!own) {
      MB[I] = T(0);
      MA[I] = T(0);
    }
  });
  lq_absorb(L, MB, MA, lane);
  extra(L, lane);
  SRBD_PHASE_FENCE();
  // ---- back to column-owned: Lu -> o.Lc, o.rs; Lx -> Lp (next stage); Y = Lxu rows
  group_transpose(blk, lane, L.Lu, 1);
  group_transpose(blk, lane, L.Lx, 1);
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    o.Lc[I] = L.Lu[I];
  });
  T du = T(0), dxx = T(0);
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    if (lane == I) {
      du = L.Lu[I];
      dxx = L.Lx[I];
    }
  });
  o.rs = du > T(0) ? T(1) / du : T(0);
  const T rsx = dxx > T(0) ? T(1) / dxx : T(0);
  // ---- the vectors: y = Lu^-1 g, k = -Lu^-T y, p_k = f - Y'y, s_k = Lx^-1 p_k
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    const T g = bc<I>(gi), f = bc<I>(fi);
    o.H[I] = isv ? g : T(0);
    o.F[I] = isv ? f : T(0);
  });
  trsv_lower(o.Lc, o.rs, o.H);
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    if (own) o.H[I] = L.Lxu[I];
  });
  trsv_upper_t_neg_axpy(o.Lc, o.rs, o.H, o.Kc);
  {
    T Hn[12];
    sfor<0, 12>([&](auto i) { Hn[decltype(i)::value] = -o.H[decltype(i)::value]; });
    tmul_acc(o.H, Hn, o.F);
  }
  SRBD_PHASE_FENCE();
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    Lp[I] = isv ? o.F[I] : L.Lx[I];
  });
  trsv_lower(L.Lx, rsx, Lp);  // VL: s_k = Lx^-1 p_k (the matrix lanes' results are discarded)
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    if (!isv) Lp[I] = L.Lx[I];
  });
}

// P (lane l: column l of P_k; VL: p_k) -> its square-root form for the next
// riccati_step_sqrt: Lp = chol(P) (column l, zeros above the diagonal) and, on VL,
// s = Lp^-1 p (the border column of the same elimination).  A non-positive pivot
// zeroes its column and its s entry (BLASFEO dpotrf_l), like chol_cols.
template <typename T>
__device__ __forceinline__ void sqrt_factor(T (&P)[12], const int lane) {
  T rs;
  chol_cols(P, lane, T(0), P, rs);
  const bool isv = lane == kVecLane;
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    const T ri = bc<I>(rs);
    if (isv) P[I] = apply_rs(P[I], ri);
    else if (lane > I) P[I] = T(0);
  });
}

}  // namespace srbd
