// riccati_scan_impl.h -- the unconstrained single-QP solve as a parallel-in-time Riccati
// (fp64, nx = nu = 12; included by riccati_unconstr_impl.h in SRBD_WITH_LATENCY builds).
// No include guard.
//
// The serial recursion P_k = f_k(P_{k+1}) costs one dependent Cholesky per stage; on one
// 16-lane group that chain is the whole latency of the reference's call pattern (one QP per
// solve(), NMPC_solver.cpp:316-330).  Here every stage becomes an element of
// an associative scan (the "conditional value function" form of the LQ problem):
//   e_k = (A, b, C, zeta, J):  A = A_k - B_k R_k^-1 S_k,   b = b_k - B_k R_k^-1 r_k,
//                              C = B_k R_k^-1 B_k',       J = Q_k - S_k' R_k^-1 S_k,
//                              zeta = q_k - S_k' R_k^-1 r_k;   e_N = (0, 0, 0, q_N, Q_N),
// and e_i (x) e_j, for e_i before e_j, is
//   M = I + C_i J_j,  [X1 | X2] = M^-1 [A_i | b_i - C_i zeta_j,  C_i A_j'],
//   A = A_j X1,  b = A_j X1_b + b_j,  C = A_j X2 + C_j,
//   J = J_i + X1'(J_j A_i),  zeta = zeta_i + X1'(J_j b_i + zeta_j).
// The suffix e_k (x) ... (x) e_N carries J = P_k, zeta = p_k.  With the N + 1 elements on N + 1
// groups, ceil(log2(N + 1)) rounds of pairwise combines (Hillis-Steele: group k takes
// e_k (x) e_{k+d}) replace the N dependent stages; then every stage forms its K_k, k_k and
// record from P_{k+1} at once (riccati.h riccati_step: the serial stage itself), and the
// forward sweep, the outputs and the fused residuals are those of the LDS kernels.
// In exact arithmetic this is the serial recursion; on SRBD QPs P_k, p_k agree with it to
// ~3e-15 relative (numpy check).  The combine's solve runs without pivoting:
// a pivot below 1e-3 of its column, a non-positive pivot of R, or a non-finite value sends
// the whole QP to the serial recursion (solve_qp) in the same launch.
// (Included inside namespace srbd::SRBD_NS.)

// diagnostic builds (-DSRBD_SCAN_DUMP=n, scripts/dev/scan_debug.py): 1 = the P, p outputs are
// the scan's J, zeta and K the element's A; 2 = the same without any combine round
#ifndef SRBD_SCAN_DUMP
#define SRBD_SCAN_DUMP 0
#endif


constexpr int kScanThreads = 512;                      // 32 groups: N + 1 <= 32 elements
constexpr int kScanNMax = kScanThreads / kGroup - 1;  // 31
constexpr int kScanLevels = 5;                         // ceil(log2(32))
constexpr int kScanBatchMax = 16;                      // QPs per launch (one workgroup each)
// An element in the scan buffer, column-owned as its group holds it: A's 12 columns and b,
// then C's 12 columns, then J's 12 columns and zeta (12 reals each; the vector lane's column
// in slot 12, scan_col).
constexpr int kScanElemA = 0, kScanElemC = 13 * 12, kScanElemJ = 25 * 12, kScanElem = 38 * 12;
// per QP: two buffers (the rounds alternate) of N + 1 elements
__host__ __device__ constexpr size_t scan_doubles_per_qp(int N) { return 2 * (size_t)(N + 1) * kScanElem; }

struct ScanElem {
  real A[12];  // lane l < 12: column l of A; VL: b
  real C[12];  // lane l < 12: column l of C; VL: 0
  real J[12];  // lane l < 12: column l of J; VL: zeta
};

__device__ __forceinline__ real* scan_slot(const ProblemArgsT<real>& a, int qp, int buf, int k) {
  return a.scan + (((size_t)qp * 2 + buf) * (size_t)(a.N + 1) + (size_t)k) * kScanElem;
}

// an element's column slot of a lane: column l on lane l < 12, the vector column (b, zeta) of
// the vector lane (kVecLane) in slot 12; the other lanes have none (-1)
__device__ __forceinline__ int scan_col(int lane) {
  return lane < kMaxDim ? lane : (lane == kVecLane ? kMaxDim : -1);
}

__device__ __forceinline__ void scan_put(real* e, int lane, const ScanElem& s) {
  const int c = scan_col(lane);
  if (c >= 0) {
    store12(e + kScanElemA + c * 12, s.A);
    store12(e + kScanElemJ + c * 12, s.J);
  }
  if (lane < kMaxDim) store12(e + kScanElemC + lane * 12, s.C);
}

// An opaque copy of a pointer, ordered after the asm blocks issued before it: the loads through
// it cannot be hoisted above the phase that precedes them (hoisted, every operand of the
// combine would be live at once and spill)
template <typename P>
__device__ __forceinline__ P* opq(P* p) {
  unsigned long long v = reinterpret_cast<unsigned long long>(p);
  asm volatile("" : "+v"(v));
  return reinterpret_cast<P*>(v);
}

// Elements written by other waves of the workgroup are read past the CU's vector L1 (agent-scope
// loads: L2-coherent); the writers publish them with __threadfence() before the barrier.  (An
// L1 line filled by an earlier round's read of the same slot would otherwise serve stale data.)
__device__ __forceinline__ void load12_l2(const real* p, real (&v)[12]) {
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    v[I] = __hip_atomic_load(p + I, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  });
}
__device__ __forceinline__ real load_l2(const real* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void zero12(real (&v)[12]) {
  sfor<0, 12>([&](auto i) { v[decltype(i)::value] = real(0); });
}

// M X = [R1 | R2] for the 12 x 12 M (column l on lane l < 12) and right-hand sides column-owned
// (R1 on lanes <= 12, R2 on lanes < 12; other lanes carry zeros): Gaussian elimination without
// pivoting, then back substitution, each lane on its own columns.  `bad` is set on the lane
// owning a pivot smaller than 1e-3 of its column's remaining entries (or not finite).
__device__ __forceinline__ void scan_solve(real (&M)[12], real (&R1)[12], real (&R2)[12], const int lane,
                                           bool& bad) {
  sfor<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    if (lane == K) {
      real cmax = real(0);
      sfor<K, 12>([&](auto i) { cmax = fmax(cmax, fabs(M[decltype(i)::value])); });
      const real p = fabs(M[K]);
      bad |= !(p >= real(1e-3) * cmax) || !(cmax < real(1e300));
    }
    const real inv = lat_recip(bc<K>(M[K]));
    const real sm = M[K] * inv, s1 = R1[K] * inv, s2 = R2[K] * inv;
    sfor<K + 1, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      const real mik = bc<K>(M[I]);  // M[I][K], read before any lane updates its M[I]
      R1[I] = fmadd(-mik, s1, R1[I]);
      R2[I] = fmadd(-mik, s2, R2[I]);
      M[I] = fmadd(-mik, sm, M[I]);
    });
    SRBD_PHASE_FENCE();
  });
  sfor_down<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    const real inv = lat_recip(bc<K>(M[K]));  // 1 / U[K][K] (the pivot above, recomputed)
    R1[K] *= inv;
    R2[K] *= inv;
    sfor<0, K>([&](auto i) {
      constexpr int I = decltype(i)::value;
      const real uik = bc<K>(M[I]);  // U[I][K]
      R1[I] = fmadd(-uik, R1[K], R1[I]);
      R2[I] = fmadd(-uik, R2[K], R2[I]);
    });
    SRBD_PHASE_FENCE();
  });
}

// e (group i, registers) <- e (x) e_j (scan buffer `ej`)
__device__ __forceinline__ void scan_combine(ScanElem& e, const real* ej, const int lane, bool& bad) {
  const bool own = lane < kMaxDim, isv = lane == kVecLane;
  real M[12], T[12], R1[12], R2[12];
  {
    // J_j with zeta_j on VL
    real Jj[12];
    if (own || isv) {
      load12_l2(opq(ej) + kScanElemJ + scan_col(lane) * 12, Jj);
    } else {
      zero12(Jj);
    }
    // M = I + C_i J_j (lanes < 12); VL: C_i zeta_j
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      M[I] = lane == I ? real(1) : real(0);
    });
    sym_mul_col(e.C, Jj, M);
    // T = J_j [A_i | b_i] + [0 | zeta_j]
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      T[I] = isv ? Jj[I] : real(0);
    });
    sym_mul_col(Jj, e.A, T);
  }
  // R1 = [A_i | b_i - C_i zeta_j]; the VL's M is not a column of M
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    R1[I] = isv ? e.A[I] - M[I] : (own ? e.A[I] : real(0));
    if (!own) M[I] = real(0);
  });
  SRBD_PHASE_FENCE();
  {
    // R2 = C_i A_j' (lane l: C_i times row l of A_j)
    real Ar[12];
    const real* ea = opq(ej);
    sfor<0, 12>([&](auto m) {
      constexpr int Mi = decltype(m)::value;
      Ar[Mi] = own ? load_l2(ea + kScanElemA + Mi * 12 + lane) : real(0);
    });
    zero12(R2);
    sym_mul_col(e.C, Ar, R2);
  }
  SRBD_PHASE_FENCE();
  scan_solve(M, R1, R2, lane, bad);  // R1 <- X1 = [X_A | X_b], R2 <- X2
  SRBD_PHASE_FENCE();
  // J = J_i + X_A' T (VL: zeta_i + X_A' T_VL), made exactly symmetric
  tmul_acc(R1, T, e.J);
  symmetrize_avg(e.J, lane);
  SRBD_PHASE_FENCE();
  {
    real Aj[12];
    if (own || isv) {
      load12_l2(opq(ej) + kScanElemA + scan_col(lane) * 12, Aj);
    } else {
      zero12(Aj);
    }
    // A = A_j X1 + [0 | b_j]
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      e.A[I] = isv ? Aj[I] : real(0);  // (VL: b_j)
    });
    sym_mul_col(Aj, R1, e.A);
    // C = A_j X2 + C_j, made exactly symmetric
    if (own) {
      load12_l2(opq(ej) + kScanElemC + lane * 12, e.C);
    } else {
      zero12(e.C);
    }
    sym_mul_col(Aj, R2, e.C);
    symmetrize_avg(e.C, lane);
  }
  sfor<0, 12>([&](auto i) { bad |= (lane <= kVecLane) && !(fabs(e.J[decltype(i)::value]) < real(1e300)); });
}

// the element of stage k (< N) from its QP blocks in the LDS image
__device__ __forceinline__ void scan_element(const LdsSrc& src, int k, const int lane, ScanElem& e, bool& bad) {
  const bool own = lane < kMaxDim, isv = lane == kVecLane;
  const int col = own ? lane : kMaxDim - 1;
  // L = chol(R) (no regularization: R must be positive definite here)
  real Rc[12], Lc[12], rs;
  if (own) {
    load12(src.R(k) + col * 12, Rc);
  } else {
    zero12(Rc);
  }
  chol_cols(Rc, lane, real(0), Lc, rs);
  if (own) bad |= !(rs > real(0)) || !(rs < real(1e150));
  // V = L^-1 S (VL: w = L^-1 r), Y = L^-1 B' (lane l: row l of B)
  real V[12], Y[12];
  if (own) {
    load12(src.S(k) + col * 12, V);
  } else if (isv) {
    load12(src.r(k), V);
  } else {
    zero12(V);
  }
  const real* Bb = src.B(k);
  sfor<0, 12>([&](auto m) {
    constexpr int Mi = decltype(m)::value;
    Y[Mi] = own ? Bb[Mi * 12 + lane] : real(0);
  });
  trsv_lower(Lc, rs, V);
  trsv_lower(Lc, rs, Y);
  real Vn[12];
  sfor<0, 12>([&](auto i) { Vn[decltype(i)::value] = -V[decltype(i)::value]; });
  // C = Y'Y;  J = Q - V'V (VL: zeta = q - V'w);  A = A - Y'V (VL: b - Y'w)
  zero12(e.C);
  tmul_acc(Y, Y, e.C);
  symmetrize_avg(e.C, lane);
  if (own) {
    load12(src.Q(k) + col * 12, e.J);
    load12(src.A(k) + col * 12, e.A);
  } else if (isv) {
    load12(src.q(k), e.J);
    load12(src.b(k), e.A);
  } else {
    zero12(e.J);
    zero12(e.A);
  }
  tmul_acc(V, Vn, e.J);
  symmetrize_avg(e.J, lane);
  tmul_acc(Y, Vn, e.A);
}

// the serial recursion on one group (the fallback), out of line: its registers are not the
// scan's
__device__ __noinline__ void scan_serial(const ProblemArgsT<real>& a, const LdsSrc& src, int qp, int lane,
                                         real* so) {
  solve_qp<false>(a, src, qp, lane, so);
}

template <bool RES>
__global__ void __launch_bounds__(kScanThreads, 1) riccati_scan_kernel(ProblemArgsT<real> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  real* img = reinterpret_cast<real*>(lds_raw);
  real* so = img + (a.N + 1) * kImgStage;
  __shared__ int fb[kScanLevels + 1];  // fallback votes, one slot per phase
  const int qp = blockIdx.x;
  const int N = a.N;
  const int g = threadIdx.x >> 4, lane = threadIdx.x & (kGroup - 1);
  const bool own = lane < kMaxDim, isv = lane == kVecLane;
  if (threadIdx.x <= kScanLevels) fb[threadIdx.x] = 0;
  lds_copy_qp<kScanThreads>(a, img, qp);  // (ends with a workgroup barrier)
  LdsSrc src{img};
  src.grec = a.ws;
  src.batch = a.batch;
  src.qp = qp;

  bool serial = false;
  int cur = 0;
  ScanElem e;
  if (g <= N) {
    bool bad = false;
    if (g < N) {
      scan_element(src, g, lane, e, bad);
    } else {  // e_N = (0, 0, 0, q_N, Q_N)
      zero12(e.A);
      zero12(e.C);
      if (own) {
        load12(src.Q(N) + lane * 12, e.J);
      } else if (isv) {
        load12(src.q(N), e.J);
      } else {
        zero12(e.J);
      }
      symmetrize_avg(e.J, lane);
    }
    if (bad) fb[0] = 1;
    scan_put(scan_slot(a, qp, 0, g), lane, e);
  }
  __threadfence();
  __syncthreads();
  serial = fb[0] != 0;
  int lev = 1;
  for (int d = 1; d <= (SRBD_SCAN_DUMP == 2 ? 0 : N) && !serial; d *= 2, ++lev) {
    if (g <= N) {
      bool bad = false;
      if (g + d <= N) scan_combine(e, scan_slot(a, qp, cur, g + d), lane, bad);
      if (bad) fb[lev] = 1;
      scan_put(scan_slot(a, qp, cur ^ 1, g), lane, e);
    }
    __threadfence();
    __syncthreads();
    cur ^= 1;
    serial = fb[lev] != 0;
  }
  if constexpr (SRBD_SCAN_DUMP != 0) {
    if (g <= N) {
      const real* en = scan_slot(a, qp, cur, g);
      real P[12];
      load12_l2(en + kScanElemJ + (isv ? kMaxDim : (own ? lane : kMaxDim - 1)) * 12, P);
      store_riccati_out(a, qp, g, lane, P, P);
      if (own && a.K && g < N) {  // K <- A of the element
        real Ae[12];
        load12_l2(en + kScanElemA + lane * 12, Ae);
        store12(a.K + ((size_t)qp * N + g) * 144 + (size_t)lane * 12, Ae);
      }
    }
    return;
  }
  if (serial) {
    // the serial recursion on group 0 (the LDS kernels' solve), nothing of the scan kept
    if (threadIdx.x < kGroup) scan_serial(a, src, qp, lane, so);
  } else {
    // every stage k < N: the serial stage from P_{k+1}, p_{k+1} (the scan's e_{k+1}): K_k, k_k,
    // the record and the Riccati outputs
    const int col = own ? lane : kMaxDim - 1;
    if (g < N) {
      const int k = g;
      const real* en = scan_slot(a, qp, cur, k + 1);
      real P[12];
      load12_l2(en + kScanElemJ + (isv ? kMaxDim : col) * 12, P);
      real A_[12], B_[12];
      if (isv) {
        load12(src.b(k), A_);
        zero12(B_);
      } else {
        load12(src.A(k) + col * 12, A_);
        load12(src.B(k) + col * 12, B_);
      }
      auto loadR = [&](real (&Rc)[12]) {
        if (isv) {
          zero12(Rc);
        } else {
          load12(src.R(k) + col * 12, Rc);
        }
      };
      auto loadSQ = [&](real (&Sc)[12], real (&Qc)[12]) {
        if (isv) {
          load12(src.r(k), Sc);
          load12(src.q(k), Qc);
        } else {
          load12(src.S(k) + col * 12, Sc);
          load12(src.Q(k) + col * 12, Qc);
        }
      };
      StageFactor<real> f;
      riccati_step<1, false>(P, A_, B_, loadR, loadSQ, lane, a.reg, f);
      store_rec(src.rec(k), lane, f.Kc, f.F);
      store_riccati_out(a, qp, k, lane, f.F, f.Kc);
    } else if (g == N) {  // terminal: P_N = Q_N, p_N = q_N
      real P[12];
      if (isv) {
        load12(src.q(N), P);
      } else {
        load12(src.Q(N) + col * 12, P);
      }
      store_rec_P(src.rec(N), lane, P);
      store_riccati_out(a, qp, N, lane, P, P);
    }
    __threadfence();
    __syncthreads();  // every record is in the workspace
    if (threadIdx.x < kGroup) fwd_sweep(a, src, qp, lane, so);
  }
  if constexpr (RES) {
    __syncthreads();  // the solution copy is complete
    ResLds acc{};
    acc.img = img;
    acc.so = so;
    acc.N = N;
    unconstr_residuals_body(a, acc, qp);
  }
}
