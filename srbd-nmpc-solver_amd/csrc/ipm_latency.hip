// ipm_latency.hip -- the box / general-constraint IPM for small batches: one workgroup per QP,
// the whole solve (init, every iteration, outputs) in one launch, the serial recursions on
// fp64 matrix cores.
//
// Same algorithm as the batched IPM (ipm_box_impl.h) and the oracle (oracle/ocp_qp_oracle.c
// oracle_solve): HPIPM's d_ocp_qp_ipm_solve (hpipm_d_ocp_qp_ipm.h:238) in the classical
// Riccati form (ric_alg 0, NMPC_solver.cpp:81), Mehrotra predictor-corrector, and HPIPM's
// iterative refinement of the step when the mode asks for it (Balance 2 / Robust 4 corrections,
// itref_corr_max; the reference test's compareResults runs Balance, test/ocp_qp_ipm_solver.cpp:243).
// Another summation order: results agree
// with the batched kernels' and the oracle's to rounding, not bit for bit.
//
// Why a separate kernel.  In the batched kernels a QP is one 16-lane group that walks its
// stages serially in every phase; for a lone QP that is a chain of 12-wide DPP products
// (RB -> F1 ~10.5 us per stage, B2 -> F2 ~4.2 us: DESIGN.md 4.9), ~2.8 ms for a box-u N = 20
// solve.  Here only what is recursive in the stage index stays serial:
//   * the factorization (backward, one stage after another) on matrix cores exactly like the
//     unconstrained single-QP kernel (riccati_latency_impl.h: wave 0 the Riccati products and
//     the Cholesky, wave 1 one stage behind with K, the record and the closed loop Acl),
//     with the predictor's right-hand side as the tiles' 13th column;
//   * the corrector's backward vector recursion, reduced to one matrix-vector product per
//     stage, p_k = Acl_k' p_k+1 + c_k with c_k = g~x + K'g~u + Acl_k' P_k+1 b~_k formed
//     for every stage at once beforehand;
//   * the forward recursions dx_k+1 = Acl_k dx_k + bcl_k (one product per stage).
// Everything else -- residuals, barrier terms, the Hessian updates, du = K dx + k, dpi, the
// step lengths and the update -- runs with one 16-lane group per stage, all stages at once.
//
// Memory: the iterate, the barrier state, the steps and the closed-loop rows in LDS; the
// barrier-augmented stage blocks (R~, S~, Q~, r~, q~, b~) and the factorization record
// (K | k rows, P, p, L) in the QP's workspace, where the next recursion reads them from L2
// one stage ahead of their use.  QP data is read where it lies (HBM / L2).
#include "kernels.h"
#include "mfma_lat.h"

// dev builds only (make variant VFLAGS=-DSRBD_LAT_SQRT_C=1): the square root with C rows here too
// (ipm_latency_ok): at -O3 that instantiation leaves the C-free one on C = 0 data, at -O1 / -O2
// it does not
#ifndef SRBD_LAT_SQRT_C
#define SRBD_LAT_SQRT_C 0
#endif



namespace srbd {
namespace ipm_lat {

constexpr int kThreads = 512;
constexpr int kGroups = kThreads / kGroup;  // one stage per 16-lane group
constexpr double kThr0 = 0.1;               // HPIPM init_var minimum slack
constexpr double kTau = 0.995;              // fraction to the boundary

// stage record in the QP's workspace (doubles); K | k rows and P, p as kernels.h kWs*
constexpr int kRK = 0, kRP = 156, kRp = 234, kRL = 246, kRrs = 324;
// the stage's barrier-augmented blocks: b~, R~, S~ (nu x nx), Q~ (column-major), r~, q~
constexpr int kRb = 336, kRR = 348, kRS = 492, kRQ = 636, kRr = 780, kRq = 792;
constexpr int kRStage = 804;
static_assert(kRStage % 2 == 0, "16-byte aligned stage records");

constexpr int kRedSlots = 8;
// general rows, per stage and 12-row chunk: bars [48], steps [48], row values [12], Gamma [12]
constexpr int kGenChunk = 120;
// the factorization's operand ring (three stages): A, B, then the record's b~ R~ S~ Q~ r~ q~
constexpr int kSA = 0, kSB = 144, kSb = 288, kSR = 300, kSS = 444, kSQ = 588, kSr = 732, kSq = 744;
constexpr int kSlot = 756;
static_assert(kSb - kSA == 2 * 144 && kRR - kRb == kSR - kSb && kRq - kRb == kSq - kSb, "ring = A, B, record blocks");

// [N+1][12] buffers before the general rows: 15 vectors, 4 x 48 barrier blocks
constexpr int kV12 = 31;
__host__ __device__ constexpr size_t lds_doubles(int N, int nch) {
  return (size_t)kV12 * (N + 1) * 12 + (size_t)nch * (N + 1) * kGenChunk + (size_t)N * 156 + 648 +
         (size_t)kGroups * kRedSlots + 3 * kSlot;
}

// Offsets, not stored pointers: every address is formed from the one __shared__ base, so the
// compiler keeps LDS accesses as ds_read / ds_write (a pointer table in memory would turn them
// into flat accesses through the stack).
struct Lds {
  double* base;
  int S;    // (N + 1) * 12
  int N, nch;
  int cur;  // which of the two x / pi buffers holds the current iterate (stage_pass writes the other)
  // [N+1][12]: iterate (x, pi double-buffered), step, residuals, corrector gradients, k and p
  __device__ double* v12(int i) const { return base + i * S; }
  __device__ double* xb(int b) const { return v12(b ? 13 : 0); }
  __device__ double* pib(int b) const { return v12(b ? 14 : 2); }
  __device__ double* x() const { return xb(cur); }
  __device__ double* pi() const { return pib(cur); }
  __device__ double* u() const { return v12(1); }
  __device__ double* dx() const { return v12(3); }
  __device__ double* du() const { return v12(4); }
  __device__ double* dpi() const { return v12(5); }
  __device__ double* rgu() const { return v12(6); }
  __device__ double* rgx() const { return v12(7); }
  __device__ double* rb() const { return v12(8); }
  __device__ double* gtu() const { return v12(9); }
  __device__ double* gtx() const { return v12(10); }
  __device__ double* kv() const { return v12(11); }
  __device__ double* pv() const { return v12(12); }
  // [N+1][48]: box barrier state of u / x (lam_l, lam_u, t_l, t_u) and its step
  // (dt_l, dt_u, dlam_l, dlam_u)
  __device__ double* bu() const { return base + 15 * S; }
  __device__ double* bx() const { return base + 19 * S; }
  __device__ double* su() const { return base + 23 * S; }
  __device__ double* sx() const { return base + 27 * S; }
  // iterative refinement (itref_corr_max) takes buffers that are dead between an iteration's
  // stage pass and the next one: the check's r_u, r_x in gtu, gtx (the corrector's gradients),
  // r_b and the correction's P_k+1 r_b in the other x / pi buffer (the next stage pass writes
  // it afresh), the correction's dx in gtu once its recursion no longer needs r_u
  __device__ int ref_b() const { return cur ? 0 : 13; }   // = xb(cur ^ 1)
  __device__ int ref_pb() const { return cur ? 2 : 14; }  // = pib(cur ^ 1)
  static constexpr int kRefDx = 9;                        // gtu
  // general rows, [N+1][nch][kGenChunk]
  __device__ double* gb(int k, int ch) const { return base + kV12 * S + (k * nch + ch) * kGenChunk; }
  __device__ double* acl() const { return base + kV12 * S + (N + 1) * nch * kGenChunk; }  // [N][156]
  // factorization hand-over: G/H tile, two Y tiles, two L factors
  __device__ double* scr() const { return acl() + N * 156; }
  __device__ double* red() const { return scr() + 648; }  // [kGroups][kRedSlots]
  __device__ double* ring() const { return red() + kGroups * kRedSlots; }  // [3][kSlot]
};

__device__ __forceinline__ Lds carve(double* base, int N, int nch) {
  Lds L;
  L.base = base;
  L.S = (N + 1) * 12;
  L.N = N;
  L.nch = nch;
  L.cur = 0;
  return L;
}

// An opaque copy of a thread index or the QP index at the top of each phase: the phases are
// inlined into one kernel loop, and without this the compiler hoists their address arithmetic
// out of the loop and keeps it live across every other phase (976 B/lane of scratch).
__device__ __forceinline__ int opq(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
// QP data (QP-major, the only layout the constrained solve takes: srbd_qp_capi.hip check_dims)
struct Qp {
  const ProblemArgsT<double>& a;
  int q, N;
  __device__ size_t qi() const { return (size_t)opq(q); }  // (opaque: see opq)
  __device__ const double* A(int k) const { return a.A + (qi() * N + k) * 144; }
  __device__ const double* B(int k) const { return a.B + (qi() * N + k) * 144; }
  __device__ const double* b(int k) const { return a.b + (qi() * N + k) * 12; }
  __device__ const double* Q(int k) const { return a.Q + (qi() * (N + 1) + k) * 144; }
  __device__ const double* S(int k) const { return a.S + (qi() * N + k) * 144; }
  __device__ const double* R(int k) const { return a.R + (qi() * N + k) * 144; }
  __device__ const double* qv(int k) const { return a.q + (qi() * (N + 1) + k) * 12; }
  __device__ const double* rv(int k) const { return a.r + (qi() * N + k) * 12; }
  __device__ double* rec(int k) const { return a.ws + qi() * a.ws_qp + (size_t)k * kRStage; }
  // row r of D_k / C_k (ng x 12, column-major): element j at [j * ng]; null when absent
  // (D_N: no input; C_0: dropped with x_0, ocp_qp_ipm_solver.cpp:128)
  __device__ const double* Drow(int k, int r) const {
    return (a.D && k < N) ? a.D + (qi() * N + k) * a.ng * 12 + r : nullptr;
  }
  __device__ const double* Crow(int k, int r) const {
    return (a.C && k > 0) ? a.C + (qi() * (N + 1) + k) * a.ng * 12 + r : nullptr;
  }
};

struct Side {
  double lb, ub, ml, mu;
};
__device__ __forceinline__ Side side_at(const double* lb, const double* ub, const double* lm,
                                        const double* um, size_t o) {
  const double ml = lm ? lm[o] : 1.0, mu = um ? um[o] : 1.0;
  return Side{lb[o], ub[o], ml != 0.0 ? 1.0 : 0.0, mu != 0.0 ? 1.0 : 0.0};
}
__device__ __forceinline__ Side side_u(const Qp& Q, int k, int i) {
  const ProblemArgsT<double>& a = Q.a;
  if (!a.lbu || k >= Q.N || i >= 12) return Side{0, 0, 0, 0};
  return side_at(a.lbu, a.ubu, a.lbu_mask, a.ubu_mask, ((size_t)Q.q * Q.N + k) * 12 + i);
}
__device__ __forceinline__ Side side_x(const Qp& Q, int k, int i) {
  const ProblemArgsT<double>& a = Q.a;
  if (!a.lbx || k == 0 || i >= 12) return Side{0, 0, 0, 0};  // stage-0 x bounds dropped
  return side_at(a.lbx, a.ubx, a.lbx_mask, a.ubx_mask, ((size_t)Q.q * (Q.N + 1) + k) * 12 + i);
}
__device__ __forceinline__ Side side_g(const Qp& Q, int k, int r) {
  const ProblemArgsT<double>& a = Q.a;
  if (r >= a.ng) return Side{0, 0, 0, 0};
  return side_at(a.lg, a.ug, a.lg_mask, a.ug_mask, ((size_t)Q.q * (Q.N + 1) + k) * a.ng + r);
}

struct Bar {
  double ll, lu, tl, tu;
};
struct BarStep {
  double dtl, dtu, dll, dlu;
};
__device__ __forceinline__ Bar ld_bar(const double* p, int i) { return Bar{p[i], p[12 + i], p[24 + i], p[36 + i]}; }
__device__ __forceinline__ void st_bar(double* p, int i, const Bar& b) {
  p[i] = b.ll;
  p[12 + i] = b.lu;
  p[24 + i] = b.tl;
  p[36 + i] = b.tu;
}
__device__ __forceinline__ BarStep ld_step(const double* p, int i) {
  return BarStep{p[i], p[12 + i], p[24 + i], p[36 + i]};
}
__device__ __forceinline__ void st_step(double* p, int i, const BarStep& d) {
  p[i] = d.dtl;
  p[12 + i] = d.dtu;
  p[24 + i] = d.dll;
  p[36 + i] = d.dlu;
}

// HPIPM init_var for one box-bounded variable: project into the box by thr0, t, lam = mu0 / t
__device__ __forceinline__ Bar init_box(const Side& s, double& v, double mu0) {
  Bar bb{0.0, 0.0, 1.0, 1.0};
  if (s.ml == 0.0 && s.mu == 0.0) return bb;
  double tl = v - s.lb, tu = s.ub - v;
  if (s.ml != 0.0 && s.mu != 0.0) {
    if (tl < kThr0) {
      if (tu < kThr0) {
        v = 0.5 * (s.lb + s.ub);
        tl = tu = kThr0;
      } else {
        tl = kThr0;
        v = s.lb + kThr0;
        tu = s.ub - v;
      }
    } else if (tu < kThr0) {
      tu = kThr0;
      v = s.ub - kThr0;
      tl = v - s.lb;
    }
  } else if (s.ml != 0.0) {
    if (tl < kThr0) {
      tl = kThr0;
      v = s.lb + kThr0;
    }
  } else if (tu < kThr0) {
    tu = kThr0;
    v = s.ub - kThr0;
  }
  bb.tl = s.ml != 0.0 ? tl : 1.0;
  bb.tu = s.mu != 0.0 ? tu : 1.0;
  bb.ll = s.ml != 0.0 ? mu0 / tl : 0.0;
  bb.lu = s.mu != 0.0 ? mu0 / tu : 0.0;
  return bb;
}
// Gamma / gamma of one side pair (ipm_box_impl.h gamma_of): rm = lam t + ext - smu
__device__ __forceinline__ void gamma_of(const Side& s, const Bar& b, double v, double el, double eu,
                                         double smu, double& G, double& g) {
  G = 0.0;
  g = 0.0;
  if (s.ml != 0.0) {
    const double rd = v - s.lb - b.tl, rm = b.ll * b.tl + el - smu;
    G += b.ll / b.tl;
    g += (rm + b.ll * rd) / b.tl;
  }
  if (s.mu != 0.0) {
    const double rd = s.ub - v - b.tu, rm = b.lu * b.tu + eu - smu;
    G += b.lu / b.tu;
    g -= (rm + b.lu * rd) / b.tu;
  }
}
__device__ __forceinline__ BarStep bar_step(const Side& s, const Bar& b, double v, double dv, double el,
                                            double eu, double smu) {
  BarStep d{0.0, 0.0, 0.0, 0.0};
  if (s.ml != 0.0) {
    d.dtl = (v - s.lb - b.tl) + dv;
    d.dll = -(b.ll * b.tl + el - smu + b.ll * d.dtl) / b.tl;
  }
  if (s.mu != 0.0) {
    d.dtu = (s.ub - v - b.tu) - dv;
    d.dlu = -(b.lu * b.tu + eu - smu + b.lu * d.dtu) / b.tu;
  }
  return d;
}
__device__ __forceinline__ void ratio(const Side& s, const Bar& b, const BarStep& d, double& ap, double& ad) {
  if (s.ml != 0.0) {
    if (d.dtl < 0.0) ap = fmin(ap, -b.tl / d.dtl);
    if (d.dll < 0.0) ad = fmin(ad, -b.ll / d.dll);
  }
  if (s.mu != 0.0) {
    if (d.dtu < 0.0) ap = fmin(ap, -b.tu / d.dtu);
    if (d.dlu < 0.0) ad = fmin(ad, -b.lu / d.dlu);
  }
}
__device__ __forceinline__ void aff_sums(const Side& s, const Bar& b, const BarStep& d, double& s1, double& s2) {
  if (s.ml != 0.0) {
    s1 += b.ll * d.dtl + b.tl * d.dll;
    s2 += d.dll * d.dtl;
  }
  if (s.mu != 0.0) {
    s1 += b.lu * d.dtu + b.tu * d.dlu;
    s2 += d.dlu * d.dtu;
  }
}
__device__ __forceinline__ double nabs(double v) { return v == v ? fabs(v) : __builtin_inf(); }
__device__ __forceinline__ bool huge(double v) { return !(fabs(v) < 1.3e150); }
__device__ __forceinline__ double stepv(double v, double a, double d) { return a != 0.0 ? fma(a, d, v) : v; }
// A value every lane holds the same copy of (the block reductions), moved to SGPRs: the kernel
// loop keeps ~10 such scalars live across the factorization, which needs every VGPR.
__device__ __forceinline__ double uni(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ double g16sum(double v) {
  v += __shfl_xor(v, 8, kGroup);
  v += __shfl_xor(v, 4, kGroup);
  v += __shfl_xor(v, 2, kGroup);
  v += __shfl_xor(v, 1, kGroup);
  return v;
}
__device__ __forceinline__ double g16max(double v) {
  v = fmax(v, __shfl_xor(v, 8, kGroup));
  v = fmax(v, __shfl_xor(v, 4, kGroup));
  v = fmax(v, __shfl_xor(v, 2, kGroup));
  v = fmax(v, __shfl_xor(v, 1, kGroup));
  return v;
}
__device__ __forceinline__ double g16min(double v) {
  v = fmin(v, __shfl_xor(v, 8, kGroup));
  v = fmin(v, __shfl_xor(v, 4, kGroup));
  v = fmin(v, __shfl_xor(v, 2, kGroup));
  v = fmin(v, __shfl_xor(v, 1, kGroup));
  return v;
}

// 12 strided values p[i * ld] (a row of a column-major block), 0 where p is null
__device__ __forceinline__ void load_strided(const double* p, int ld, double (&v)[12]) {
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    v[I] = p ? p[I * ld] : 0.0;
  });
}
__device__ __forceinline__ void load12z(const double* p, double (&v)[12]) {
  if (p) {
    load12(p, v);
  } else {
    sfor<0, 12>([&](auto i) { v[decltype(i)::value] = 0.0; });
  }
}

// (P v)_jj + acc for an element-owned v (lane j holds v_j), P from a stage record's kRP slot:
// P packed (classical), or SQRT its factor Lp, applied as Lp (Lp' v) -- exactly the P the next
// stage's factorization used (the batched kernels' rec_P_mul, ipm_box_impl.h)
template <bool SQRT>
__device__ __forceinline__ double rec_P_apply(const double* rkP, int jj, double v, double acc) {
  double M[12];
  if constexpr (SQRT) {
    load_packed_lcol_d(rkP, jj, M);
    const double t = dot_bcast(M, v, 0.0);  // (Lp' v)_jj
    load_packed_lrow_d(rkP, jj, M);
    return dot_bcast(M, t, acc);
  } else {
    load_packed_sym(rkP, jj, M);
    return dot_bcast(M, v, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// block-wide reductions of per-group partials: slot values written by each group's lane 0,
// reduced by every thread after the barrier (same order everywhere: uniform results)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void red_put(const Lds& L, int slot, double v) {
  if ((threadIdx.x & 15) == 0) L.red()[(threadIdx.x >> 4) * kRedSlots + slot] = v;
}
__device__ __forceinline__ double red_sum(const Lds& L, int slot) {
  double s = 0.0;
  for (int g = 0; g < kGroups; ++g) s += L.red()[g * kRedSlots + slot];
  return s;
}
__device__ __forceinline__ double red_max(const Lds& L, int slot) {
  double s = 0.0;
  for (int g = 0; g < kGroups; ++g) {
    const double v = L.red()[g * kRedSlots + slot];
    s = (v > s || v != v) ? v : s;
  }
  return s;
}
__device__ __forceinline__ double red_min(const Lds& L, int slot) {
  double s = 1e30;
  for (int g = 0; g < kGroups; ++g) s = fmin(s, L.red()[g * kRedSlots + slot]);
  return s;
}

// ---------------------------------------------------------------------------------------------
// phase: initial point (HPIPM init_var, ipm_box_impl.h kPhInit)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void init_point(const Qp Q, const Lds L) {
  const ProblemArgsT<double>& a = Q.a;
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  double ncl = 0.0;
  for (int k = grp; k <= N; k += kGroups) {
    double uv = 0.0, xv = 0.0;
    if (k < N) {
      double v = (a.warm_start && el) ? a.u[((size_t)Q.q * N + k) * 12 + j] : 0.0;
      const Side s = side_u(Q, k, j);
      const Bar bb = init_box(s, v, a.mu0);
      ncl += s.ml + s.mu;
      if (el) {
        st_bar(L.bu() + k * 48, j, bb);
        st_step(L.su() + k * 48, j, BarStep{0, 0, 0, 0});
        L.u()[k * 12 + j] = v;
      }
      uv = el ? v : 0.0;
    } else if (el) {
      st_bar(L.bu() + k * 48, j, Bar{0, 0, 1, 1});
      st_step(L.su() + k * 48, j, BarStep{0, 0, 0, 0});
      L.u()[k * 12 + j] = 0.0;
    }
    {
      double v = k == 0 ? (el ? a.x0[(size_t)Q.q * 12 + j] : 0.0)
                        : ((a.warm_start && el) ? a.x[((size_t)Q.q * (N + 1) + k) * 12 + j] : 0.0);
      const Side s = side_x(Q, k, j);
      const Bar bb = init_box(s, v, a.mu0);
      ncl += s.ml + s.mu;
      if (el) {
        st_bar(L.bx() + k * 48, j, bb);
        st_step(L.sx() + k * 48, j, BarStep{0, 0, 0, 0});
        L.x()[k * 12 + j] = v;
        L.pi()[k * 12 + j] = 0.0;
      }
      xv = el ? v : 0.0;
    }
    // general rows: t = max(v - lg, thr0), max(ug - v, thr0) at the initial point
    for (int ch = 0; ch < L.nch; ++ch) {
      const int r = ch * 12 + j;
      const bool ok = el && r < a.ng;
      double Dr[12], Cr[12];
      load_strided(ok ? Q.Drow(k, r) : nullptr, a.ng, Dr);
      load_strided(ok ? Q.Crow(k, r) : nullptr, a.ng, Cr);
      const double v = dot_bcast(Cr, xv, dot_bcast(Dr, uv, 0.0));
      const Side s = ok ? side_g(Q, k, r) : Side{0, 0, 0, 0};
      Bar bb{0.0, 0.0, 1.0, 1.0};
      if (s.ml != 0.0) {
        bb.tl = fmax(v - s.lb, kThr0);
        bb.ll = a.mu0 / bb.tl;
      }
      if (s.mu != 0.0) {
        bb.tu = fmax(s.ub - v, kThr0);
        bb.lu = a.mu0 / bb.tu;
      }
      ncl += s.ml + s.mu;
      if (el) {
        double* g = L.gb(k, ch);
        st_bar(g, j, bb);
        st_step(g + 48, j, BarStep{0, 0, 0, 0});
        g[96 + j] = v;
      }
    }
  }
  red_put(L, 0, g16sum(ncl));
}

// ---------------------------------------------------------------------------------------------
// phase: the previous step applied (alpha_p on x, u, t; alpha_d on pi, lam), the residuals at the
// new iterate (oracle compute_residuals; HPIPM d_ocp_qp_res_compute) and, with PRED, the
// predictor's barrier-augmented stage blocks R~, S~, Q~, r~, q~, b~ for the factorization -- one
// pass per stage, the R, S, Q columns loaded once for both.  x and pi are double-buffered:
// stage k reads the old x_k+1, pi_k+1 and their steps and forms the new values itself, so no
// stage waits for its neighbour's update (the new iterate goes to buffer cur ^ 1).
// ---------------------------------------------------------------------------------------------
template <bool HAS_C, bool PRED, bool SQRT = false>
__device__ __forceinline__ void stage_pass(const Qp Q, const Lds L, double ap, double ad);

// column j of chunk ch's rows of D_k (or C_k): v[i] = D[ch * 12 + i][j], 0 past ng / when absent
template <bool ISC>
__device__ __forceinline__ void gen_col(const Qp& Q, int k, int ch, int jj, bool el, double (&v)[12]) {
  const int rr = ch * 12, ng = Q.a.ng;
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    const bool iok = el && rr + I < ng;
    const double* p = iok ? (ISC ? Q.Crow(k, rr + I) : Q.Drow(k, rr + I)) : nullptr;
    v[I] = p ? p[(size_t)ng * jj] : 0.0;
  });
}
// row j of chunk ch (lane j = row ch * 12 + j): v[i] = D[ch * 12 + j][i]
template <bool ISC>
__device__ __forceinline__ void gen_row(const Qp& Q, int k, int ch, int j, bool el, double (&v)[12]) {
  const int r = ch * 12 + j;
  const bool ok = el && r < Q.a.ng;
  load_strided(ok ? (ISC ? Q.Crow(k, r) : Q.Drow(k, r)) : nullptr, Q.a.ng, v);
}
// C[i] += sum_r X[r][i] Gamma_r Y[r][j] over the general rows (column j of X'Gamma Y; X = D or C
// row-owned on the chunk's lanes, Y's column j on lane j, Gamma from the chunk's LDS slot)
// SYM: as sums of the scaled rows' products, (sqrt(Gamma) X)'(sqrt(Gamma) Y), so D'Gamma D and
// C'Gamma C are exactly symmetric (the batched kernels' g_hess form): the square-root chain
// factorizes the P these terms enter, and a Gamma of 1e13 times rounding-level asymmetry breaks
// that Cholesky (the classical form keeps Gamma on one side, as round 5 measured it)
template <bool XC, bool YC, bool SYM = false>
__device__ __forceinline__ void gen_syrk(const Qp& Q, const Lds& L, int k, int j, int jj, bool el,
                                         double (&C)[12]) {
  for (int ch = 0; ch < L.nch; ++ch) {
    double Xr[12], Yc[12];
    gen_row<XC>(Q, k, ch, j, el, Xr);
    gen_col<YC>(Q, k, ch, jj, el, Yc);
    const double G = el ? L.gb(k, ch)[108 + j] : 0.0;
    if constexpr (SYM) {
      const double sG = __builtin_sqrt(G);
      sfor<0, 12>([&](auto i) { Xr[decltype(i)::value] *= sG; });
      sfor<0, 12>([&](auto rs) {
        constexpr int R = decltype(rs)::value;
        fma_bcast_src<R>(C, Xr, bc<R>(sG) * Yc[R]);
      });
    } else {
      sfor<0, 12>([&](auto rs) {
        constexpr int R = decltype(rs)::value;
        fma_bcast_src<R>(C, Xr, bc<R>(G) * Yc[R]);
      });
    }
  }
}

template <bool HAS_C, bool PRED, bool SQRT>
__device__ __forceinline__ void stage_pass(const Qp Q, const Lds L, double ap, double ad) {
  const ProblemArgsT<double>& a = Q.a;
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  const int jj = el ? j : 11;
  const double* xo = L.xb(L.cur);
  const double* po = L.pib(L.cur);
  double* xw = L.xb(L.cur ^ 1);
  double* pw = L.pib(L.cur ^ 1);
  double mg = 0.0, mb = 0.0, md = 0.0, mm = 0.0, musum = 0.0, objl = 0.0;
  auto upd = [&](double* bp, const double* sp) {
    Bar b = ld_bar(bp, j);
    const BarStep d = ld_step(sp, j);
    b.tl = stepv(b.tl, ap, d.dtl);
    b.tu = stepv(b.tu, ap, d.dtu);
    b.ll = stepv(b.ll, ad, d.dll);
    b.lu = stepv(b.lu, ad, d.dlu);
    st_bar(bp, j, b);
    return b;
  };
  for (int k = grp; k <= N; k += kGroups) {
    // ---- the step: stage k's own state in place, x_k+1 / pi_k+1 from the old buffer ----
    double uj = 0.0, xj = 0.0, pij = 0.0, xnj = 0.0, pinj = 0.0;
    Bar bu{0, 0, 1, 1}, bx{0, 0, 1, 1};
    if (el) {
      if (k < N) {
        uj = stepv(L.u()[k * 12 + j], ap, L.du()[k * 12 + j]);
        L.u()[k * 12 + j] = uj;
        xnj = stepv(xo[(k + 1) * 12 + j], ap, L.dx()[(k + 1) * 12 + j]);
        pinj = stepv(po[(k + 1) * 12 + j], ad, L.dpi()[(k + 1) * 12 + j]);
      }
      xj = xo[k * 12 + j];
      pij = po[k * 12 + j];
      if (k > 0) {  // (x_0 = x0 is fixed; pi_0 is not an iterate)
        xj = stepv(xj, ap, L.dx()[k * 12 + j]);
        pij = stepv(pij, ad, L.dpi()[k * 12 + j]);
      }
      xw[k * 12 + j] = xj;
      pw[k * 12 + j] = pij;
      bu = upd(L.bu() + k * 48, L.su() + k * 48);
      bx = upd(L.bx() + k * 48, L.sx() + k * 48);
    }
    // ---- residuals (the R, S, Q columns are loaded again, from L1 / L2, for the Hessian
    // blocks below: kept live across the general rows they spilled) ----
    double gu = 0.0, gx;
    double M[12];
    double sx = 0.0;  // (S x)_j
    if (k < N) {
      load12(Q.R(k) + jj * 12, M);
      const double t1 = dot_bcast(M, uj, 0.0);
      load_strided(Q.S(k) + jj, 12, M);
      sx = dot_bcast(M, xj, 0.0);
      const double rj = el ? Q.rv(k)[j] : 0.0;
      load12(Q.B(k) + jj * 12, M);
      const double bpi = dot_bcast(M, pinj, 0.0);
      gu = t1 + sx + rj + bpi;
      double o = uj * (0.5 * t1 + rj);
      if (k == 0) o += uj * sx;
      objl += el ? o : 0.0;
    }
    load12(Q.Q(k) + jj * 12, M);
    {
      const double t1 = dot_bcast(M, xj, 0.0);
      const double qj = el ? Q.qv(k)[j] : 0.0;
      gx = t1 + qj - pij;
      if (k > 0) {
        double o = xj * (0.5 * t1 + qj);
        if (k < N) o += uj * sx;
        objl += el ? o : 0.0;
      }
      if (k < N) {
        load12(Q.S(k) + jj * 12, M);
        gx += dot_bcast(M, uj, 0.0);
        load12(Q.A(k) + jj * 12, M);
        gx += dot_bcast(M, pinj, 0.0);
      }
    }
    // box rows: gradient terms, rd / rm; Gamma, gamma of the predictor
    double Gu = 0.0, gam_u = 0.0, Gx = 0.0, gam_x = 0.0;
    if (k < N) {
      const Side s = side_u(Q, k, j);
      gu -= (s.ml != 0.0 ? bu.ll : 0.0) - (s.mu != 0.0 ? bu.lu : 0.0);
      if (s.ml != 0.0) {
        const double rd = uj - s.lb - bu.tl, rm = bu.ll * bu.tl;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      if (s.mu != 0.0) {
        const double rd = s.ub - uj - bu.tu, rm = bu.lu * bu.tu;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      if (PRED && el) gamma_of(s, bu, uj, 0.0, 0.0, 0.0, Gu, gam_u);
    }
    if (k > 0) {
      const Side s = side_x(Q, k, j);
      gx -= (s.ml != 0.0 ? bx.ll : 0.0) - (s.mu != 0.0 ? bx.lu : 0.0);
      if (s.ml != 0.0) {
        const double rd = xj - s.lb - bx.tl, rm = bx.ll * bx.tl;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      if (s.mu != 0.0) {
        const double rd = s.ub - xj - bx.tu, rm = bx.lu * bx.tu;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      if (PRED && el) gamma_of(s, bx, xj, 0.0, 0.0, 0.0, Gx, gam_x);
    }
    // general rows (lane j = row ch * 12 + j of the chunk): the step, values, rd / rm, gradient
    // terms; the predictor's Gamma (kept for the Hessian passes) and gamma
    double gpu = 0.0, gpx = 0.0;  // D'gamma, C'gamma
    for (int ch = 0; ch < L.nch; ++ch) {
      const int r = ch * 12 + j;
      const bool ok = el && r < a.ng;
      double* g = L.gb(k, ch);
      const Bar b = el ? upd(g, g + 48) : Bar{0, 0, 1, 1};
      double Dr[12], Cr[12];
      gen_row<false>(Q, k, ch, j, el, Dr);
      if constexpr (HAS_C) {
        gen_row<true>(Q, k, ch, j, el, Cr);
      } else {
        sfor<0, 12>([&](auto i) { Cr[decltype(i)::value] = 0.0; });
      }
      const double v = dot_bcast(Cr, xj, dot_bcast(Dr, uj, 0.0));
      const Side sg = ok ? side_g(Q, k, r) : Side{0, 0, 0, 0};
      if (el) g[96 + j] = v;
      if (sg.ml != 0.0) {
        const double rd = v - sg.lb - b.tl, rm = b.ll * b.tl;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      if (sg.mu != 0.0) {
        const double rd = sg.ub - v - b.tu, rm = b.lu * b.tu;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      const double cr = (sg.ml != 0.0 ? b.ll : 0.0) - (sg.mu != 0.0 ? b.lu : 0.0);
      double G = 0.0, gam = 0.0;
      if (PRED && ok) gamma_of(sg, b, v, 0.0, 0.0, 0.0, G, gam);
      if (PRED && el) g[108 + j] = G;
      double Yc[12];
      gen_col<false>(Q, k, ch, jj, el, Yc);
      gu -= dot_bcast(Yc, cr, 0.0);
      if (PRED) gpu = dot_bcast(Yc, gam, gpu);
      if constexpr (HAS_C) {
        gen_col<true>(Q, k, ch, jj, el, Yc);
        gx -= dot_bcast(Yc, cr, 0.0);
        if (PRED) gpx = dot_bcast(Yc, gam, gpx);
      }
    }
    if (k < N) mg = fmax(mg, el ? nabs(gu) : 0.0);
    if (k > 0) mg = fmax(mg, el ? nabs(gx) : 0.0);
    double rbj = 0.0;
    if (k < N) {
      double Br[12];
      load_strided(Q.A(k) + jj, 12, M);
      load_strided(Q.B(k) + jj, 12, Br);
      const double t1 = dot_bcast(M, xj, 0.0), t2 = dot_bcast(Br, uj, 0.0);
      rbj = t1 + t2 + (el ? Q.b(k)[j] : 0.0) - xnj;
      mb = fmax(mb, el ? nabs(rbj) : 0.0);
    }
    if (el) {
      L.rgu()[k * 12 + j] = gu;
      L.rgx()[k * 12 + j] = gx;
      L.rb()[k * 12 + j] = rbj;
    }
    if (!PRED) continue;
    // ---- the predictor's stage blocks into the record ----
    double* rk = Q.rec(k);
    double Rc[12], Sc[12], Qc[12];
    if (k < N) {
      load12(Q.R(k) + jj * 12, Rc);
      load12(Q.S(k) + jj * 12, Sc);
      sfor<0, 12>([&](auto i) { Rc[decltype(i)::value] += decltype(i)::value == j ? Gu : 0.0; });
      gen_syrk<false, false, SQRT>(Q, L, k, j, jj, el, Rc);  // R~ = R + diag(Gamma_u) + D'Gamma D
      if constexpr (HAS_C) gen_syrk<false, true, SQRT>(Q, L, k, j, jj, el, Sc);  // S~ = S + D'Gamma C
      if (el) {
        store12(rk + kRR + j * 12, Rc);
        store12(rk + kRS + j * 12, Sc);
        rk[kRr + j] = gu + gam_u + gpu;
        rk[kRb + j] = rbj;
      }
    }
    load12(Q.Q(k) + jj * 12, Qc);
    sfor<0, 12>([&](auto i) { Qc[decltype(i)::value] += decltype(i)::value == j ? Gx : 0.0; });
    if constexpr (HAS_C) gen_syrk<true, true, SQRT>(Q, L, k, j, jj, el, Qc);  // Q~ = Q + diag(Gamma_x) + C'Gamma C
    if (el) {
      store12(rk + kRQ + j * 12, Qc);
      rk[kRq + j] = gx + gam_x + gpx;
    }
  }
  red_put(L, 0, g16max(mg));
  red_put(L, 1, g16max(mb));
  red_put(L, 2, g16max(md));
  red_put(L, 3, g16max(mm));
  red_put(L, 4, g16sum(el ? musum : 0.0));
  red_put(L, 5, g16sum(objl));
}

// ---------------------------------------------------------------------------------------------
// phase: the corrector's gradient: gamma with the predictor's dlam dt and sigma mu (HPIPM's
// res_m = lam t + dlam_aff dt_aff - sigma mu), g~ = res_g + gamma terms into gtu / gtx
// ---------------------------------------------------------------------------------------------
template <bool HAS_C>
__device__ __forceinline__ void corr_terms(const Qp Q, const Lds L, double smu) {
  const ProblemArgsT<double>& a = Q.a;
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  const int jj = el ? j : 11;
  for (int k = grp; k <= N; k += kGroups) {
    double gam_u = 0.0, gam_x = 0.0, G = 0.0;
    if (k < N && el) {
      const BarStep d = ld_step(L.su() + k * 48, j);
      gamma_of(side_u(Q, k, j), ld_bar(L.bu() + k * 48, j), L.u()[k * 12 + j], d.dll * d.dtl, d.dlu * d.dtu, smu,
               G, gam_u);
    }
    if (k > 0 && el) {
      const BarStep d = ld_step(L.sx() + k * 48, j);
      gamma_of(side_x(Q, k, j), ld_bar(L.bx() + k * 48, j), L.x()[k * 12 + j], d.dll * d.dtl, d.dlu * d.dtu, smu,
               G, gam_x);
    }
    double gu = (el ? L.rgu()[k * 12 + j] : 0.0) + gam_u;
    double gx = (el ? L.rgx()[k * 12 + j] : 0.0) + gam_x;
    for (int ch = 0; ch < L.nch; ++ch) {
      const int r = ch * 12 + j;
      const bool ok = el && r < a.ng;
      const double* g = L.gb(k, ch);
      double gam = 0.0;
      if (ok) {
        const BarStep d = ld_step(g + 48, j);
        gamma_of(side_g(Q, k, r), ld_bar(g, j), g[96 + j], d.dll * d.dtl, d.dlu * d.dtu, smu, G, gam);
      }
      double Mc[12];
      gen_col<false>(Q, k, ch, jj, el, Mc);
      gu = dot_bcast(Mc, gam, gu);
      if constexpr (HAS_C) {
        gen_col<true>(Q, k, ch, jj, el, Mc);
        gx = dot_bcast(Mc, gam, gx);
      }
    }
    if (el) {
      L.gtu()[k * 12 + j] = gu;
      L.gtx()[k * 12 + j] = gx;
    }
  }
}

// [P | p] in the tiles' C/D layout (wave 0) -> [Lp | s]: Lp = chol(P) (lower; a non-positive pivot
// zeroes its column, BLASFEO dpotrf_l, riccati.h sqrt_factor) and s = Lp^-1 p, the border column
// of the same elimination, through the G/H tile (column-owned Cholesky, then back).  Lp also
// goes to the stage record's P slot (rkP, packed; row group 0 writes): the sweeps apply P as
// Lp (Lp' v), the P this factorization continues with.
__device__ __forceinline__ lat_d4 sqrt_tile(const lat_d4& Pt, double* gh, int g, int c, double* rkP) {
  const bool cv = c < 12, cw = c <= 12;
  lds_wave_fence();
  sfor<0, 3>([&](auto rr) {
    constexpr int R = decltype(rr)::value;
    if (cw) gh[c * 12 + g + 4 * R] = Pt[R];
  });
  lds_wave_fence();
  double Pc[12], Lc[12], rs;
  sfor<0, 12>([&](auto i) {
    const double v = gh[(cw ? c : 12) * 12 + decltype(i)::value];
    Pc[decltype(i)::value] = cw ? v : 0.0;
  });
  // (pivots by lat_recip, as the G factor: IEEE division measured 2% slower at batch 1, box-u,
  // with the same iteration counts -- profiles/round6/sqrt_recip/)
  lat_chol(Pc, c, 0.0, Lc, rs, [](auto) {});
  lds_wave_fence();
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    const double ri = bc<I>(rs);
    // lane c < 12: column c of Lp (zero above the diagonal); lane 12: s
    Lc[I] = cv ? (I >= c ? Lc[I] : 0.0) : Lc[I] * ri;
    if (cw && g == 0) gh[c * 12 + I] = Lc[I];
  });
  if (cv && g == 0) store_packed_col(rkP, c, Lc);
  lds_wave_fence();
  lat_d4 o;
  sfor<0, 4>([&](auto rr) {
    constexpr int R = decltype(rr)::value;
    const int row = g + 4 * R < 12 ? g + 4 * R : 11;
    const double v = gh[(cw ? c : 12) * 12 + row];
    o[R] = (g + 4 * R < 12 && cw) ? v : 0.0;
  });
  lds_wave_fence();
  return o;
}

// ---------------------------------------------------------------------------------------------
// phase: the factorization (backward, serial in k) on matrix cores -- riccati_latency_impl.h's
// sweep.  Wave 0: stage k's products and Cholesky; wave 1: stage k+1's K, record and closed
// loop; wave 2: stage k-1's operands (A, B from the QP, R~ S~ Q~ r~ q~ b~ from the record) into
// the LDS ring, so no global load sits on the chain.  Records per stage: [K | k] rows, P packed,
// p, L packed + 1 / diag; [Acl | bcl] rows in LDS.
// SQRT (ric_alg 1, hpipm-cpp's default; riccati.h riccati_step_sqrt): the chain carries the factor
// Lp of P_k+1 and s = Lp^-1 p_k+1 instead of [P | p], and the same MFMAs form MB = Lp'B,
// MA = Lp'[A | b~] + [0 | s], G = R~ + MB'MB, [H | g] = [S~ | r~] + MB'MA, [F | f] = [Q~ | q~] +
// MA'MA (sums of squares: the classical B'PB, B'P[A | b~], A'P[A | b~] in exact arithmetic);
// P_k = F - Y'Y is factorized again for the next stage (sqrt_tile: a second Cholesky on the
// chain) and the record keeps that factor Lp, with p explicit (HPIPM's p-form).
// ---------------------------------------------------------------------------------------------
template <bool SQRT>
__device__ __forceinline__ void factorize(const Qp Q, const Lds L) {
  const ProblemArgsT<double>& a = Q.a;
  const int N = Q.N;
  const int wave = threadIdx.x >> 6, l = opq(threadIdx.x & 63);
  const int g = l >> 4, c = l & 15;
  const bool cv = c < 12, cw = c <= 12;
  const int cc = cv ? c : 11;
  double* const gh = L.scr();
  double* const ybuf = L.scr() + 156;
  double* const lbuf = L.scr() + 3 * 156;
  double* const ring = L.ring();
  auto slot = [&](int k) { return ring + (k % 3) * kSlot; };
  auto load_slot = [&](int k) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2* s2 = reinterpret_cast<d2*>(slot(k));
    const d2* A2 = reinterpret_cast<const d2*>(Q.A(k));
    const d2* B2 = reinterpret_cast<const d2*>(Q.B(k));
    const d2* I2 = reinterpret_cast<const d2*>(Q.rec(k) + kRb);
    for (int t = l; t < 72; t += 64) {
      s2[kSA / 2 + t] = A2[t];
      s2[kSB / 2 + t] = B2[t];
    }
    for (int t = l; t < (kSlot - kSb) / 2; t += 64) s2[kSb / 2 + t] = I2[t];
  };
  lat_d4 Pt;
  if (wave == 0) {
    const double* rn = Q.rec(N);
    sfor<0, 4>([&](auto rr) {
      constexpr int R = decltype(rr)::value;
      const int row = g + 4 * R < 12 ? g + 4 * R : 11;
      const double v = rn[cv ? kRQ + c * 12 + row : kRq + row];
      Pt[R] = (g + 4 * R < 12 && cw) ? v : 0.0;
    });
    double* wn = Q.rec(N);
    if constexpr (SQRT) {
      sfor<0, 3>([&](auto rr) {
        constexpr int R = decltype(rr)::value;
        if (c == 12) wn[kRp + g + 4 * R] = Pt[R];
      });
      Pt = sqrt_tile(Pt, gh, g, c, wn + kRP);
    } else {
      sfor<0, 3>([&](auto rr) {
        constexpr int R = decltype(rr)::value;
        const int row = g + 4 * R;
        if (cv && row >= c) wn[kRP + packed_col(c) + row - c] = Pt[R];
        if (c == 12) wn[kRp + row] = Pt[R];
      });
    }
  } else if (wave == 2) {
    load_slot(N - 1);
  }
  __syncthreads();
  auto finish_stage = [&](int jst) {
    const double* lb = lbuf + (jst & 1) * 90;
    const double* yb = ybuf + (jst & 1) * 156;
    const double* sl = slot(jst);
    double Lc[12], Yc[12], Kc[12];
    load_packed_lcol(lb, cc, Lc);
    const double rs = lb[78 + cc];
    sfor<0, 12>([&](auto i) { Yc[decltype(i)::value] = cw ? yb[c * 12 + decltype(i)::value] : 0.0; });
    trsv_upper_t_neg_axpy(Lc, rs, Yc, Kc);  // lane c < 12: K[:, c]; lane 12: k
    double* rj = Q.rec(jst);
    if (l < 16 && cw)
      sfor<0, 12>([&](auto i) { rj[kRK + decltype(i)::value * 13 + c] = Kc[decltype(i)::value]; });
    for (int t = l; t < 90; t += 64) rj[kRL + t] = lb[t];
    // [Acl | bcl][:, c] = [A | b~][:, c] + B [K | k][:, c]
    double Ac[12], Bc[12];
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      const double av = sl[cv ? kSA + c * 12 + I : kSb + I];
      Ac[I] = cw ? av : 0.0;
      const double bv = sl[kSB + cc * 12 + I];
      Bc[I] = cv ? bv : 0.0;
    });
    sfor<0, 12>([&](auto m) {
      constexpr int M = decltype(m)::value;
      fma_bcast_src<M>(Ac, Bc, Kc[M]);
    });
    if (l < 16 && cw)
      sfor<0, 12>([&](auto i) { L.acl()[jst * 156 + decltype(i)::value * 13 + c] = Ac[decltype(i)::value]; });
  };
#pragma unroll 1
  for (int k = N - 1; k >= 0; --k) {
    if (wave == 0) {
      tstamp(70);
      const double* sl = slot(k);
      double bo[3], ao[3];
      sfor<0, 3>([&](auto kb) {
        constexpr int KB = decltype(kb)::value;
        const int m = 4 * KB + g;
        const double bv = sl[kSB + cc * 12 + m];
        bo[KB] = cv ? bv : 0.0;  // B[m][c]: B operand of P B; A operand (B') of B'WB, B'W
        const double av = sl[cv ? kSA + c * 12 + m : kSb + m];
        ao[KB] = cw ? av : 0.0;  // [A | b~][m][c]: B operand of P [A | b~]; A operand (A') of A'W
      });
      lat_d4 Rt, St, Qt;
      sfor<0, 4>([&](auto rr) {
        constexpr int R = decltype(rr)::value;
        const bool rok = g + 4 * R < 12;
        const int row = rok ? g + 4 * R : 11;
        const double rv = sl[kSR + cc * 12 + row];
        const double sv = sl[cv ? kSS + c * 12 + row : kSr + row];
        const double qv = sl[cv ? kSQ + c * 12 + row : kSq + row];
        Rt[R] = rok && cv ? rv : 0.0;
        St[R] = rok && cw ? sv : 0.0;
        Qt[R] = rok && cw ? qv : 0.0;
      });
      // WB = P B; G = R~ + B'WB (the critical path)
      lat_d4 WB = {0.0, 0.0, 0.0, 0.0};
      sfor<0, 3>([&](auto kb) { WB = lat_mfma(Pt[decltype(kb)::value], bo[decltype(kb)::value], WB); });
      lat_d4 Gt = Rt;
      if constexpr (SQRT) {  // (the A operand Pt is Lp: WB = Lp'B = MB, G = R~ + MB'MB)
        sfor<0, 3>([&](auto kb) { Gt = lat_mfma(WB[decltype(kb)::value], WB[decltype(kb)::value], Gt); });
      } else {
        sfor<0, 3>([&](auto kb) { Gt = lat_mfma(bo[decltype(kb)::value], WB[decltype(kb)::value], Gt); });
      }
      // W = P [A | b~] + [0 | p]; [H | g] = [S~ | r~] + B'W; [F | f] = [Q~ | q~] + A'W: one per pivot
      lat_d4 Wt;
      sfor<0, 4>([&](auto rr) { Wt[decltype(rr)::value] = c == 12 ? Pt[decltype(rr)::value] : 0.0; });
      lat_d4 Ht = St, Ft = Qt;
      auto wh = [&](auto kk) {
        constexpr int K = decltype(kk)::value;
        if constexpr (K < 3) {
          Wt = lat_mfma(Pt[K], ao[K], Wt);
        } else if constexpr (K < 9) {
          constexpr int KB = (K - 3) / 2;
          if constexpr ((K - 3) % 2 == 0) {
            Ht = lat_mfma(bo[KB], Wt[KB], Ht);
          } else {
            Ft = lat_mfma(ao[KB], Wt[KB], Ft);
          }
        }
      };
      // SQRT: W = MA; H = S~ + MB'MA, F = Q~ + MA'MA (MB = WB kept for H)
      auto wh_sqrt = [&](auto kk) {
        constexpr int K = decltype(kk)::value;
        if constexpr (K < 3) {
          Wt = lat_mfma(Pt[K], ao[K], Wt);
        } else if constexpr (K < 9) {
          constexpr int KB = (K - 3) / 2;
          if constexpr ((K - 3) % 2 == 0) {
            Ht = lat_mfma(WB[KB], Wt[KB], Ht);
          } else {
            Ft = lat_mfma(Wt[KB], Wt[KB], Ft);
          }
        }
      };
      lds_wave_fence();
      sfor<0, 3>([&](auto rr) {
        constexpr int R = decltype(rr)::value;
        if (cv) gh[c * 12 + g + 4 * R] = Gt[R];
      });
      lds_wave_fence();
      double Gc[12], Lc[12], rs;
      sfor<0, 12>([&](auto i) {
        const double v = gh[cc * 12 + decltype(i)::value];
        Gc[decltype(i)::value] = cv ? v : 0.0;
      });
      tstamp(71);
      if constexpr (SQRT) {
        lat_chol(Gc, c, a.reg, Lc, rs, wh_sqrt);
      } else {
        lat_chol(Gc, c, a.reg, Lc, rs, wh);
      }
      tstamp(72);
      // [Y | y] = L^-1 [H | g]
      lds_wave_fence();
      sfor<0, 3>([&](auto rr) {
        constexpr int R = decltype(rr)::value;
        if (cw) gh[c * 12 + g + 4 * R] = Ht[R];
      });
      lds_wave_fence();
      double Yc[12];
      sfor<0, 12>([&](auto i) {
        const double v = gh[(cw ? c : 12) * 12 + decltype(i)::value];
        Yc[decltype(i)::value] = cw ? v : 0.0;
      });
      trsv_lower(Lc, rs, Yc);
      tstamp(73);
      double* yb = ybuf + (k & 1) * 156;
      double* lb = lbuf + (k & 1) * 90;
      if (l < 16) {
        if (cw) store12(yb + c * 12, Yc);
        if (cv) {
          store_packed_col(lb, c, Lc);
          lb[78 + c] = rs;
        }
      }
      lds_wave_fence();
      // [P | p]_k = [F | f] - Y'[Y | y], P symmetrized by averaging (the oracle's and the batched
      // kernels' symmetrization): unsymmetrized, the next stage's products read P
      // as A operand (P') and as B operand (P), and the endgame stalls the stationarity residual
      // near 3e-7 on QPs whose barrier terms reach ~1e10 (random C / D rows), 61 / 64 on the
      // degenerate family; symmetrized 64 / 64.  (F + K'H with K = -L^-T Y on the chain, the
      // batched kernels' form, measured 61 / 64 here and 4% slower.)
      lat_d4 Pn = Ft;
      sfor<0, 3>([&](auto kb) {
        constexpr int KB = decltype(kb)::value;
        const double yv = yb[(cw ? c : 12) * 12 + 4 * KB + g];
        const double yB = cw ? yv : 0.0;
        const double yA = cv ? -yv : 0.0;
        Pn = lat_mfma(yA, yB, Pn);
      });
      sfor<0, 3>([&](auto rr) {
        constexpr int R = decltype(rr)::value;
        if (cv) gh[c * 12 + g + 4 * R] = Pn[R];
      });
      lds_wave_fence();
      sfor<0, 3>([&](auto rr) {
        constexpr int R = decltype(rr)::value;
        const double t = gh[(g + 4 * R) * 12 + cc];  // P[c][g + 4 R]
        if (cv) Pn[R] = 0.5 * (Pn[R] + t);
      });
      lds_wave_fence();
      tstamp(75);
      Pt = Pn;
      double* rk = Q.rec(k);
      if constexpr (SQRT) {
        sfor<0, 3>([&](auto rr) {
          constexpr int R = decltype(rr)::value;
          if (c == 12) rk[kRp + g + 4 * R] = Pt[R];
        });
        Pt = sqrt_tile(Pn, gh, g, c, rk + kRP);
      } else {
        sfor<0, 3>([&](auto rr) {
          constexpr int R = decltype(rr)::value;
          const int row = g + 4 * R;
          if (cv && row >= c) rk[kRP + packed_col(c) + row - c] = Pt[R];
          if (c == 12) rk[kRp + row] = Pt[R];
        });
      }
    } else if (wave == 1) {
      if (k < N - 1) finish_stage(k + 1);
    } else if (wave == 2) {
      if (k > 0) load_slot(k - 1);
    }
    __syncthreads();
  }
  if (wave == 1) finish_stage(0);
}

// ---------------------------------------------------------------------------------------------
// phase: forward recursion dx_k+1 = Acl_k dx_k + bcl_k, dx_0 = 0 (wave 0, row-owned)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void forward(const Lds L, int N, int out = 3) {
  if ((threadIdx.x >> 6) != 0) return;
  double* const dxo = L.v12(out);  // dx (3), or the refinement's correction
  const int c = opq(threadIdx.x & 15);
  const bool cv = c < 12;
  const int row = cv ? c : 11;
  double xv = 0.0;
  double Ar[12], bv;
  auto load_row = [&](int k, double (&R)[12], double& b) {
    const double* r = L.acl() + k * 156 + row * 13;
    sfor<0, 12>([&](auto j) { R[decltype(j)::value] = r[decltype(j)::value]; });
    b = r[12];
  };
  load_row(0, Ar, bv);
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    if (threadIdx.x < 12) dxo[k * 12 + c] = xv;
    double An[12], bn = 0.0;
    if (k + 1 < N) {
      load_row(k + 1, An, bn);
    } else {
      sfor<0, 12>([&](auto j) { An[decltype(j)::value] = 0.0; });
    }
    const double xn = dot_bcast(Ar, xv, bv);
    xv = cv ? xn : 0.0;
    sfor<0, 12>([&](auto j) { Ar[decltype(j)::value] = An[decltype(j)::value]; });
    bv = bn;
  }
  if (threadIdx.x < 12) dxo[N * 12 + c] = xv;
}

// ---------------------------------------------------------------------------------------------
// phase: the step of every stage from dx (du = K dx + k, dpi = P dx + p, the bounds' dt /
// dlam), the step ratios and the predictor's mu_aff sums.  CORR: k, p of the corrector (kv,
// pv), dlam_aff dt_aff and sigma mu in the complementarity rows.
// ---------------------------------------------------------------------------------------------
template <bool CORR, bool SQRT>
__device__ __forceinline__ void step_pass(const Qp Q, const Lds L, double smu, bool final_step) {
  const ProblemArgsT<double>& a = Q.a;
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  const int jj = el ? j : 11;
  double ap = 1e30, ad = 1e30, s1 = 0.0, s2 = 0.0;
  bool bad = false;
  for (int k = grp; k <= N; k += kGroups) {
    const double* rk = Q.rec(k);
    const double dxj = el ? L.dx()[k * 12 + j] : 0.0;
    double duj = 0.0, dpij = 0.0;
    if (k < N) {
      double Kr[12];
      sfor<0, 12>([&](auto i) { Kr[decltype(i)::value] = rk[kRK + jj * 13 + decltype(i)::value]; });
      const double kvj = CORR ? L.kv()[k * 12 + jj] : rk[kRK + jj * 13 + 12];
      duj = dot_bcast(Kr, dxj, kvj);
      if (!el) duj = 0.0;
    }
    if (k > 0) {
      if constexpr (SQRT) {
        const double pvj = CORR ? L.pv()[k * 12 + jj] : rk[kRp + jj];
        dpij = rec_P_apply<true>(rk + kRP, jj, dxj, pvj);
      } else {
        double Pr[12];
        load_packed_sym(rk + kRP, jj, Pr);
        const double pvj = CORR ? L.pv()[k * 12 + jj] : rk[kRp + jj];
        dpij = dot_bcast(Pr, dxj, pvj);
      }
      if (!el) dpij = 0.0;
    }
    if (el) {
      L.du()[k * 12 + j] = duj;
      L.dpi()[k * 12 + j] = dpij;
    }
    if (final_step) bad |= el && (huge(duj) || huge(dxj) || huge(dpij));
    if (k < N && el) {
      const Side s = side_u(Q, k, j);
      const Bar b = ld_bar(L.bu() + k * 48, j);
      double e1 = 0.0, e2 = 0.0;
      if (CORR) {
        const BarStep p = ld_step(L.su() + k * 48, j);
        e1 = p.dll * p.dtl;
        e2 = p.dlu * p.dtu;
      }
      const BarStep d = bar_step(s, b, L.u()[k * 12 + j], duj, e1, e2, CORR ? smu : 0.0);
      ratio(s, b, d, ap, ad);
      if (!CORR) aff_sums(s, b, d, s1, s2);
      if (final_step) bad |= huge(d.dtl) || huge(d.dtu) || huge(d.dll) || huge(d.dlu);
      st_step(L.su() + k * 48, j, d);
    }
    if (k > 0 && el) {
      const Side s = side_x(Q, k, j);
      const Bar b = ld_bar(L.bx() + k * 48, j);
      double e1 = 0.0, e2 = 0.0;
      if (CORR) {
        const BarStep p = ld_step(L.sx() + k * 48, j);
        e1 = p.dll * p.dtl;
        e2 = p.dlu * p.dtu;
      }
      const BarStep d = bar_step(s, b, L.x()[k * 12 + j], dxj, e1, e2, CORR ? smu : 0.0);
      ratio(s, b, d, ap, ad);
      if (!CORR) aff_sums(s, b, d, s1, s2);
      if (final_step) bad |= huge(d.dtl) || huge(d.dtu) || huge(d.dll) || huge(d.dlu);
      st_step(L.sx() + k * 48, j, d);
    }
    for (int ch = 0; ch < L.nch; ++ch) {
      const int r = ch * 12 + j;
      const bool ok = el && r < a.ng;
      double Dr[12], Cr[12];
      load_strided(ok ? Q.Drow(k, r) : nullptr, a.ng, Dr);
      load_strided(ok ? Q.Crow(k, r) : nullptr, a.ng, Cr);
      const double dv = dot_bcast(Cr, dxj, dot_bcast(Dr, duj, 0.0));
      if (ok) {
        double* g = L.gb(k, ch);
        const Side s = side_g(Q, k, r);
        const Bar b = ld_bar(g, j);
        double e1 = 0.0, e2 = 0.0;
        if (CORR) {
          const BarStep p = ld_step(g + 48, j);
          e1 = p.dll * p.dtl;
          e2 = p.dlu * p.dtu;
        }
        const BarStep d = bar_step(s, b, g[96 + j], dv, e1, e2, CORR ? smu : 0.0);
        ratio(s, b, d, ap, ad);
        if (!CORR) aff_sums(s, b, d, s1, s2);
        if (final_step) bad |= huge(d.dtl) || huge(d.dtu) || huge(d.dll) || huge(d.dlu);
        st_step(g + 48, j, d);
      }
    }
  }
  red_put(L, 0, g16min(ap));
  red_put(L, 1, g16min(ad));
  red_put(L, 2, g16sum(s1));
  red_put(L, 3, g16sum(s2));
  red_put(L, 4, g16max(bad ? 1.0 : 0.0));
}

// ---------------------------------------------------------------------------------------------
// corrector right-hand side.  c_k = g~x_k + K_k' g~u_k + Acl_k' (P_k+1 b~_k) for every stage
// (P_k+1 b~_k kept in dpi), then the recursion p_k = Acl_k' p_k+1 + c_k (wave 0), then per
// stage g_k = B_k'(P_k+1 b~_k + p_k+1) + g~u_k, k_k = -(L L')^-1 g_k, bcl_k = b~_k + B_k k_k.
// (The oracle's p_k = f + K'g with f = A'Pb + g~x, g = B'Pb + g~u, Pb = P b~ + p_k+1.)
// ---------------------------------------------------------------------------------------------
// Right-hand side buffers (v12 indices): the corrector's g~u = gtu, g~x = gtx, b~ = rb, P b~ kept
// in dpi; the refinement's correction: r_u, r_x in gtu, gtx, r_b in kCrb, P r_b in kCpb.
struct Rhs {
  int gu, gx, b, pb;
};
constexpr Rhs kRhsCorr{9, 10, 8, 5};
template <bool SQRT>
__device__ __forceinline__ void corr_rhs_stages(const Qp Q, const Lds L, Rhs h = kRhsCorr) {
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  const int jj = el ? j : 11;
  const double* gu = L.v12(h.gu);
  const double* gx = L.v12(h.gx);
  const double* bt = L.v12(h.b);
  double* pbo = L.v12(h.pb);
  for (int k = grp; k <= N; k += kGroups) {
    if (k == N) {
      if (el) L.pv()[N * 12 + j] = gx[N * 12 + j];
      continue;
    }
    double M[12];
    double pb;
    if constexpr (SQRT) {
      const double bj = el ? bt[k * 12 + j] : 0.0;
      pb = rec_P_apply<true>(Q.rec(k + 1) + kRP, jj, bj, 0.0);
    } else {
      load_packed_sym(Q.rec(k + 1) + kRP, jj, M);
      const double bj = el ? bt[k * 12 + j] : 0.0;
      pb = dot_bcast(M, bj, 0.0);
    }
    if (!el) pb = 0.0;
    const double* rk = Q.rec(k);
    sfor<0, 12>([&](auto i) { M[decltype(i)::value] = rk[kRK + decltype(i)::value * 13 + jj]; });
    double ck = dot_bcast(M, el ? gu[k * 12 + j] : 0.0, el ? gx[k * 12 + j] : 0.0);
    sfor<0, 12>([&](auto i) { M[decltype(i)::value] = L.acl()[k * 156 + decltype(i)::value * 13 + jj]; });
    ck = dot_bcast(M, pb, ck);
    if (el) {
      pbo[k * 12 + j] = pb;
      L.pv()[k * 12 + j] = ck;
    }
  }
}
__device__ __forceinline__ void corr_rhs_chain(const Lds L, int N) {
  if ((threadIdx.x >> 6) != 0) return;
  const int c = opq(threadIdx.x & 15);
  const bool cv = c < 12;
  const int cc = cv ? c : 11;
  double pv = cv ? L.pv()[N * 12 + c] : 0.0;
  double M[12];
  auto load_col = [&](int k, double (&C)[12]) {
    sfor<0, 12>([&](auto i) { C[decltype(i)::value] = L.acl()[k * 156 + decltype(i)::value * 13 + cc]; });
  };
  load_col(N - 1, M);
#pragma unroll 1
  for (int k = N - 1; k >= 0; --k) {
    double Mn[12];
    if (k > 0) {
      load_col(k - 1, Mn);
    } else {
      sfor<0, 12>([&](auto i) { Mn[decltype(i)::value] = 0.0; });
    }
    const double ck = cv ? L.pv()[k * 12 + c] : 0.0;
    const double pn = dot_bcast(M, pv, ck);
    pv = cv ? pn : 0.0;
    if (threadIdx.x < 12) L.pv()[k * 12 + c] = pv;
    sfor<0, 12>([&](auto i) { M[decltype(i)::value] = Mn[decltype(i)::value]; });
  }
}
__device__ __forceinline__ void corr_k_stages(const Qp Q, const Lds L, Rhs h = kRhsCorr) {
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  const int jj = el ? j : 11;
  const double* gu = L.v12(h.gu);
  const double* bt = L.v12(h.b);
  const double* pb = L.v12(h.pb);
  for (int k = grp; k < N; k += kGroups) {
    double M[12];
    load12(Q.B(k) + jj * 12, M);
    const double w = el ? pb[k * 12 + j] + L.pv()[(k + 1) * 12 + j] : 0.0;
    double gk = dot_bcast(M, w, el ? gu[k * 12 + j] : 0.0);
    if (!el) gk = 0.0;
    // k = -(L L')^-1 g: L's columns on lanes 0..11, the right-hand side on lane 12
    const double* rk = Q.rec(k);
    double Lc[12], Gv[12], Kc[12];
    load_packed_lcol(rk + kRL, jj, Lc);
    const double rs = rk[kRrs + jj];
    sfor<0, 12>([&](auto i) { Gv[decltype(i)::value] = bc<decltype(i)::value>(gk); });
    trsv_lower(Lc, rs, Gv);
    trsv_upper_t_neg_axpy(Lc, rs, Gv, Kc);
    double kk = 0.0;
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      const double v = bc<12>(Kc[I]);
      kk = j == I ? v : kk;
    });
    // bcl_k = b~_k + B_k k_k (row j of B)
    load_strided(Q.B(k) + jj, 12, M);
    const double bcl = dot_bcast(M, kk, el ? bt[k * 12 + j] : 0.0);
    if (el) {
      L.kv()[k * 12 + j] = kk;
      L.acl()[k * 156 + j * 13 + 12] = bcl;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// iterative refinement of the step (HPIPM itref_corr_max: Balance 2, Robust 4; the batched
// kernels' kPhIR / kPhIS / kPhF3, oracle lin_res).  The check: the linear residual of the Newton
// system at the step (du, dx, dpi and the barrier steps) in its full form -- QP Hessian,
// multiplier steps, dynamics; the dt / dlam rows hold by construction --
//   r_u = res_g,u + R du + S dx + B'dpi_k+1 + (dlam_u - dlam_l)_u + D'(dlam_u - dlam_l)_rows
//   r_x = res_g,x + S'du + Q dx + A'dpi_k+1 - dpi_k + (..)_x + C'(..)_rows        (k >= 1)
//   r_b = res_b + A dx + B du - dx_k+1                                          (k < N)
// into gtu, gtx (dead after the corrector) and the other x buffer; its infinity norms to red
// slots 0, 1.
// ---------------------------------------------------------------------------------------------
template <bool HAS_C>
__device__ __forceinline__ void lin_res_pass(const Qp Q, const Lds L) {
  const ProblemArgsT<double>& a = Q.a;
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  const int jj = el ? j : 11;
  double ng = 0.0, nb = 0.0;
  for (int k = grp; k <= N; k += kGroups) {
    const double duj = (el && k < N) ? L.du()[k * 12 + j] : 0.0;
    const double dxj = (el && k > 0) ? L.dx()[k * 12 + j] : 0.0;
    const double dpnj = (el && k < N) ? L.dpi()[(k + 1) * 12 + j] : 0.0;
    double ru = el ? L.rgu()[k * 12 + j] : 0.0;
    double rx = el ? L.rgx()[k * 12 + j] - L.dpi()[k * 12 + j] : 0.0;
    if (el && k < N) {
      const Side s = side_u(Q, k, j);
      const BarStep d = ld_step(L.su() + k * 48, j);
      ru += s.mu * d.dlu - s.ml * d.dll;
    }
    if (el && k > 0) {
      const Side s = side_x(Q, k, j);
      const BarStep d = ld_step(L.sx() + k * 48, j);
      rx += s.mu * d.dlu - s.ml * d.dll;
    }
    for (int ch = 0; ch < L.nch; ++ch) {
      const int r = ch * 12 + j;
      const bool ok = el && r < a.ng;
      double dl = 0.0;
      if (ok) {
        const Side sg = side_g(Q, k, r);
        const BarStep d = ld_step(L.gb(k, ch) + 48, j);
        dl = sg.mu * d.dlu - sg.ml * d.dll;
      }
      double Yc[12];
      gen_col<false>(Q, k, ch, jj, el, Yc);
      ru = dot_bcast(Yc, dl, ru);
      if constexpr (HAS_C) {
        gen_col<true>(Q, k, ch, jj, el, Yc);
        rx = dot_bcast(Yc, dl, rx);
      }
    }
    double M[12];
    double rb = 0.0;
    if (k < N) {
      load12(Q.R(k) + jj * 12, M);
      ru = dot_bcast(M, duj, ru);  // + R du
      load_strided(Q.S(k) + jj, 12, M);
      ru = dot_bcast(M, dxj, ru);  // + S dx
      load12(Q.B(k) + jj * 12, M);
      ru = dot_bcast(M, dpnj, ru);  // + B'dpi_k+1
      load12(Q.S(k) + jj * 12, M);
      rx = dot_bcast(M, duj, rx);  // + S'du
      load12(Q.A(k) + jj * 12, M);
      rx = dot_bcast(M, dpnj, rx);  // + A'dpi_k+1
      load_strided(Q.A(k) + jj, 12, M);
      rb = dot_bcast(M, dxj, el ? L.rb()[k * 12 + j] - L.dx()[(k + 1) * 12 + j] : 0.0);  // + A dx
      load_strided(Q.B(k) + jj, 12, M);
      rb = dot_bcast(M, duj, rb);  // + B du
    }
    load12(Q.Q(k) + jj * 12, M);
    rx = dot_bcast(M, dxj, rx);  // + Q dx
    if (!(el && k < N)) ru = 0.0;
    if (!(el && k > 0)) rx = 0.0;  // (x_0 is fixed)
    if (!(el && k < N)) rb = 0.0;
    ng = fmax(ng, fmax(nabs(ru), nabs(rx)));
    nb = fmax(nb, nabs(rb));
    if (el) {
      L.gtu()[k * 12 + j] = ru;
      L.gtx()[k * 12 + j] = rx;
      L.v12(L.ref_b())[k * 12 + j] = rb;
    }
  }
  red_put(L, 0, g16max(ng));
  red_put(L, 1, g16max(nb));
}

// The correction (solved by the corrector's recursion on the check's residual: ddx in gtu, k, p
// of the correction in kv, pv) added to the step: du += K ddx + k, dx += ddx, dpi += P ddx + p;
// the barrier steps are linear in the primal step (ddt = +-ddv, ddlam = -lam ddt / t); then the
// step ratios of the whole step and the non-finite check, as step_pass leaves them.
template <bool SQRT>
__device__ __forceinline__ void corr_apply_pass(const Qp Q, const Lds L) {
  const ProblemArgsT<double>& a = Q.a;
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  const int jj = el ? j : 11;
  double ap = 1e30, ad = 1e30;
  bool bad = false;
  auto upd = [&](const Side& sd, const Bar& b, BarStep& d, double dv) {
    if (sd.ml != 0.0) {
      d.dtl += dv;
      d.dll -= b.ll * dv / b.tl;
    }
    if (sd.mu != 0.0) {
      d.dtu -= dv;
      d.dlu += b.lu * dv / b.tu;
    }
  };
  const double* cdx = L.v12(Lds::kRefDx);
  for (int k = grp; k <= N; k += kGroups) {
    const double* rk = Q.rec(k);
    const double cxj = el ? cdx[k * 12 + j] : 0.0;
    double cuj = 0.0, cpj = 0.0;
    if (k < N) {
      double Kr[12];
      sfor<0, 12>([&](auto i) { Kr[decltype(i)::value] = rk[kRK + jj * 13 + decltype(i)::value]; });
      cuj = dot_bcast(Kr, cxj, L.kv()[k * 12 + jj]);
      if (!el) cuj = 0.0;
    }
    if (k > 0) {
      if constexpr (SQRT) {
        cpj = rec_P_apply<true>(rk + kRP, jj, cxj, L.pv()[k * 12 + jj]);
      } else {
        double Pr[12];
        load_packed_sym(rk + kRP, jj, Pr);
        cpj = dot_bcast(Pr, cxj, L.pv()[k * 12 + jj]);
      }
      if (!el) cpj = 0.0;
    }
    if (el) {
      double duj = 0.0;
      if (k < N) {
        duj = L.du()[k * 12 + j] + cuj;
        L.du()[k * 12 + j] = duj;
      }
      const double dxj = L.dx()[k * 12 + j] + cxj;
      L.dx()[k * 12 + j] = dxj;
      double dpj = 0.0;
      if (k > 0) {
        dpj = L.dpi()[k * 12 + j] + cpj;
        L.dpi()[k * 12 + j] = dpj;
      }
      bad |= huge(duj) || huge(dxj) || huge(dpj);
    }
    if (k < N && el) {
      const Side s = side_u(Q, k, j);
      const Bar b = ld_bar(L.bu() + k * 48, j);
      BarStep d = ld_step(L.su() + k * 48, j);
      upd(s, b, d, cuj);
      ratio(s, b, d, ap, ad);
      bad |= huge(d.dtl) || huge(d.dtu) || huge(d.dll) || huge(d.dlu);
      st_step(L.su() + k * 48, j, d);
    }
    if (k > 0 && el) {
      const Side s = side_x(Q, k, j);
      const Bar b = ld_bar(L.bx() + k * 48, j);
      BarStep d = ld_step(L.sx() + k * 48, j);
      upd(s, b, d, cxj);
      ratio(s, b, d, ap, ad);
      bad |= huge(d.dtl) || huge(d.dtu) || huge(d.dll) || huge(d.dlu);
      st_step(L.sx() + k * 48, j, d);
    }
    for (int ch = 0; ch < L.nch; ++ch) {
      const int r = ch * 12 + j;
      const bool ok = el && r < a.ng;
      double Dr[12], Cr[12];
      load_strided(ok ? Q.Drow(k, r) : nullptr, a.ng, Dr);
      load_strided(ok ? Q.Crow(k, r) : nullptr, a.ng, Cr);
      const double dv = dot_bcast(Cr, cxj, dot_bcast(Dr, cuj, 0.0));
      if (ok) {
        double* g = L.gb(k, ch);
        const Side s = side_g(Q, k, r);
        const Bar b = ld_bar(g, j);
        BarStep d = ld_step(g + 48, j);
        upd(s, b, d, dv);
        ratio(s, b, d, ap, ad);
        bad |= huge(d.dtl) || huge(d.dtu) || huge(d.dll) || huge(d.dlu);
        st_step(g + 48, j, d);
      }
    }
  }
  red_put(L, 0, g16min(ap));
  red_put(L, 1, g16min(ad));
  red_put(L, 4, g16max(bad ? 1.0 : 0.0));
}

// ---------------------------------------------------------------------------------------------
// phase: outputs (ipm_box_impl.h kPhOut): x, u, pi with the stage-0 rebuild
// pi_0 = Q0 x0 + S0'u0 + q0 + A0'(P_1 res_b0 + pi_1) (ocp_qp_ipm_solver.cpp:347-373), and the
// Riccati getters of the last factorization: P, K; p = pi - P x, k = u - K x
// ---------------------------------------------------------------------------------------------
template <bool SQRT>
__device__ __forceinline__ void outputs(const Qp Q, const Lds L) {
  const ProblemArgsT<double>& a = Q.a;
  const int N = Q.N, grp = opq(threadIdx.x >> 4), j = opq(threadIdx.x & 15);
  const bool el = j < 12;
  const int jj = el ? j : 11;
  const size_t q = (size_t)Q.q;
  for (int k = grp; k <= N; k += kGroups) {
    const double* rk = Q.rec(k);
    const double xj = el ? L.x()[k * 12 + j] : 0.0;
    const double uj = (el && k < N) ? L.u()[k * 12 + j] : 0.0;
    double pij = el ? L.pi()[k * 12 + j] : 0.0;
    if (k == 0) {
      double M[12];
      double t;
      if constexpr (SQRT) {
        t = rec_P_apply<true>(Q.rec(1) + kRP, jj, el ? L.rb()[j] : 0.0, el ? L.pi()[12 + j] : 0.0);
      } else {
        load_packed_sym(Q.rec(1) + kRP, jj, M);
        t = dot_bcast(M, el ? L.rb()[j] : 0.0, el ? L.pi()[12 + j] : 0.0);
      }
      if (!el) t = 0.0;
      load12(Q.Q(0) + jj * 12, M);
      double p0 = dot_bcast(M, xj, el ? Q.qv(0)[j] : 0.0);
      load12(Q.S(0) + jj * 12, M);
      p0 = dot_bcast(M, uj, p0);
      load12(Q.A(0) + jj * 12, M);
      p0 = dot_bcast(M, t, p0);
      pij = el ? p0 : 0.0;
    }
    if (el) {
      a.x[(q * (N + 1) + k) * 12 + j] = xj;
      a.pi[(q * (N + 1) + k) * 12 + j] = pij;
      if (k < N) a.u[(q * N + k) * 12 + j] = uj;
    }
    if (a.P || a.p) {
      double Pr[12];
      if constexpr (SQRT) {  // P = Lp Lp': column jj = sum_K Lp[:, K] Lp[jj][K]
        double Lr[12];
        load_packed_lrow_d(rk + kRP, jj, Lr);
        sfor<0, 12>([&](auto i) { Pr[decltype(i)::value] = 0.0; });
        tmul_acc(Lr, Lr, Pr);
      } else {
        load_packed_sym(rk + kRP, jj, Pr);
      }
      double px;
      if constexpr (SQRT) {
        px = rec_P_apply<true>(rk + kRP, jj, xj, 0.0);
      } else {
        px = dot_bcast(Pr, xj, 0.0);
      }
      if (el && a.P) store12(a.P + (q * (N + 1) + k) * 144 + (size_t)j * 12, Pr);
      if (el && a.p) a.p[(q * (N + 1) + k) * 12 + j] = pij - px;
    }
    if (k < N && (a.K || a.k)) {
      double Kr[12];
      sfor<0, 12>([&](auto i) { Kr[decltype(i)::value] = rk[kRK + jj * 13 + decltype(i)::value]; });
      const double kx = dot_bcast(Kr, xj, 0.0);
      if (el && a.k) a.k[(q * N + k) * 12 + j] = uj - kx;
      if (el && a.K) {
        double Kc[12];
        sfor<0, 12>([&](auto i) { Kc[decltype(i)::value] = rk[kRK + decltype(i)::value * 13 + j]; });
        store12(a.K + (q * N + k) * 144 + (size_t)j * 12, Kc);
      }
    }
  }
}

// ITREF: HPIPM's iterative refinement of the step (Balance / Robust; a separate instantiation so
// the Speed path keeps its registers)
// SQRT: ric_alg 1 (factorize<true>, the records' P slot holding the factor Lp), with lq_fact 1's
// check of the predictor (HPIPM switches such a QP to the LQ factorization, which this kernel does
// not have: it raises a.lat_lq_flag and the C-ABI solves the batch again on the batched kernels).
template <bool HAS_C, bool ITREF, bool SQRT>
__global__ void __launch_bounds__(kThreads, 1) ipm_latency_kernel(ProblemArgsT<double> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const int N = a.N;
  const int nch = (a.ng + 11) / 12;
  Lds L = carve(reinterpret_cast<double*>(lds_raw), N, nch);
  const Qp Q{a, (int)blockIdx.x, N};
  const bool t0 = threadIdx.x == 0;
  double* const stat = a.stat ? a.stat + (size_t)Q.q * a.stat_rows * kStatCols : nullptr;

  tstamp(63);
  init_point(Q, L);
  __syncthreads();
  tstamp(64);
  const double nc = uni(red_sum(L, 0));
  const double nc_inv = uni(nc > 0.0 ? 1.0 / nc : 0.0);
  double last_amin = 1.0, res_g = 0.0, res_b = 0.0, res_d = 0.0, res_m = 0.0, obj = 0.0;
  double alpha_p = 0.0, alpha_d = 0.0;  // the step the next stage pass applies (none at first)
  int iter = 0, status = -1;
#pragma unroll 1
  for (;;) {
    __syncthreads();  // (red reuse)
    tstamp(50);
    stage_pass<HAS_C, true, SQRT>(Q, L, alpha_p, alpha_d);
    __syncthreads();
    L.cur ^= 1;  // the new iterate
    tstamp(51);
    res_g = uni(red_max(L, 0));
    res_b = uni(red_max(L, 1));
    res_d = uni(red_max(L, 2));
    res_m = uni(red_max(L, 3));
    const double musum = uni(red_sum(L, 4));
    obj = uni(red_sum(L, 5));
    const double mu = uni(musum * nc_inv);
    if (stat && t0) {
      double* row = stat + (size_t)iter * kStatCols;
      row[5] = mu;
      row[6] = res_g;
      row[7] = res_b;
      row[8] = res_d;
      row[9] = res_m;
      row[10] = obj;
    }
    // exit test (HPIPM order: NaN / converged / iter_max / min step)
    if (!(res_g == res_g) || !(res_b == res_b) || !(res_d == res_d) || !(res_m == res_m) || !(mu == mu) ||
        res_g == __builtin_inf() || res_b == __builtin_inf()) {
      status = 3;
    } else if (res_g <= a.tol_stat && res_b <= a.tol_eq && res_d <= a.tol_ineq && res_m <= a.tol_comp) {
      status = 0;
    } else if (iter >= a.iter_max) {
      status = 1;
    } else if (iter > 0 && last_amin < a.alpha_min) {
      status = 2;
    }
    if (status >= 0) break;
    double* const next = (stat && t0) ? stat + (size_t)(iter + 1) * kStatCols : nullptr;

    // ---- predictor (the stage blocks are in the records: stage_pass) ----
    factorize<SQRT>(Q, L);
    __syncthreads();
    tstamp(53);
    forward(L, N);
    __syncthreads();
    tstamp(54);
    const bool pc = a.pred_corr != 0;
    step_pass<false, SQRT>(Q, L, 0.0, !pc);
    __syncthreads();
    tstamp(55);
    double ap = uni(red_min(L, 0)), ad = uni(red_min(L, 1));
    bool bad = uni(red_max(L, 4)) > 0.0;
    if constexpr (SQRT) {
      if (a.lq_fact == 1) {
        // HPIPM lq_fact 1 (d_ocp_qp_ipm_solve): the predictor step's linear residual above 1e-5
        // (or NaN) switches the QP to the LQ factorization -- not built here: leave, and let the
        // C-ABI solve the batch on the batched kernels (ipm_box_impl.h kPhIRP / kPhLqChk).  The
        // check's buffers (gtu, gtx, the other x / pi) are dead here; its slots 0, 1 are the
        // step ratios, already read (slots 2, 3 hold the mu_aff sums, untouched).
        __syncthreads();
        lin_res_pass<HAS_C>(Q, L);
        __syncthreads();
        const double ngr = uni(red_max(L, 0)), nbr = uni(red_max(L, 1));
        if (!(ngr <= 1e-5) || !(nbr <= 1e-5)) {
          status = kLatNeedsLq;
          if (t0 && a.lat_lq_flag) __hip_atomic_store(a.lat_lq_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    if (pc) {
      const double aa = fmin(1.0, fmin(ap, ad));
      const double S1 = uni(red_sum(L, 2)), S2 = uni(red_sum(L, 3));
      const double mu_aff = (musum + aa * (S1 + aa * S2)) * nc_inv;
      double sg = mu > 0.0 ? mu_aff / mu : 0.0;
      sg = sg * sg * sg;
      if (sg > 1.0) sg = 1.0;
      const double smu = uni(sg * mu);
      if (next) {
        next[0] = aa;
        next[1] = mu_aff;
        next[2] = sg;
      }
      // ---- corrector: same factors, new gradient ----
      __syncthreads();
      corr_terms<HAS_C>(Q, L, smu);
      __syncthreads();
      tstamp(56);
      corr_rhs_stages<SQRT>(Q, L);
      __syncthreads();
      tstamp(57);
      corr_rhs_chain(L, N);
      __syncthreads();
      tstamp(58);
      corr_k_stages(Q, L);
      __syncthreads();
      tstamp(59);
      forward(L, N);
      __syncthreads();
      tstamp(60);
      step_pass<true, SQRT>(Q, L, smu, true);
      __syncthreads();
      tstamp(61);
      ap = uni(red_min(L, 0));
      ad = uni(red_min(L, 1));
      bad = uni(red_max(L, 4)) > 0.0;
    }
    // ---- iterative refinement of the final step (Balance / Robust) ----
    if (ITREF && a.itref_corr_max > 0) {
      double n0g = 0.0, n0b = 0.0;
      int cnt = 0;
#pragma unroll 1
      for (int ir = 0; ir < a.itref_corr_max; ++ir) {
        __syncthreads();  // (red reuse)
        lin_res_pass<HAS_C>(Q, L);
        __syncthreads();
        const double ngr = uni(red_max(L, 0)), nbr = uni(red_max(L, 1));
        if (ir == 0) {
          n0g = ngr;
          n0b = nbr;
        }
        if (next) {  // HPIPM stat: lin_res_stat, lin_res_eq of the last check
          next[14] = ngr;
          next[15] = nbr;
        }
        if ((ngr < a.tol_stat || ngr < 1e-3 * n0g) && (nbr < a.tol_eq || nbr < 1e-3 * n0b)) break;
        // the correction: the corrector's recursion with (r_u, r_x, r_b) as right-hand side
        const Rhs ref{9, 10, L.ref_b(), L.ref_pb()};
        corr_rhs_stages<SQRT>(Q, L, ref);
        __syncthreads();
        corr_rhs_chain(L, N);
        __syncthreads();
        corr_k_stages(Q, L, ref);
        __syncthreads();
        forward(L, N, Lds::kRefDx);
        __syncthreads();
        corr_apply_pass<SQRT>(Q, L);
        __syncthreads();
        ap = uni(red_min(L, 0));
        ad = uni(red_min(L, 1));
        bad = uni(red_max(L, 4)) > 0.0;
        ++cnt;
        if (next) next[13] = cnt;  // HPIPM stat: itref_corr
      }
    }
    if (bad) {
      ap = 0.0;
      ad = 0.0;
    }
    if (!a.split_step) {
      ap = fmin(ap, ad);
      ad = ap;
    }
    alpha_p = uni(fmin(1.0, kTau * ap));
    alpha_d = uni(fmin(1.0, kTau * ad));
    if (next) {
      next[3] = alpha_p;
      next[4] = alpha_d;
    }
    last_amin = uni(fmin(alpha_p, alpha_d));
    ++iter;
  }
  // decided at the initial point (converged, or NaN data): the factorization of the returned
  // iterate, as the batched kernels' exiting sweep has it (HPIPM getters and the stage-0 pi
  // rebuild read it; its stage blocks are in the records: stage_pass)
  if (iter == 0 && status != kLatNeedsLq) factorize<SQRT>(Q, L);
  __syncthreads();
  tstamp(65);
  outputs<SQRT>(Q, L);
  __syncthreads();
  tstamp(66);
  if (t0) {
    if (a.status) a.status[Q.q] = status;
    if (a.iter) a.iter[Q.q] = nc > 0.0 ? iter : 0;
    if (a.res) {
      a.res[(size_t)Q.q * 4 + 0] = res_g;
      a.res[(size_t)Q.q * 4 + 1] = res_b;
      a.res[(size_t)Q.q * 4 + 2] = res_d;
      a.res[(size_t)Q.q * 4 + 3] = res_m;
    }
    if (a.obj) a.obj[Q.q] = obj;
  }
}

}  // namespace ipm_lat

bool ipm_latency_ok(const ProblemArgsT<double>& a, int max_batch) {
  if (a.batch < 1 || a.batch > max_batch) return false;
  if (a.nx != 12 || a.nu != 12 || a.N < 1) return false;
  // ric_alg 1 with lq_fact 0, or 1 with the switch flag (the kernel checks the predictor and
  // flags a switch to LQ, a.lat_lq_flag; not with a warm start: the re-solve after a switch would
  // find the first attempt's x, u in the buffers the warm start reads); lq_fact 2 (Robust with
  // the square root) factorizes by LQ throughout: batched kernels
  if (a.lq_fact > 1 || (a.lq_fact == 1 && (!a.lat_lq_flag || a.warm_start)) || a.warm_start > 1 || a.warm_bars ||
      a.skip_last_rb)
    return false;
  // the square root with C rows measured weaker than the batched kernels' (round 6: 2 of 12 random
  // QPs with C and D rows stopped at min step, iteration counts +2 against the oracle's): those
  // stay on the batched kernels; C-free rows (the friction cone) and boxes run here
  if (!SRBD_LAT_SQRT_C && a.ric_alg && a.C && a.ng > 0) return false;
  const int nch = (a.ng + 11) / 12;
  if (ipm_lat::lds_doubles(a.N, nch) * sizeof(double) > 160 * 1024) return false;
  return a.ws && a.ws_qp >= (size_t)(a.N + 1) * ipm_lat::kRStage;
}

hipError_t launch_ipm_latency(const ProblemArgsT<double>& a, hipStream_t stream) {
  // (the LDS limit is set once per device: prepare_ipm_latency_device, srbd_qp_create)
  const int nch = (a.ng + 11) / 12;
  const size_t bytes = ipm_lat::lds_doubles(a.N, nch) * sizeof(double);
  const dim3 grid(a.batch), block(ipm_lat::kThreads);
  const int v = (a.C && a.ng > 0 ? 4 : 0) | (a.itref_corr_max > 0 ? 2 : 0) | (a.ric_alg ? 1 : 0);
  switch (v) {
#define SRBD_LAT_CASE(V, C, I, Q) \
  case V: hipLaunchKernelGGL((ipm_lat::ipm_latency_kernel<C, I, Q>), grid, block, bytes, stream, a); break;
    SRBD_LAT_CASE(0, false, false, false)
    SRBD_LAT_CASE(1, false, false, true)
    SRBD_LAT_CASE(2, false, true, false)
    SRBD_LAT_CASE(3, false, true, true)
    SRBD_LAT_CASE(4, true, false, false)
    SRBD_LAT_CASE(6, true, true, false)
#if SRBD_LAT_SQRT_C
    SRBD_LAT_CASE(5, true, false, true)
    SRBD_LAT_CASE(7, true, true, true)
#endif
#undef SRBD_LAT_CASE
  }
  return hipGetLastError();
}

// Per-device attribute (hipFuncSetAttribute costs tens of microseconds: once per handle, on
// the handle's device, like prepare_riccati_device)
hipError_t prepare_ipm_latency_device() {
  constexpr int kBytes = 160 * 1024;
  const void* fns[] = {reinterpret_cast<const void*>(&ipm_lat::ipm_latency_kernel<true, false, false>),
                       reinterpret_cast<const void*>(&ipm_lat::ipm_latency_kernel<false, false, false>),
                       reinterpret_cast<const void*>(&ipm_lat::ipm_latency_kernel<true, true, false>),
                       reinterpret_cast<const void*>(&ipm_lat::ipm_latency_kernel<false, true, false>),
                       reinterpret_cast<const void*>(&ipm_lat::ipm_latency_kernel<false, false, true>),
                       reinterpret_cast<const void*>(&ipm_lat::ipm_latency_kernel<false, true, true>),
#if SRBD_LAT_SQRT_C
                       reinterpret_cast<const void*>(&ipm_lat::ipm_latency_kernel<true, false, true>),
                       reinterpret_cast<const void*>(&ipm_lat::ipm_latency_kernel<true, true, true>),
#endif
  };
  hipError_t e = hipSuccess;
  for (const void* f : fns)
    if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kBytes);
  return e;
}

}  // namespace srbd

#if SRBD_TSTAMP
// Diagnostic builds only: this translation unit's stamp buffer (the latency IPM), as
// srbd_qp_diag_tstamps does for the unconstrained kernels.
extern "C" int srbd_qp_diag_tstamps_lat(unsigned long long* out, int cap) {
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
