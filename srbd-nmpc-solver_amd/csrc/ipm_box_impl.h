// ipm_box_impl.h -- body of the batched IPM, instantiated once per precision by
// ipm_box.hip (SRBD_REAL = double / float, namespace SRBD_NS), the way HPIPM
// generates its d_ and s_ solvers from one source.  No include guard: included twice.
// The kernel code is documented in ipm_box.hip.

namespace srbd {
namespace SRBD_NS {

using real = SRBD_REAL;

constexpr real kThr0 = real(0.1);     // minimum initial slack (HPIPM init_var)

// phase kernels (one launch each, per IPM iteration; see launch_ipm_box)
constexpr int kPhInit = 0, kPhRB = 1, kPhF1 = 2, kPhB2 = 3, kPhF2 = 4, kPhOut = 5;
// iterative refinement of the corrector step: IR = residual of the step's linear system
// and the check, IS = the correction's backward recursion, F3 = its forward sweep
constexpr int kPhIR = 6, kPhF3 = 7, kPhIS = 8;
// HPIPM lq_fact 1: the predictor step's linear residual (IRP, IR's arithmetic) and the switch
constexpr int kPhIRP = 9, kPhLqChk = 10;
constexpr real kLqSwitch = real(1e-5);  // d_ocp_qp_ipm_solve: refactorize by LQ above this
// per-QP scalar state, kQsSize reals at the head of the QP's workspace
constexpr int kQsAlphaP = 0, kQsAlphaD = 1, kQsLastAmin = 2, kQsMu = 3, kQsMuSum = 4,
              kQsSigmaMu = 5, kQsStatus = 6, kQsIter = 7, kQsNc = 8, kQsResStat = 9,
              kQsResEq = 10, kQsResIneq = 11, kQsResComp = 12, kQsObj = 13,
              // iterative refinement of this iteration's step: corrections applied, done flag,
              // the first check's linear-residual norms (HPIPM's itref_qp_norm0)
              kQsItCnt = 14, kQsItDone = 15, kQsItN0g = 16, kQsItN0b = 17,
              // HPIPM lq_fact: the stage factorizations are LQ (sticky: lq_fact 2 from the start,
              // lq_fact 1 once a predictor's linear residual exceeded 1e-5), and the pending redo
              // of this iteration's factorization + predictor by LQ (lq_fact 1)
              kQsForceLq = 18, kQsLqRedo = 19, kQsSize = 20;
constexpr real kStepTau = real(0.995);  // fraction to the boundary

__device__ __forceinline__ real gsum(real v) {
  v += __shfl_xor(v, 8, kGroup);
  v += __shfl_xor(v, 4, kGroup);
  v += __shfl_xor(v, 2, kGroup);
  v += __shfl_xor(v, 1, kGroup);
  return v;
}
__device__ __forceinline__ real gmax(real v) {
  v = fmax(v, __shfl_xor(v, 8, kGroup));
  v = fmax(v, __shfl_xor(v, 4, kGroup));
  v = fmax(v, __shfl_xor(v, 2, kGroup));
  v = fmax(v, __shfl_xor(v, 1, kGroup));
  return v;
}
__device__ __forceinline__ real gmin(real v) {
  v = fmin(v, __shfl_xor(v, 8, kGroup));
  v = fmin(v, __shfl_xor(v, 4, kGroup));
  v = fmin(v, __shfl_xor(v, 2, kGroup));
  v = fmin(v, __shfl_xor(v, 1, kGroup));
  return v;
}
// NaN, or too large to square in this precision (sqrt(max) / 1e4: 1.8e15 in fp32)
__device__ __forceinline__ bool huge(real v) {
  constexpr real kHuge = sizeof(real) == 4 ? real(1.8e15) : real(1.3e150);
  return !(__builtin_fabs(v) < kHuge);
}
// v + a d, with a = 0 (no step taken) leaving v as it is whatever d holds
__device__ __forceinline__ real step(real v, real a, real d) { return a != real(0.0) ? fmadd(a, d, v) : v; }
// |v| propagating NaN (max with NaN would drop it)
__device__ __forceinline__ real nabs(real v) { return v == v ? fabs(v) : real(__builtin_inf()); }

template <typename T>
__device__ __forceinline__ T dot12(const T (&a)[12], const T (&b)[12], T acc) {
  sfor<0, 12>([&](auto j) {
    constexpr int J = decltype(j)::value;
    acc = fmadd(a[J], b[J], acc);
  });
  return acc;
}

// barrier state of one variable: lam_l, lam_u, t_l, t_u
struct Bar {
  real ll, lu, tl, tu;
};
__device__ __forceinline__ Bar load_bar(const real* stk, int which, int i) {
  const real* p = stk + kStLam + which * 48;
  return Bar{p[i], p[12 + i], p[24 + i], p[36 + i]};
}
__device__ __forceinline__ void store_bar(real* stk, int which, int i, const Bar& b) {
  real* p = stk + kStLam + which * 48;
  p[i] = b.ll;
  p[12 + i] = b.lu;
  p[24 + i] = b.tl;
  p[36 + i] = b.tu;
}
// step of one variable's barrier pair: dt_l, dt_u, dlam_l, dlam_u
struct BarStep {
  real dtl, dtu, dll, dlu;
};
__device__ __forceinline__ BarStep load_bstep(const real* stk, int which, int i) {
  const real* p = stk + kStDlt + which * 48;
  return BarStep{p[i], p[12 + i], p[24 + i], p[36 + i]};
}
__device__ __forceinline__ void store_bstep(real* stk, int which, int i, const BarStep& d) {
  real* p = stk + kStDlt + which * 48;
  p[i] = d.dtl;
  p[12 + i] = d.dtu;
  p[24 + i] = d.dll;
  p[36 + i] = d.dlu;
}

// One inequality side on one variable (box bound, dense per variable).
struct Side {
  real lb, ub;   // bounds
  real ml, mu;   // 1 if the lower / upper bound is active, else 0
};

// Barrier state of one variable / row from a warm-start buffer (p[0] lam_l, p[12] lam_u,
// p[24] t_l, p[36] t_u): the stored values on active sides, the cold init's defaults
// (lam 0, t 1) on inactive ones -- whatever the buffer holds there (an fp32 pass never
// steps the state of a bound family the problem does not have) is not taken over.
__device__ __forceinline__ Bar warm_bar(const real* p, const Side& s) {
  const bool l = s.ml != real(0.0), u = s.mu != real(0.0);
  return Bar{l ? p[0] : real(0.0), u ? p[12] : real(0.0), l ? p[24] : real(1.0), u ? p[36] : real(1.0)};
}

// The RB sweep's per-group LDS blocks (A, B, S: 3 x 144 reals per QP group).  One
// function, so one allocation per kernel: the fused RB -> F1 kernel's F1 reuses them.
// RB also stages each stage's factor record there (kRecSize reals) once the blocks are dead
// (kRecImg: the box kernels and the fp32 general-row kernels; the fp64 general-row ones, at
// their register limit, store the record directly).
// The record is 348 reals, below the block's 432 since the open-loop sweeps (round 3), so the
// fp32 general-row kernels stage it too with no more LDS: cone fp32 N = 40 175.4 vs 180.2 ms
// (round 6, same-box A/B against direct stores, profiles/round6/ab_recimg_cone_n40_f32.log).
// The fp64 general-row kernels (not benchmarked; they spill) keep direct stores.
template <int GEN>
constexpr bool kRecImg = GEN == 0 || sizeof(real) == 4;
template <int GEN>
constexpr int kGroupLds = kRecImg<GEN> && kRecSize > 3 * 144 ? kRecSize : 3 * 144;
template <int GEN>
__device__ __forceinline__ real* group_lds_blocks() {
  __shared__ __attribute__((aligned(16))) real blocks[(256 / kGroup) * kGroupLds<GEN>];
  return blocks + (threadIdx.x / kGroup) * kGroupLds<GEN>;
}

// B2 takes P_{k+1} b~_k from the record (kRecPb, written by RB) instead of reading P_{k+1}
// back: classical Riccati in fp64 (box-u 77.16 -> 76.35 ms same-box); the fp32 general-row RB
// is at its register limit and spilled 12 B/lane more for it (cone fp32 +1.1%), the square root
// records Lp and multiplies it out in B2 as before.
template <bool SQRT>
constexpr bool kRecPbOn = !SQRT && sizeof(real) == 8;

// A factor record from the group's LDS image to the workspace as whole 16-byte pieces
// (16 lanes x 16 B per instruction; box-u 79.3 -> 76.5 ms same-box).  Plain stores: F1, B2
// and F2 read the record again within the iteration (non-temporal stores of stages >= 4
// measured the same).
__device__ __forceinline__ void rec_copy(real* rec, const real* img, int lane) {
  typedef real v4 __attribute__((ext_vector_type(16 / sizeof(real))));
  constexpr int kPieces = kRecSize * (int)sizeof(real) / 16;
  static_assert(kRecSize * sizeof(real) % 16 == 0, "whole pieces");
  const v4* s = reinterpret_cast<const v4*>(img);
  v4* d = reinterpret_cast<v4*>(rec);
  for (int p = lane; p < kPieces; p += kGroup) d[p] = s[p];
}

template <bool FULL, int GEN>
struct Ctx {
  int N, nx, nu, lane, qp;
  bool isv;
  int ng, nch;    // general rows, 12-row chunks
  size_t stride;  // workspace doubles per stage
  size_t ws_qp;   // workspace doubles per QP
  // Batch base pointers (wave-uniform, SGPRs).  The per-QP pointers below are
  // recomputed at every use from an opaque copy of qp, so the compiler cannot
  // hoist ~27 64-bit per-lane pointers into VGPRs for the whole kernel.
  const real *bA, *bB, *bb, *bQ, *bS, *bR, *bq, *br, *bx0;
  const real *blbu, *bubu, *blbum, *bubum, *blbx, *bubx, *blbxm, *bubxm;
  const real *bC, *bD, *blg, *bug, *blgm, *bugm;
  real *bxo, *buo, *bpi, *bws;

  __device__ size_t oq() const {
    int v = qp;
    asm("" : "+v"(v));
    return (size_t)v;
  }
  __device__ size_t iq() const { return oq(); }  // input QP index
  __device__ size_t sN() const { return iq() * N; }
  __device__ size_t sN1() const { return iq() * (N + 1); }
  __device__ size_t oN() const { return oq() * N; }
  __device__ size_t oN1() const { return oq() * (N + 1); }
  __device__ const real* A() const { return bA + sN() * nxx(); }
  __device__ const real* B() const { return bB + sN() * nxu(); }
  __device__ const real* b() const { return bb + sN() * nx; }
  __device__ const real* Q() const { return bQ + sN1() * nxx(); }
  __device__ const real* S() const { return bS + sN() * nxu(); }
  __device__ const real* R() const { return bR + sN() * nuu(); }
  __device__ const real* q() const { return bq + sN1() * nx; }
  __device__ const real* r() const { return br + sN() * nu; }
  __device__ const real* x0() const { return bx0 + iq() * nx; }
  __device__ const real* lbu() const { return blbu ? blbu + sN() * nu : nullptr; }
  __device__ const real* ubu() const { return bubu ? bubu + sN() * nu : nullptr; }
  __device__ const real* lbum() const { return blbum ? blbum + sN() * nu : nullptr; }
  __device__ const real* ubum() const { return bubum ? bubum + sN() * nu : nullptr; }
  __device__ const real* lbx() const { return blbx ? blbx + sN1() * nx : nullptr; }
  __device__ const real* ubx() const { return bubx ? bubx + sN1() * nx : nullptr; }
  __device__ const real* lbxm() const { return blbxm ? blbxm + sN1() * nx : nullptr; }
  __device__ const real* ubxm() const { return bubxm ? bubxm + sN1() * nx : nullptr; }
  __device__ const real* C() const { return bC ? bC + sN1() * ng * nx : nullptr; }
  __device__ const real* D() const { return bD ? bD + sN() * ng * nu : nullptr; }
  __device__ const real* lg() const { return blg + sN1() * ng; }
  __device__ const real* ug() const { return bug + sN1() * ng; }
  __device__ const real* lgm() const { return blgm ? blgm + sN1() * ng : nullptr; }
  __device__ const real* ugm() const { return bugm ? bugm + sN1() * ng : nullptr; }
  __device__ real* x() const { return bxo + oN1() * nx; }
  __device__ real* u() const { return buo + oN() * nu; }
  __device__ real* pi() const { return bpi + oN1() * nx; }
  __device__ real* ws() const { return bws + oq() * ws_qp; }

  __device__ size_t nxx() const { return FULL ? 144 : (size_t)nx * nx; }
  __device__ size_t nxu() const { return FULL ? 144 : (size_t)nx * nu; }
  __device__ size_t nuu() const { return FULL ? 144 : (size_t)nu * nu; }
  __device__ real* st(int k) const {
    return ws() + kQsSize + (size_t)k * (GEN ? stride : (size_t)kIpmStage);
  }
  // state of constraint chunk ch at stage k: bars [48], steps [48], row values [12]
  __device__ real* gs(int k, int ch) const { return st(k) + kIpmStage + ch * kGenChunk; }
  // per-stage general-row vectors (kGenVec) after the chunks
  __device__ real* gv(int k) const { return st(k) + kIpmStage + nch * kGenChunk; }
  // row i of chunk ch (element-owned): lg <= v <= ug
  // (The side loaders read a valid address on every lane and mask the result with selects:
  // a load under a branch is waited for inside that branch, one memory round trip each.
  // The optional mask arrays are chosen by their wave-uniform base pointers.)
  __device__ static Side side_at(const real* lb, const real* ub, const real* lm, const real* um, size_t o,
                                 bool ok) {
    const real l = lb[o], u = ub[o];
    const real ml = (lm ? lm : lb)[o], mu = (um ? um : ub)[o];
    const bool al = (ml != real(0.0)) | (lm == nullptr), au = (mu != real(0.0)) | (um == nullptr);
    return Side{ok ? l : real(0.0), ok ? u : real(0.0), ok && al ? real(1.0) : real(0.0),
                ok && au ? real(1.0) : real(0.0)};
  }
  __device__ Side side_g(int k, int ch, int i) const {
    const int r = ch * kMaxDim + i;
    const bool ok = i < kMaxDim && r < ng;
    const size_t o = (sN1() + k) * ng + (ok ? r : 0);
    return side_at(blg, bug, blgm, bugm, o, ok);
  }
  // row-owned C / D rows of chunk ch (lane i = row); C_0 dropped like the
  // reference's x0 embedding (nx[0] = 0), D_N absent
  __device__ void g_row(int k, int ch, int i, real (&Cr)[12], real (&Dr)[12]) const {
    const int r = ch * kMaxDim + i;
    const bool ok = i < kMaxDim && r < ng;
    const bool cok = GEN == 2 && ok && bC && k > 0, dok = ok && bD && k < N;
    const real* cb = C() ? C() + (size_t)k * ng * nx + r : nullptr;
    const real* db = D() ? D() + (size_t)k * ng * nu + r : nullptr;
    sfor<0, 12>([&](auto j) {
      constexpr int J = decltype(j)::value;
      Cr[J] = (cok && J < nx) ? cb[(size_t)J * ng] : real(0.0);
      Dr[J] = (dok && J < nu) ? db[(size_t)J * ng] : real(0.0);
    });
  }
  // value of row i of chunk ch: C_k x + D_k u (GEN == 1: no C, the product is skipped)
  __device__ real g_row_dot(int k, int ch, int i, const real (&bx)[12], const real (&bu)[12]) const {
    real Cr[12], Dr[12];
    g_row(k, ch, i, Cr, Dr);
    if constexpr (GEN == 2) return dot12(Dr, bu, dot12(Cr, bx, real(0.0)));
    return dot12(Dr, bu, real(0.0));
  }
  // the same with x, u element-owned (broadcast inside the FMAs)
  __device__ real g_row_dot_b(int k, int ch, int i, real x, real u) const {
    real Cr[12], Dr[12];
    g_row(k, ch, i, Cr, Dr);
    if constexpr (GEN == 2) return dot_bcast(Dr, u, dot_bcast(Cr, x, real(0.0)));
    return dot_bcast(Dr, u, real(0.0));
  }
  // column-owned C / D columns restricted to chunk ch (lane j = column)
  __device__ void g_col(int k, int ch, int j, real (&Cc)[12], real (&Dc)[12]) const {
    const int r0 = ch * kMaxDim;
    const bool cok = GEN == 2 && bC && k > 0 && j < nx, dok = bD && k < N && j < nu;
    const real* cb = C() ? C() + (size_t)k * ng * nx + (size_t)j * ng + r0 : nullptr;
    const real* db = D() ? D() + (size_t)k * ng * nu + (size_t)j * ng + r0 : nullptr;
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      Cc[I] = (cok && r0 + I < ng) ? cb[I] : real(0.0);
      Dc[I] = (dok && r0 + I < ng) ? db[I] : real(0.0);
    });
  }

  // ---- column-owned loads (lane = column), zero padded ----
  __device__ void col(const real* blk, int rows, int c, bool ok, real (&v)[12]) const {
    if constexpr (FULL) {
      load12(blk + c * 12, v);
    } else {
      load_col_pad(blk + (size_t)c * rows, rows, ok, v);
    }
  }
  // ---- row-owned loads (lane = row) of a column-major (rows x cols) block ----
  __device__ void row(const real* blk, int rows, int cols, int rw, bool ok, real (&v)[12]) const {
    sfor<0, 12>([&](auto j) {
      constexpr int J = decltype(j)::value;
      if constexpr (FULL) {
        v[J] = blk[rw + J * 12];
      } else {
        v[J] = (ok && J < cols) ? blk[(size_t)rw + (size_t)J * rows] : real(0.0);
      }
    });
  }
  // element i of a length-n vector (0 beyond n)
  __device__ real el(const real* v, int n, int i) const {
    if constexpr (FULL) {
      return i < 12 ? v[i] : real(0.0);
    } else {
      return i < n ? v[i] : real(0.0);
    }
  }
  // per-variable barrier state exists only for the bound families that are given
  // (which 0: u, 1: x): absent ones are neither loaded nor stored
  // (FULL only: the generic-size kernels keep the unconditional accesses, their
  // spill-heavy code generation faulted with the uniform branches added)
  __device__ bool has_bars(int which) const {
    if constexpr (!FULL) return true;
    return which ? blbx != nullptr : blbu != nullptr;
  }
  __device__ Bar bar(const real* stk, int which, int i) const {
    return has_bars(which) ? load_bar(stk, which, i) : Bar{real(0.0), real(0.0), real(1.0), real(1.0)};
  }
  __device__ void put_bar(real* stk, int which, int i, const Bar& b) const {
    if (has_bars(which)) store_bar(stk, which, i, b);
  }
  __device__ BarStep bstep(const real* stk, int which, int i) const {
    return has_bars(which) ? load_bstep(stk, which, i) : BarStep{real(0.0), real(0.0), real(0.0), real(0.0)};
  }
  __device__ void put_bstep(real* stk, int which, int i, const BarStep& d) const {
    if (has_bars(which)) store_bstep(stk, which, i, d);
  }
  // (An absent family reads element 0 of q instead and is masked: no branch either.)
  __device__ Side side_u(int k, int i) const {
    const bool has = blbu != nullptr, ok = has && i < nu && k < N;
    const size_t o = has ? (sN() + (k < N ? k : N - 1)) * nu + (ok ? i : 0) : 0;
    return side_at(has ? blbu : bq, has ? bubu : bq, blbum, bubum, o, ok);
  }
  __device__ Side side_x(int k, int i) const {
    const bool has = blbx != nullptr, ok = has && i < nx && k > 0;  // stage-0 x bounds dropped
    const size_t o = has ? (sN1() + k) * nx + (ok ? i : 0) : 0;
    return side_at(has ? blbx : bq, has ? bubx : bq, blbxm, bubxm, o, ok);
  }
};

// LDS staging of one 12 x 12 block per QP group (lane j < 12 writes column j)
__device__ __forceinline__ void lds_put_col(real* blk, int lane, const real (&v)[12]) {
  if (lane < kMaxDim) store12(blk + lane * 12, v);
}
__device__ __forceinline__ void lds_get_col(const real* blk, int c, real (&v)[12]) {
  load12(blk + c * 12, v);
}
__device__ __forceinline__ void lds_get_row(const real* blk, int r, real (&v)[12]) {
  sfor<0, 12>([&](auto j) {
    constexpr int J = decltype(j)::value;
    v[J] = blk[J * 12 + r];
  });
}
// (lds_wave_fence: qp_group.h)

// general-constraint chunk state (see kGenChunk)
__device__ __forceinline__ Bar load_gbar(const real* g, int i) {
  return Bar{g[i], g[12 + i], g[24 + i], g[36 + i]};
}
__device__ __forceinline__ void store_gbar(real* g, int i, const Bar& b) {
  g[i] = b.ll;
  g[12 + i] = b.lu;
  g[24 + i] = b.tl;
  g[36 + i] = b.tu;
}
__device__ __forceinline__ BarStep load_gstep(const real* g, int i) {
  return BarStep{g[48 + i], g[60 + i], g[72 + i], g[84 + i]};
}
__device__ __forceinline__ void store_gstep(real* g, int i, const BarStep& d) {
  g[48 + i] = d.dtl;
  g[60 + i] = d.dtu;
  g[72 + i] = d.dll;
  g[84 + i] = d.dlu;
}
constexpr int kGenVal = 96;


// Gamma (Hessian add) and gamma (gradient add) of one variable:
// Gamma = lam_l/t_l + lam_u/t_u,
// gamma = (rm_l + lam_l rd_l)/t_l - (rm_u + lam_u rd_u)/t_u, with
// rm = lam t + extra - sigma_mu (extra = dlam_aff dt_aff in the corrector).
__device__ __forceinline__ void gamma_of(const Side& s, const Bar& b, real v, real ext_l,
                                         real ext_u, real smu, real& G, real& g) {
  G = real(0.0);
  g = real(0.0);
  if (s.ml != real(0.0)) {
    const real rd = v - s.lb - b.tl;
    const real rm = b.ll * b.tl + ext_l - smu;
    G += b.ll / b.tl;
    g += (rm + b.ll * rd) / b.tl;
  }
  if (s.mu != real(0.0)) {
    const real rd = s.ub - v - b.tu;
    const real rm = b.lu * b.tu + ext_u - smu;
    G += b.lu / b.tu;
    g -= (rm + b.lu * rd) / b.tu;
  }
}

// dt / dlam of one variable given its primal step dv.
__device__ __forceinline__ BarStep bar_step(const Side& s, const Bar& b, real v, real dv,
                                            real ext_l, real ext_u, real smu) {
  BarStep d{real(0.0), real(0.0), real(0.0), real(0.0)};
  if (s.ml != real(0.0)) {
    const real rd = v - s.lb - b.tl;
    d.dtl = rd + dv;
    d.dll = -(b.ll * b.tl + ext_l - smu + b.ll * d.dtl) / b.tl;
  }
  if (s.mu != real(0.0)) {
    const real rd = s.ub - v - b.tu;
    d.dtu = rd - dv;
    d.dlu = -(b.lu * b.tu + ext_u - smu + b.lu * d.dtu) / b.tu;
  }
  return d;
}

__device__ __forceinline__ void ratio(const Side& s, const Bar& b, const BarStep& d, real& ap,
                                      real& ad) {
  if (s.ml != real(0.0)) {
    if (d.dtl < real(0.0)) ap = fmin(ap, -b.tl / d.dtl);
    if (d.dll < real(0.0)) ad = fmin(ad, -b.ll / d.dll);
  }
  if (s.mu != real(0.0)) {
    if (d.dtu < real(0.0)) ap = fmin(ap, -b.tu / d.dtu);
    if (d.dlu < real(0.0)) ad = fmin(ad, -b.lu / d.dlu);
  }
}

// predictor sums for mu_aff: s1 += lam dt + t dlam, s2 += dlam dt (active sides)
__device__ __forceinline__ void aff_sums(const Side& s, const Bar& b, const BarStep& d, real& s1,
                                         real& s2) {
  if (s.ml != real(0.0)) {
    s1 += b.ll * d.dtl + b.tl * d.dll;
    s2 += d.dll * d.dtl;
  }
  if (s.mu != real(0.0)) {
    s1 += b.lu * d.dtu + b.tu * d.dlu;
    s2 += d.dlu * d.dtu;
  }
}

// gather an element-owned value (lane i < 12 holds v_i) into VL's registers
__device__ __forceinline__ void gather12(real v, real (&out)[12]) {
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    out[I] = bc<I>(v);
  });
}

// SQRT: ric_alg = 1, the square-root factorization (riccati.h riccati_step_sqrt).  The
// record's kRecP slot then holds the factor Lp of P = Lp Lp' (packed lower triangle, the
// same 78 reals) and every sweep applies P as Lp (Lp' v): the solves use exactly the P the
// next stage's factorization used (ric_alg 0 gets the same consistency by symmetrizing its
// register P_k, riccati.h SYMP).
// QP of this thread's group: the grid position, or (ProblemArgsT::qp_list) the position's
// entry of the active-QP list; -1 past the batch / the list
// (the list is on once a compaction kernel of this solve built it: ctl[kCtlListOn])
__device__ __forceinline__ const int* active_list(const ProblemArgsT<real>& a) {
  return a.qp_list && __atomic_load_n(a.ctl + kCtlListOn, __ATOMIC_RELAXED) ? a.qp_list : nullptr;
}
__device__ __forceinline__ int slot_qp(const ProblemArgsT<real>& a, int g) {
  const int* l = active_list(a);
  if (l) return g < l[a.batch] ? l[g] : -1;
  return g < a.batch ? g : -1;
}
__device__ __forceinline__ int group_qp(const ProblemArgsT<real>& a) {
  return slot_qp(a, (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 4));
}

// LQ (ric_alg 1 only), HPIPM's lq_fact: the RB factorizations by Cholesky (0, 1) or by LQ
// (riccati.h riccati_step_lq: 2, 3), of every QP (0, 2) or, for lq_fact 1's per-QP switch
// (kQsForceLq), of the QPs not switched (1) / switched (3).  lq_fact 1 launches 1 and 3 one after
// the other, so each instantiation keeps its own registers (one kernel with both paths spilled
// 540 B/lane into the Cholesky path too).
template <int LQ>
constexpr bool kLqFactor = LQ >= 2;
template <bool FULL, int GEN, int PH, bool SQRT = false, int LQ = 0>
__device__ __forceinline__ void ipm_phase(const ProblemArgsT<real>& a) {
  // the refinement check runs stage-parallel: group g on QP slot g / (N + 1), stage
  // g % (N + 1) (its rows are independent across stages); every other phase: one QP per group
  int kst = 0;
  int qp;
  if constexpr (PH == kPhIR || PH == kPhIRP) {
    const int g = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 4);
    const int slot = g / (a.N + 1);
    kst = g - slot * (a.N + 1);
    qp = slot_qp(a, slot);
  } else {
    qp = group_qp(a);
  }
  const int lane = threadIdx.x & (kGroup - 1);
  if (qp < 0) return;
  const int N = a.N;
  const int nx = FULL ? 12 : a.nx;
  const int nu = FULL ? 12 : a.nu;
  const int col = lane < kMaxDim ? lane : kMaxDim - 1;
  const int li = lane < kMaxDim ? lane : 0;  // element index used for addressing
  const bool xel = lane < nx, uel = lane < nu;

  Ctx<FULL, GEN> c;
  c.N = N;
  c.nx = nx;
  c.nu = nu;
  c.lane = lane;
  c.isv = lane == kVecLane;
  c.qp = qp;
  c.ng = a.ng;
  c.nch = (a.ng + kMaxDim - 1) / kMaxDim;
  c.stride = (size_t)kIpmStage + (size_t)c.nch * kGenChunk + (c.nch ? kGenVec : 0);
  c.ws_qp = a.ws_qp;
  c.bA = a.A; c.bB = a.B; c.bb = a.b; c.bQ = a.Q; c.bS = a.S; c.bR = a.R; c.bq = a.q; c.br = a.r;
  c.bx0 = a.x0;
  c.blbu = a.lbu; c.bubu = a.ubu; c.blbum = a.lbu_mask; c.bubum = a.ubu_mask;
  c.blbx = a.lbx; c.bubx = a.ubx; c.blbxm = a.lbx_mask; c.bubxm = a.ubx_mask;
  c.bC = GEN ? a.C : nullptr; c.bD = GEN ? a.D : nullptr;
  c.blg = a.lg; c.bug = a.ug; c.blgm = a.lg_mask; c.bugm = a.ug_mask;
  c.bxo = a.x; c.buo = a.u; c.bpi = a.pi; c.bws = a.ws;
  const real reg = a.reg;
  // precision of the stage factorization G = R + D'Gamma D + B'PB (riccati.h chol_g):
  // double in the fp32 kernels with C-free general rows (the friction cone), whose fp32
  // factorization broke down on the cone's Gamma of 1e8-1e10
  using greal = std::conditional_t<sizeof(real) == 4 && GEN == 1, double, real>;
  // (P x)_col + acc for an element-owned x (lane j holds x_j), P from a stage record's kRecP
  // slot: packed P (ric_alg 0) or its factor Lp (ric_alg 1)
  // the record's kRecP slot holds the factor Lp (ric_alg 1) or P
  constexpr bool kRecFactor = SQRT;
  auto rec_P_mul = [&](const real* rec, real xv, real acc) -> real {
    if constexpr (kRecFactor) {
      real Lv[12];
      load_packed_lcol_d(rec + kRecP, col, Lv);
      const real t = dot_bcast(Lv, xv, real(0.0));  // (Lp' x)_col
      load_packed_lrow_d(rec + kRecP, col, Lv);
      return dot_bcast(Lv, t, acc);                 // (Lp t)_col + acc
    } else {
      real Pc[12];
      load_packed_sym(rec + kRecP, col, Pc);
      return dot_bcast(Pc, xv, acc);
    }
  };

  // ---- general rows (GEN): Gamma / gamma and their images under C, D ----
  // Gamma / gamma of row `lane` of chunk ch (corrector: + dlam_aff dt_aff - sigma mu)
  auto g_gamma = [&](int k, int ch, bool corr, real smu, real& G, real& gg) {
    G = real(0.0);
    gg = real(0.0);
    if (lane < kMaxDim) {
      const real* g = c.gs(k, ch);
      real el = real(0.0), eu = real(0.0);
      if (corr) {
        const BarStep d = load_gstep(g, lane);
        el = d.dll * d.dtl;
        eu = d.dlu * d.dtu;
      }
      gamma_of(c.side_g(k, ch, lane), load_gbar(g, lane), g[kGenVal + lane], el, eu, smu, G, gg);
    }
  };
  // gradient adds of lane j: radd = (D'gamma)_j, qadd = (C'gamma)_j
  auto g_grad = [&](int k, bool corr, real smu, real& radd, real& qadd) {
    radd = real(0.0);
    qadd = real(0.0);
    for (int ch = 0; ch < c.nch; ++ch) {
      real G, gg, bg[12], Cc[12], Dc[12];
      g_gamma(k, ch, corr, smu, G, gg);
      gather12(gg, bg);
      c.g_col(k, ch, col, Cc, Dc);
      if constexpr (GEN == 2) qadd = dot12(Cc, bg, qadd);
      radd = dot12(Dc, bg, radd);
    }
  };
  // Hessian adds (column-owned): which 0: M1 = R += D'Gamma D;
  // 1: M1 = S += D'Gamma C, M2 = Q += C'Gamma C;  2: M1 = Q += C'Gamma C.
  // Formed from the scaled rows sqrt(Gamma) D, sqrt(Gamma) C, so D'Gamma D and C'Gamma C
  // are sums of the same products in both triangles: exactly symmetric (a Gamma of 1e12
  // times rounding-level asymmetry stalled degenerate endgames).
  auto g_hess = [&](int k, int which, real (&M1)[12], real (&M2)[12]) {
    for (int ch = 0; ch < c.nch; ++ch) {
      real G, gg, Gb[12], Cc[12], Dc[12];
      g_gamma(k, ch, false, real(0.0), G, gg);
      gather12(__builtin_sqrt(G), Gb);
      c.g_col(k, ch, col, Cc, Dc);
      sfor<0, 12>([&](auto i) {
        constexpr int I = decltype(i)::value;
        Dc[I] *= Gb[I];
        Cc[I] *= Gb[I];
      });
      if (which == 0) {
        tmul_acc(Dc, Dc, M1);
      } else if (which == 1) {
        tmul_acc(Dc, Cc, M1);
        tmul_acc(Cc, Cc, M2);
      } else {
        tmul_acc(Cc, Cc, M1);
      }
    }
  };


  real* const qs = c.ws();  // per-QP scalar state (kQs*)
  if constexpr (PH == kPhInit) {
  // =================== init (var_init_scheme 0, relative form) ===================
  real ncl = real(0.0);
  // warm_start 2: continue from a whole iterate -- x, u, pi from the solution buffers, the
  // barrier state from a.warm_bars (HPIPM's warm_start = 2 level; used by the fp64
  // continuation of srbd_qp_settings.f64_rescue).  A non-finite value or a t <= 0 anywhere
  // in the QP falls back to the cold start.
  const size_t warm_w = 96 + (size_t)c.nch * 48;
  const real* wb = a.warm_start == 2 && a.warm_bars
                       ? a.warm_bars + (size_t)c.oq() * (size_t)(N + 1) * warm_w
                       : nullptr;
  bool cont = false;
  if (wb) {
    int bad = 0;
    // an active side needs a finite lam > 0 and t > 0 (a multiplier that underflowed to 0
    // would pin the fraction-to-boundary step at 0); inactive sides and absent families
    // are not read (warm_bar substitutes the cold defaults there)
    auto chk = [&](real v, bool pos) { bad |= !__builtin_isfinite(v) || (pos && !(v > real(0.0))); };
    auto chk_bar = [&](const real* p, const Side& s) {
      if (s.ml != real(0.0)) {
        chk(p[0], true);
        chk(p[24], true);
      }
      if (s.mu != real(0.0)) {
        chk(p[12], true);
        chk(p[36], true);
      }
    };
    for (int k = 0; k <= N && lane < kMaxDim; ++k) {
      const real* w = wb + (size_t)k * warm_w;
      if (k < N) chk_bar(w + lane, c.side_u(k, lane));  // (no u_N)
      chk_bar(w + 48 + lane, c.side_x(k, lane));
      for (int ch = 0; ch < c.nch; ++ch) chk_bar(w + 96 + ch * 48 + lane, c.side_g(k, ch, lane));
      if (k < N && uel) chk(c.u()[(size_t)k * nu + lane], false);
      if (k > 0 && xel) {
        chk(c.x()[(size_t)k * nx + lane], false);
        chk(c.pi()[(size_t)k * nx + lane], false);
      }
    }
    cont = gsum(real(bad)) == real(0.0);
  }
  if (cont) {
    for (int k = 0; k <= N; ++k) {
      real* stk = c.st(k);
      const real* w = wb + (size_t)k * warm_w;
      if (lane < kMaxDim) {
        store_bar(stk, 1, lane, warm_bar(w + 48 + lane, c.side_x(k, lane)));
        store_bar(stk, 0, lane, k < N ? warm_bar(w + lane, c.side_u(k, lane))
                                      : Bar{real(0.0), real(0.0), real(1.0), real(1.0)});
      }
      const real ui = (k < N && uel) ? c.u()[(size_t)k * nu + li] : real(0.0);
      real xi;
      if (k == 0) {
        xi = xel ? c.x0()[li] : real(0.0);
        if (xel) {
          c.x()[lane] = xi;
          c.pi()[lane] = real(0.0);
        }
      } else {
        xi = xel ? c.x()[(size_t)k * nx + li] : real(0.0);
      }
      if (k < N) {
        const Side s = c.side_u(k, lane);
        ncl += s.ml + s.mu;
      }
      {
        const Side s = c.side_x(k, lane);
        ncl += s.ml + s.mu;
      }
      if constexpr (GEN) {
        real bxi[12], bui[12];
        gather12(xi, bxi);
        gather12(ui, bui);
        for (int ch = 0; ch < c.nch; ++ch) {
          const real v = c.g_row_dot(k, ch, lane, bxi, bui);
          const Side s = c.side_g(k, ch, lane);
          ncl += s.ml + s.mu;
          if (lane < kMaxDim) {
            real* g = c.gs(k, ch);
            store_gbar(g, lane, warm_bar(w + 96 + ch * 48 + lane, s));
            store_gstep(g, lane, BarStep{0, 0, 0, 0});
            g[kGenVal + lane] = v;
          }
        }
      }
      if (lane < kMaxDim) {
        stk[kStStep + lane] = real(0.0);
        stk[kStStep + 12 + lane] = real(0.0);
        stk[kStStep + 24 + lane] = real(0.0);
        store_bstep(stk, 0, lane, BarStep{0, 0, 0, 0});
        store_bstep(stk, 1, lane, BarStep{0, 0, 0, 0});
      }
    }
  }
  for (int k = 0; k <= N && !cont; ++k) {
    real* stk = c.st(k);
    real ui = real(0.0), xi = real(0.0);  // initial u_k, x_k (element-owned)
    // u_k
    if (k < N) {
      real v = (a.warm_start && uel) ? c.u()[(size_t)k * nu + li] : real(0.0);
      const Side s = c.side_u(k, lane);
      Bar bb{real(0.0), real(0.0), real(1.0), real(1.0)};
      if (s.ml != real(0.0) || s.mu != real(0.0)) {
        real tl = v - s.lb, tu = s.ub - v;
        if (s.ml != real(0.0) && s.mu != real(0.0)) {
          if (tl < kThr0) {
            if (tu < kThr0) {
              v = real(0.5) * (s.lb + s.ub);
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
        } else if (s.ml != real(0.0)) {
          if (tl < kThr0) {
            tl = kThr0;
            v = s.lb + kThr0;
          }
        } else if (tu < kThr0) {
          tu = kThr0;
          v = s.ub - kThr0;
        }
        bb.tl = s.ml != real(0.0) ? tl : real(1.0);
        bb.tu = s.mu != real(0.0) ? tu : real(1.0);
        bb.ll = s.ml != real(0.0) ? a.mu0 / tl : real(0.0);
        bb.lu = s.mu != real(0.0) ? a.mu0 / tu : real(0.0);
      }
      ncl += s.ml + s.mu;
      if (lane < kMaxDim) store_bar(stk, 0, lane, bb);
      if (uel) c.u()[(size_t)k * nu + lane] = v;
      ui = uel ? v : real(0.0);
    }
    // x_k
    {
      real v;
      if (k == 0) {
        v = xel ? c.x0()[li] : real(0.0);
      } else {
        v = (a.warm_start && xel) ? c.x()[(size_t)k * nx + li] : real(0.0);
      }
      const Side s = c.side_x(k, lane);
      Bar bb{real(0.0), real(0.0), real(1.0), real(1.0)};
      if (s.ml != real(0.0) || s.mu != real(0.0)) {
        real tl = v - s.lb, tu = s.ub - v;
        if (s.ml != real(0.0) && s.mu != real(0.0)) {
          if (tl < kThr0) {
            if (tu < kThr0) {
              v = real(0.5) * (s.lb + s.ub);
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
        } else if (s.ml != real(0.0)) {
          if (tl < kThr0) {
            tl = kThr0;
            v = s.lb + kThr0;
          }
        } else if (tu < kThr0) {
          tu = kThr0;
          v = s.ub - kThr0;
        }
        bb.tl = s.ml != real(0.0) ? tl : real(1.0);
        bb.tu = s.mu != real(0.0) ? tu : real(1.0);
        bb.ll = s.ml != real(0.0) ? a.mu0 / tl : real(0.0);
        bb.lu = s.mu != real(0.0) ? a.mu0 / tu : real(0.0);
      }
      ncl += s.ml + s.mu;
      if (lane < kMaxDim) store_bar(stk, 1, lane, bb);
      if (xel) {
        c.x()[(size_t)k * nx + lane] = v;
        c.pi()[(size_t)k * nx + lane] = real(0.0);
      }
      xi = xel ? v : real(0.0);
    }
    // general rows: t = max(v - lg, thr0), max(ug - v, thr0) at the initial
    // x_k / u_k (no projection possible), lam = mu0 / t
    if constexpr (GEN) {
      real bxi[12], bui[12];
      gather12(xi, bxi);
      gather12(ui, bui);
      for (int ch = 0; ch < c.nch; ++ch) {
        const real v = c.g_row_dot(k, ch, lane, bxi, bui);
        const Side s = c.side_g(k, ch, lane);
        Bar bb{real(0.0), real(0.0), real(1.0), real(1.0)};
        if (s.ml != real(0.0)) {
          bb.tl = fmax(v - s.lb, kThr0);
          bb.ll = a.mu0 / bb.tl;
        }
        if (s.mu != real(0.0)) {
          bb.tu = fmax(s.ub - v, kThr0);
          bb.lu = a.mu0 / bb.tu;
        }
        ncl += s.ml + s.mu;
        if (lane < kMaxDim) {
          real* g = c.gs(k, ch);
          store_gbar(g, lane, bb);
          store_gstep(g, lane, BarStep{0, 0, 0, 0});
          g[kGenVal + lane] = v;
        }
      }
    }
    if (lane < kMaxDim) {
      // zero step: the first RU pass applies nothing
      stk[kStStep + lane] = real(0.0);
      stk[kStStep + 12 + lane] = real(0.0);
      stk[kStStep + 24 + lane] = real(0.0);
      store_bstep(stk, 0, lane, BarStep{0, 0, 0, 0});
      store_bstep(stk, 1, lane, BarStep{0, 0, 0, 0});
    }
  }
  const real nc = gsum(lane < kMaxDim ? ncl : real(0.0));
  if (lane == 0) {
    qs[kQsAlphaP] = real(0.0);
    qs[kQsAlphaD] = real(0.0);
    qs[kQsLastAmin] = real(1.0);
    qs[kQsSigmaMu] = real(0.0);
    qs[kQsStatus] = -real(1.0);
    qs[kQsIter] = real(0.0);
    qs[kQsNc] = nc;
    qs[kQsForceLq] = a.lq_fact == 2 ? real(1.0) : real(0.0);
    qs[kQsLqRedo] = real(0.0);
  }

    return;
  }
  const real nc = qs[kQsNc];
  const real nc_inv = nc > real(0.0) ? real(1.0) / nc : real(0.0);
  int status = (int)qs[kQsStatus];
  const int iter = (int)qs[kQsIter];
  if constexpr (PH == kPhOut) {
    const real res_stat = qs[kQsResStat], res_eq = qs[kQsResEq], res_ineq = qs[kQsResIneq];
    const real res_comp = qs[kQsResComp], obj = qs[kQsObj];
    if (status < 0) status = 1;  // not reached: the last RB sweep always decides
    const int par = iter & 1;
  // =================== outputs ===================
  // Riccati factors of the last completed iteration (HPIPM's getters); the
  // exiting sweep's own factorization is used only when no step was taken.
  const int out_par = iter > 0 ? (par ^ 1) : par;
  // pi_0 := Q0 x0 + S0'u0 + q0 + A0'(pi_1 + P_1 res_b0): the value of the
  // stage-0 rebuild (ocp_qp_ipm_solver.cpp:347-373) with p_1 = pi_1 - P_1 x_1.
  {
    const real* st0 = c.st(0);
    const real* st1 = c.st(1) + out_par * kRecSize;
    real bx0[12], bu0[12];
    gather12(xel ? c.x()[li] : real(0.0), bx0);
    gather12(uel ? c.u()[li] : real(0.0), bu0);
    real t = rec_P_mul(st1, lane < kMaxDim ? st0[kStRes + 24 + lane] : real(0.0),
                       xel ? c.pi()[(size_t)nx + lane] : real(0.0));
    if (!xel) t = real(0.0);
    real bt[12];
    gather12(t, bt);
    real Qc[12], Sc[12], Ac[12];
    c.col(c.Q(), nx, col, xel, Qc);
    c.col(c.S(), nu, col, xel, Sc);
    c.col(c.A(), nx, col, xel, Ac);
    real p0 = c.el(c.q(), nx, li);
    sfor<0, 12>([&](auto j) {
      constexpr int J = decltype(j)::value;
      p0 = fmadd(Qc[J], bx0[J], p0);
      p0 = fmadd(Sc[J], bu0[J], p0);
      p0 = fmadd(Ac[J], bt[J], p0);
    });
    if (xel) c.pi()[lane] = p0;
  }
  if (a.P || a.p || a.K || a.k) {
    // Riccati matrices of the last factorization (HPIPM's get_ric_* getters),
    // vectors by consistency: p_k = pi_k - P_k x_k, k_k = u_k - K_k x_k.
    const size_t nxx = (size_t)nx * nx, nxu = (size_t)nx * nu;
    for (int k = 0; k <= N; ++k) {
      const real* stk = c.st(k) + out_par * kRecSize;
      real bxk[12];
      gather12(xel ? c.x()[(size_t)k * nx + li] : real(0.0), bxk);
      real Pc[12];
      if constexpr (kRecFactor) {  // P = Lp Lp': column l = sum_K Lp[:, K] Lp[l][K]
        real Lr[12];
        load_packed_lrow_d(stk + kRecP, col, Lr);
        sfor<0, 12>([&](auto i) { Pc[decltype(i)::value] = real(0.0); });
        tmul_acc(Lr, Lr, Pc);
      } else {
        load_packed_sym(stk + kRecP, col, Pc);
      }
      if (a.P && xel)
        sfor<0, 12>([&](auto i) {
          constexpr int I = decltype(i)::value;
          if (I < nx) a.P[((size_t)qp * (N + 1) + k) * nxx + (size_t)lane * nx + I] = Pc[I];
        });
      if (a.p) {
        const real px = rec_P_mul(stk, xel ? c.x()[(size_t)k * nx + li] : real(0.0), real(0.0));
        if (xel) a.p[((size_t)qp * (N + 1) + k) * nx + lane] = c.pi()[(size_t)k * nx + lane] - px;
      }
      if (k < N) {
        real Kc[12];
        load12(stk + kRecK + col * 12, Kc);
        if (a.K && xel)
          sfor<0, 12>([&](auto i) {
            constexpr int I = decltype(i)::value;
            if (I < nu) a.K[((size_t)qp * N + k) * nxu + (size_t)lane * nu + I] = Kc[I];
          });
        if (a.k) {
          real Kr[12];
          sfor<0, 12>([&](auto j) {
            constexpr int J = decltype(j)::value;
            Kr[J] = stk[kRecK + J * 12 + li];
          });
          real kx = real(0.0);
          sfor<0, 12>([&](auto j) {
            constexpr int J = decltype(j)::value;
            kx = fmadd(Kr[J], bxk[J], kx);
          });
          if (uel) a.k[((size_t)qp * N + k) * nu + lane] = c.u()[(size_t)k * nu + lane] - kx;
        }
      }
    }
  }
  if (lane == 0) {
    if (a.status) a.status[qp] = status;
    if (a.iter) a.iter[qp] = nc > real(0.0) ? iter : 0;
    if (a.res) {
      a.res[(size_t)qp * 4 + 0] = res_stat;
      a.res[(size_t)qp * 4 + 1] = res_eq;
      a.res[(size_t)qp * 4 + 2] = res_ineq;
      a.res[(size_t)qp * 4 + 3] = res_comp;
    }
    if (a.obj) a.obj[qp] = obj;
  }
    return;
  }
  if (status >= 0) return;  // this QP has exited
  // lq_fact 1: RB -> F1 of the QPs this instantiation factorizes, and the redo launch (RB -> F1
  // by LQ of the QPs whose check switched them)
  if constexpr (PH == kPhRB || PH == kPhF1) {
    if constexpr (LQ == 1 || LQ == 3)
      if ((qs[kQsForceLq] != real(0.0)) != (LQ == 3)) return;
    if (a.lq_redo && qs[kQsLqRedo] == real(0.0)) return;
  }
  const int par = iter & 1;  // record written by this iteration's factorization
  const real alpha_p = qs[kQsAlphaP], alpha_d = qs[kQsAlphaD], last_amin = qs[kQsLastAmin];
  if constexpr (PH == kPhRB) {
    // =========== RB (k = N..0): update + residuals + Gamma/gamma + factorization ===========
    // One backward sweep per iteration: stage k applies the previous step to its
    // variables, forms its residuals (x_{k+1}, pi_{k+1} were updated by stage k+1),
    // and factorizes its barrier-augmented block right away, so the QP data is
    // streamed once per iteration.  If the exit test after the sweep fires, this
    // sweep's factorization is simply not used (outputs read the other parity).
    // Every 12 x 12 block of stage k is read from global memory once: column-owned,
    // as the factorization needs it.  The residual products take the same
    // registers where they are column-shaped (Q x, R u, S'u, A'pi, B'pi: symmetric
    // or transposed) and a row-owned copy through LDS where they are not (A x, B u,
    // S x); S stays in LDS until the factorization's second phase asks for it.
    // LDS per QP group: A, B, S columns (3 x 144 reals).
    real* const ldsA = group_lds_blocks<GEN>();
    real* const ldsB = ldsA + 144;
    real* const ldsS = ldsA + 288;
    // The sweep's six accumulators are live across the whole factorization, where the
    // fp64 register file is at its limit: there they live in one LDS slot per lane
    // (box-u RB 68 B of scratch -> none, -2.4%); fp32 keeps them in registers (no
    // spills there, and the LDS round trips cost 1%).
    constexpr bool kAccLds = sizeof(real) == 8;
    __shared__ real rb_acc[kAccLds ? 6 * 256 : 1];
    real acc_r[6];
    real& mg = kAccLds ? rb_acc[0 * 256 + threadIdx.x] : acc_r[0];
    real& mb = kAccLds ? rb_acc[1 * 256 + threadIdx.x] : acc_r[1];
    real& md = kAccLds ? rb_acc[2 * 256 + threadIdx.x] : acc_r[2];
    real& mm = kAccLds ? rb_acc[3 * 256 + threadIdx.x] : acc_r[3];
    real& musum = kAccLds ? rb_acc[4 * 256 + threadIdx.x] : acc_r[4];
    real& objl = kAccLds ? rb_acc[5 * 256 + threadIdx.x] : acc_r[5];
    mg = mb = md = mm = musum = objl = real(0.0);
    real xn = real(0.0), pin = real(0.0);  // updated x_{k+1}, pi_{k+1} (element-owned), from stage k+1
    real P[12];
    // this QP's factorizations by LQ (HPIPM lq_fact): the general rows' sqrt(Gamma) [D'; C'] and
    // the cost-to-go are absorbed by reflections instead of summed into the Hessian
    constexpr bool use_lq = SQRT && kLqFactor<LQ>;
    const bool own = lane < kMaxDim;
    // stage ks's general-row columns sqrt(Gamma_r) [D_r'; C_r'], one 12-row chunk at a time
    auto absorb_rows = [&](int ks, LqRows<real>& L) {
      if constexpr (GEN > 0) {
        for (int ch = 0; ch < c.nch; ++ch) {
          real G, gg, Gb[12], Cc[12], Dc[12], Au[12], Ax[12];
          g_gamma(ks, ch, false, real(0.0), G, gg);
          gather12(__builtin_sqrt(G), Gb);
          c.g_col(ks, ch, col, Cc, Dc);
          sfor<0, 12>([&](auto i) {
            constexpr int I = decltype(i)::value;
            Au[I] = own ? Dc[I] * Gb[I] : real(0.0);
            Ax[I] = (GEN == 2 && own) ? Cc[I] * Gb[I] : real(0.0);
          });
          lq_absorb(L, Au, Ax, lane);
        }
      }
    };
    for (int k = N; k >= 0; --k) {
      tstamp(20);
      real* stk = c.st(k);
      real* rec = stk + par * kRecSize;
      // ---- the stage's loads that wait for none of its arithmetic, issued ahead of its
      // first store: the memory counter retires in issue order, so every load issued behind
      // a store waits for that store too, and the stage would pay one memory round trip per
      // load-after-store group.  (Addresses are valid on every lane; the values are masked
      // where the old conditional loads did not run.)  The A, B, S columns stay below, after
      // the stores: loaded here they stay live across the residual phase and spill (box-u RB
      // 424 B/lane).
      const int iu = li < nu ? li : 0, ix = li < nx ? li : 0;
      const real u_old = c.u()[(size_t)(k < N ? k : N - 1) * nu + iu];
      const real x_old = c.x()[(size_t)k * nx + ix];
      const real pi_old = c.pi()[(size_t)k * nx + ix];
      const real du_s = stk[kStStep + li], dx_s = stk[kStStep + 12 + li], dpi_s = stk[kStStep + 24 + li];
      Bar bu = c.bar(stk, 0, li), bx = c.bar(stk, 1, li);
      const BarStep du = c.bstep(stk, 0, li), dx = c.bstep(stk, 1, li);
      const Side su = c.side_u(k, lane), sx = c.side_x(k, lane);
      const real qk = c.el(c.q() + (size_t)k * nx, nx, li);
      const real rk = k < N ? c.el(c.r() + (size_t)k * nu, nu, li) : real(0.0);
      if (k == N) c.col(c.Q() + (size_t)N * c.nxx(), nx, col, xel, P);  // P_N = Q_N + ...
      // ---- apply the previous step to stage k ----
      real uk = real(0.0), xk = real(0.0), pik = real(0.0);
      if (k < N && uel) {
        uk = step(u_old, alpha_p, du_s);
        c.u()[(size_t)k * nu + lane] = uk;
      }
      if (xel) {
        if (k == 0) {
          xk = x_old;  // x_0 = x0 (never updated); pi_0 is not an iterate
        } else {
          xk = step(x_old, alpha_p, dx_s);
          pik = step(pi_old, alpha_d, dpi_s);
          c.x()[(size_t)k * nx + lane] = xk;
          c.pi()[(size_t)k * nx + lane] = pik;
        }
      }
      if (lane >= kMaxDim) {
        bu = Bar{0, 0, 1, 1};
        bx = Bar{0, 0, 1, 1};
      } else {
        bu.tl = step(bu.tl, alpha_p, du.dtl);
        bu.tu = step(bu.tu, alpha_p, du.dtu);
        bu.ll = step(bu.ll, alpha_d, du.dll);
        bu.lu = step(bu.lu, alpha_d, du.dlu);
        bx.tl = step(bx.tl, alpha_p, dx.dtl);
        bx.tu = step(bx.tu, alpha_p, dx.dtu);
        bx.ll = step(bx.ll, alpha_d, dx.dll);
        bx.lu = step(bx.lu, alpha_d, dx.dlu);
        c.put_bar(stk, 0, lane, bu);
        c.put_bar(stk, 1, lane, bx);
      }
      // ---- residual terms without the stage blocks (element-owned) ----
      real rgx = qk - pik, rgu = rk;
      // general rows, one pass per 12-row chunk with C / D read once: apply the
      // step, row values (row-owned through LDS), res_d / res_m, res_g += C'(lam_u -
      // lam_l) / D'(..), predictor Gamma / gamma, gradient adds C'gamma / D'gamma and
      // (GEN == 1) the Hessian add D'Gamma D, accumulated for the factorization
      real gra = real(0.0), gqa = real(0.0);  // D'gamma, C'gamma (lane j)
      real gea = real(0.0);                   // D'e, e = d gamma / d(sigma mu) (GEN == 1)
      // D'Gamma D, column j (GEN == 1); in double (fp32 kernel) it waits for the
      // factorization in this lane's LDS slots rather than in 24 registers
      constexpr bool kRgLds = !std::is_same_v<greal, real>;
      __shared__ greal rg_lds[kRgLds ? 12 * 256 : 1];
      greal RG[12];
      sfor<0, 12>([&](auto i) { RG[decltype(i)::value] = greal(0.0); });
      if constexpr (GEN) {
        for (int ch = 0; ch < c.nch; ++ch) {
          real* g = c.gs(k, ch);
          const Side sg = c.side_g(k, ch, lane);
          Bar bg{0, 0, 1, 1};
          if (lane < kMaxDim) {
            bg = load_gbar(g, lane);
            const BarStep d = load_gstep(g, lane);
            bg.tl = step(bg.tl, alpha_p, d.dtl);
            bg.tu = step(bg.tu, alpha_p, d.dtu);
            bg.ll = step(bg.ll, alpha_d, d.dll);
            bg.lu = step(bg.lu, alpha_d, d.dlu);
            store_gbar(g, lane, bg);
          }
          real Cc[12], Dc[12];
          c.g_col(k, ch, col, Cc, Dc);
          // row i of the chunk on lane i: v = C x + D u
          real v;
          {
            real M[12];
            lds_put_col(ldsA, lane, Dc);
            if constexpr (GEN == 2) lds_put_col(ldsB, lane, Cc);
            lds_wave_fence();
            lds_get_row(ldsA, li, M);
            v = dot_bcast(M, uk, real(0.0));
            if constexpr (GEN == 2) {
              lds_get_row(ldsB, li, M);
              v = dot_bcast(M, xk, v);
            }
            lds_wave_fence();
          }
          if (lane < kMaxDim) g[kGenVal + lane] = v;
          if (sg.ml != real(0.0)) {
            const real rd = v - sg.lb - bg.tl, rm = bg.ll * bg.tl;
            md = fmax(md, nabs(rd));
            mm = fmax(mm, nabs(rm));
            musum += rm;
          }
          if (sg.mu != real(0.0)) {
            const real rd = sg.ub - v - bg.tu, rm = bg.lu * bg.tu;
            md = fmax(md, nabs(rd));
            mm = fmax(mm, nabs(rm));
            musum += rm;
          }
          real G = real(0.0), gg = real(0.0);
          if (lane < kMaxDim) gamma_of(sg, bg, v, real(0.0), real(0.0), real(0.0), G, gg);
          const real dl = lane < kMaxDim ? bg.lu - bg.ll : real(0.0);
          if constexpr (GEN == 2) {
            rgx = dot_bcast(Cc, dl, rgx);
            gqa = dot_bcast(Cc, gg, gqa);
          }
          rgu = dot_bcast(Dc, dl, rgu);
          gra = dot_bcast(Dc, gg, gra);
          if constexpr (GEN == 1) {
            // gamma is affine in sigma mu: d gamma / d(sigma mu) = mu_row / t_u - ml / t_l
            real e = real(0.0);
            if (lane < kMaxDim) {
              if (sg.ml != real(0.0)) e -= real(1.0) / bg.tl;
              if (sg.mu != real(0.0)) e += real(1.0) / bg.tu;
            }
            gea = dot_bcast(Dc, e, gea);
          }
          if constexpr (GEN == 1) if (!use_lq) {
            // D'Gamma D from sqrt(Gamma) D: exactly symmetric (see g_hess); formed in greal
            const greal sG = __builtin_sqrt(greal(G));
            greal Dg[12];
            sfor<0, 12>([&](auto i) {
              constexpr int I = decltype(i)::value;
              Dg[I] = greal(Dc[I]) * bc<I>(sG);
            });
            if constexpr (kRgLds) {
              if (ch > 0) sfor<0, 12>([&](auto i) { RG[decltype(i)::value] = rg_lds[decltype(i)::value * 256 + threadIdx.x]; });
              tmul_acc(Dg, Dg, RG);
              sfor<0, 12>([&](auto i) { rg_lds[decltype(i)::value * 256 + threadIdx.x] = RG[decltype(i)::value]; });
            } else {
              tmul_acc(Dg, Dg, RG);
            }
          }
        }
      }
      // box terms
      if (su.ml != real(0.0)) {
        rgu -= bu.ll;
        const real rd = uk - su.lb - bu.tl, rm = bu.ll * bu.tl;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      if (su.mu != real(0.0)) {
        rgu += bu.lu;
        const real rd = su.ub - uk - bu.tu, rm = bu.lu * bu.tu;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      if (sx.ml != real(0.0)) {
        rgx -= bx.ll;
        const real rd = xk - sx.lb - bx.tl, rm = bx.ll * bx.tl;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      if (sx.mu != real(0.0)) {
        rgx += bx.lu;
        const real rd = sx.ub - xk - bx.tu, rm = bx.lu * bx.tu;
        md = fmax(md, nabs(rd));
        mm = fmax(mm, nabs(rm));
        musum += rm;
      }
      // predictor Gamma / gamma of the bounds and general rows
      real Gu = real(0.0), gu = real(0.0), Gx = real(0.0), gx = real(0.0);
      if (lane < kMaxDim) {
        gamma_of(su, bu, uk, real(0.0), real(0.0), real(0.0), Gu, gu);
        gamma_of(sx, bx, xk, real(0.0), real(0.0), real(0.0), Gx, gx);
      }
      if constexpr (GEN == 1) {
        if (lane < kMaxDim) {
          real* v = c.gv(k);
          v[lane] = gra;
          v[12 + lane] = gea;
        }
      }
      gu += gra;
      gx += gqa;
      // residuals -> stk[kStRes] and the norms, each as soon as it is complete;
      // the Newton right-hand sides are r~ = res_g,u + gamma_u, q~ = res_g,x + gamma_x
      auto finish_u = [&](real rgu_) -> real {
        if (!uel) rgu_ = real(0.0);
        mg = fmax(mg, nabs(rgu_));
        if (lane < kMaxDim) stk[kStRes + lane] = rgu_;
        return lane < kMaxDim ? rgu_ + gu : real(0.0);
      };
      auto finish_x = [&](real rgx_) -> real {
        if (!xel) rgx_ = real(0.0);
        if (k > 0) mg = fmax(mg, nabs(rgx_));
        if (lane < kMaxDim) stk[kStRes + 12 + lane] = rgx_;
        return lane < kMaxDim ? rgx_ + gx : real(0.0);
      };
      auto finish_b = [&](real rb_) -> real {
        if (!xel) rb_ = real(0.0);
        if (k < N) mb = fmax(mb, nabs(rb_));
        if (lane < kMaxDim) stk[kStRes + 24 + lane] = rb_;
        return rb_;
      };
      SRBD_PHASE_FENCE();
      tstamp(21);
      if (k == N) {
        // terminal stage: P_N = Q_N + diag(Gamma_x) (+ C'Gamma C), p_N = q~_N (Q_N loaded above)
        const real qx = dot_bcast(P, xk, real(0.0));
        if (k > 0) objl += xk * (real(0.5) * qx + qk);
        finish_u(real(0.0));  // no u_N: res_g,u = 0
        finish_b(real(0.0));
        const real qt = finish_x(rgx + qx);
        real qv[12];
        gather12(qt, qv);
        if constexpr (GEN == 2) if (!use_lq) g_hess(N, 2, P, P);
        sfor<0, 12>([&](auto i) {
          constexpr int I = decltype(i)::value;
          if (lane == I) P[I] += Gx;
          if (c.isv) P[I] = qv[I];
        });
        if (c.isv) store12(rec + kRecPv, P);
        if constexpr (SQRT && !kRecFactor)
          if (lane < kMaxDim) store_packed_col(rec + kRecP, lane, P);
        if constexpr (SQRT) {  // (kRecFactor: the record keeps the factor)
          if (GEN == 2 && use_lq) {
            // L_N = LQ([chol(Q_N + Gamma_x) | sqrt(Gamma) C_N']), s_N = L_N^-1 q~_N
            LqRows<real> L;
            real Pm[12], rsx;
            sfor<0, 12>([&](auto i) {
              constexpr int I = decltype(i)::value;
              L.Lu[I] = real(0.0);
              L.Lxu[I] = real(0.0);
              Pm[I] = c.isv ? real(0.0) : P[I];
            });
            chol_cols(Pm, lane, real(0.0), L.Lx, rsx);
            group_transpose(ldsB, lane, L.Lx, -1);
            absorb_rows(N, L);
            group_transpose(ldsB, lane, L.Lx, 1);
            real dd = real(0.0);
            sfor<0, 12>([&](auto i) {
              if (lane == decltype(i)::value) dd = L.Lx[decltype(i)::value];
            });
            rsx = dd > real(0.0) ? real(1.0) / dd : real(0.0);
            trsv_lower(L.Lx, rsx, P);  // VL: s_N (the matrix lanes' results are replaced)
            sfor<0, 12>([&](auto i) {
              if (!c.isv) P[decltype(i)::value] = L.Lx[decltype(i)::value];
            });
          } else {
            sqrt_factor(P, lane);
          }
        }
        if constexpr (!SQRT || kRecFactor)
          if (lane < kMaxDim) store_packed_col(rec + kRecP, lane, P);
      } else {
        // ---- A, B (kept by the factorization), S (kept in LDS): residual products ----
        real A_[12], B_[12], Sh[12], Rh[12];
        c.col(c.A() + (size_t)k * c.nxx(), nx, col, xel, A_);
        c.col(c.B() + (size_t)k * c.nxu(), nx, col, uel, B_);
        c.col(c.S() + (size_t)k * c.nxu(), nu, col, xel, Sh);
        // the box kernels take R with them (one round trip less); the general-row kernels,
        // at their register limit, when the factorization asks for it (cone +0.7% otherwise)
        constexpr bool kEarlyR = GEN == 0;
        if constexpr (kEarlyR) c.col(c.R() + (size_t)k * c.nuu(), nu, col, uel, Rh);
        const real bk = c.el(c.b() + (size_t)k * nx, nx, li);
        rgx = dot_bcast(A_, pin, rgx);  // + A'pi_{k+1}
        rgu = dot_bcast(B_, pin, rgu);  // + B'pi_{k+1}
        lds_put_col(ldsA, lane, A_);
        lds_put_col(ldsB, lane, B_);
        real sxu;  // (S x)_l
        rgx = dot_bcast(Sh, uk, rgx);  // + S'u
        lds_put_col(ldsS, lane, Sh);
        lds_wave_fence();
        real rb;  // res_b = A x + B u + b - x_{k+1}
        {
          real M[12];
          lds_get_row(ldsA, li, M);
          rb = dot_bcast(M, xk, bk - xn);
          lds_get_row(ldsB, li, M);
          rb = dot_bcast(M, uk, rb);
          lds_get_row(ldsS, li, M);
          sxu = dot_bcast(M, xk, real(0.0));
        }
        rgu += sxu;
        rb = finish_b(rb);
        // P_{k+1} b~_k, kept in the record for B2: the corrector's b~ is the predictor's, so
        // B2 reads these 12 values instead of P_{k+1} (78) back (classical Riccati; the square
        // root's record holds Lp, B2 multiplies it out as before)
        real pbk = real(0.0);
        if constexpr (kRecPbOn<SQRT>) pbk = dot_bcast(P, rb, real(0.0));
        real bv[12];
        gather12(rb, bv);
        sfor<0, 12>([&](auto i) {
          constexpr int I = decltype(i)::value;
          if (c.isv) {
            A_[I] = bv[I];
            B_[I] = real(0.0);
          }
        });
        SRBD_PHASE_FENCE();
        real rt = real(0.0);
        auto loadR = [&](greal (&Rc)[12]) {
          real (&Rr)[12] = Rh;
          if constexpr (!kEarlyR) c.col(c.R() + (size_t)k * c.nuu(), nu, col, uel, Rr);
          const real ru = dot_bcast(Rr, uk, real(0.0));  // R u, before the barrier Hessian goes in
          objl += uk * (real(0.5) * ru + rk + sxu);
          rt = finish_u(rgu + ru);
          if constexpr (GEN == 2) if (!use_lq) g_hess(k, 0, Rr, Rr);
          sfor<0, 12>([&](auto i) {
            constexpr int I = decltype(i)::value;
            Rc[I] = greal(Rr[I]);
            if constexpr (GEN == 1) if (!use_lq) Rc[I] += greal(kRgLds ? rg_lds[I * 256 + threadIdx.x] : RG[I]);
            if (lane == I) Rc[I] += (I < nu) ? greal(Gu) : greal(1.0);  // padded inputs: R = 1
            if (c.isv) Rc[I] = greal(0.0);
          });
        };
        auto loadSQ = [&](real (&Sc)[12], real (&Qc)[12]) {
          lds_get_col(ldsS, col, Sc);
          c.col(c.Q() + (size_t)k * c.nxx(), nx, col, xel, Qc);
          const real qx = dot_bcast(Qc, xk, real(0.0));
          if (k > 0) objl += xk * (real(0.5) * qx + qk);
          const real qt = finish_x(rgx + qx);
          if constexpr (GEN == 2) if (!use_lq) g_hess(k, 1, Sc, Qc);  // C = 0: D'Gamma C = C'Gamma C = 0
          sfor<0, 12>([&](auto i) {
            constexpr int I = decltype(i)::value;
            const real rI = bc<I>(rt), qI = bc<I>(qt);
            if (lane == I) Qc[I] += Gx;
            if (c.isv) {
              Sc[I] = rI;
              Qc[I] = qI;
            }
          });
        };
        tstamp(22);
        StageFactor<real> f;
        if constexpr (SQRT) {
          if constexpr (use_lq) {
            auto loadR_lq = [&](real (&Rc)[12]) {
              greal Rg[12];
              loadR(Rg);
              sfor<0, 12>([&](auto i) { Rc[decltype(i)::value] = real(Rg[decltype(i)::value]); });
            };
            riccati_step_lq(P, A_, B_, loadR_lq, loadSQ, lane, reg, f, ldsB,
                            [&](LqRows<real>& L, int) { absorb_rows(k, L); });
          } else {
            // (HPIPM's square-root form: P_k = F - Y'Y as the trailing block of the joint factor)
            riccati_step_sqrt<1, false, greal>(P, A_, B_, loadR, loadSQ, lane, reg, f);
          }
        } else {
          // P_k = F + K'H, symmetrized (riccati.h SYMP); H waits in the group's B block (dead
          // since the residual products; the record image overwrites it only afterwards)
          riccati_step<1, true, greal>(P, A_, B_, loadR, loadSQ, lane, reg, f, NoMid{}, ldsB + lane * 12);
        }
        // The factor record goes through the group's LDS image (its A, B, S blocks are
        // dead by now) and leaves as whole 16-byte pieces instead of ~40 scattered
        // per-lane stores (the kRecP slot holds P, or its factor Lp for SQRT).
        lds_wave_fence();
        real* const img = kRecImg<GEN> ? ldsA : rec;
        if (lane < kMaxDim) {
          store_packed_col(img + kRecL, lane, f.Lc);
          store12(img + kRecK + lane * 12, f.Kc);
          if constexpr (!kRecFactor) store_packed_col(img + kRecP, lane, f.F);
          img[kRecRs + lane] = f.rs;
          if constexpr (kRecPbOn<SQRT>) img[kRecPb + lane] = pbk;
        }
        if (c.isv) {
          store12(img + kRecKv, f.Kc);
          store12(img + kRecPv, f.F);
        }
        if (!(SQRT && use_lq))  // (riccati_step_lq leaves the next factor in P)
          sfor<0, 12>([&](auto i) {
            constexpr int I = decltype(i)::value;
            P[I] = f.F[I];
          });
        if constexpr (SQRT) {
          if (!use_lq) sqrt_factor(P, lane);
          if constexpr (kRecFactor)
            if (lane < kMaxDim) store_packed_col(img + kRecP, lane, P);
        }
        lds_wave_fence();
        if constexpr (kRecImg<GEN>) rec_copy(rec, img, lane);
        // the next stage overwrites this group's LDS blocks: reads done first
        lds_wave_fence();
        tstamp(23);
      }
      xn = xk;
      pin = pik;
    }
    const real res_stat = gmax(lane < kMaxDim ? mg : real(0.0));
    const real res_eq = gmax(lane < kMaxDim ? mb : real(0.0));
    const real res_ineq = gmax(lane < kMaxDim ? md : real(0.0));
    const real res_comp = gmax(lane < kMaxDim ? mm : real(0.0));
    const real obj = gsum(lane < kMaxDim ? objl : real(0.0));
    const real musum_all = gsum(lane < kMaxDim ? musum : real(0.0));
    const real mu = musum_all * nc_inv;
    real* const stat_row = a.stat && lane == 0
                           ? a.stat + ((size_t)qp * a.stat_rows + iter) * kStatCols
                           : nullptr;
    if (stat_row) {
      stat_row[5] = mu;
      stat_row[6] = res_stat;
      stat_row[7] = res_eq;
      stat_row[8] = res_ineq;
      stat_row[9] = res_comp;
      stat_row[10] = obj;
    }
    // ---- exit test (HPIPM order: converged / iter_max / min step / NaN) ----
    {
      const bool isnan_ = !(res_stat == res_stat) || !(res_eq == res_eq) ||
                          !(res_ineq == res_ineq) || !(res_comp == res_comp) || !(mu == mu) ||
                          res_stat == real(__builtin_inf()) || res_eq == real(__builtin_inf());
      if (isnan_) {
        status = 3;
      } else if (res_stat <= a.tol_stat && res_eq <= a.tol_eq && res_ineq <= a.tol_ineq &&
                 res_comp <= a.tol_comp && (iter > 0 || a.warm_start != 2)) {
        // (a continued iterate -- warm_start 2, an fp32 pass's -- takes one fp64 step first)
        status = 0;
      } else if (iter >= a.iter_max) {
        status = 1;
      } else if (iter > 0 && last_amin < a.alpha_min) {
        status = 2;
      }
    }
    if (lane == 0) {
      qs[kQsMu] = mu;
      qs[kQsMuSum] = musum_all;
      qs[kQsResStat] = res_stat;
      qs[kQsResEq] = res_eq;
      qs[kQsResIneq] = res_ineq;
      qs[kQsResComp] = res_comp;
      qs[kQsObj] = obj;
      qs[kQsStatus] = (real)status;
    }

    return;
  }
  if constexpr (PH == kPhIR || PH == kPhIRP || PH == kPhIS || PH == kPhF3 || PH == kPhLqChk) {
    // ============== iterative refinement of the step (HPIPM itref_corr_max) ==============
    // The step (du, dx, dpi and the bounds' dt, dlam) solves the Newton system only up to the
    // factorization's rounding.  IR (one group per stage) forms the linear residual of that system at the
    // step in its full form -- QP Hessian and multiplier steps, not the Gamma-reduced one, so
    // no right-hand side of the corrector is needed again (the dt / dlam rows hold exactly by
    // construction, bar_step) --
    //   r_u = res_g,u + R du + S dx + B'dpi_{k+1} + D'(dlam_u - dlam_l)   (boxes: D = I)
    //   r_x = res_g,x + S'du + Q dx + A'dpi_{k+1} - dpi_k + C'(dlam_u - dlam_l)   (k >= 1)
    //   r_b = res_b + A dx + B du - dx_{k+1}
    // Its infinity norms decide, as in HPIPM: below the tolerances (or 1e-3 of the first
    // check's) the refinement stops.  Otherwise IS (k = N..0) runs the corrector's backward
    // recursion with (r_u, r_x, r_b) as its right-hand side (same factors: the record of this
    // iteration's RB) and F3 (k = 0..N) forms the correction, adds it to the step, updates
    // dt / dlam (linear in the primal step: ddt = +-ddv, ddlam = -lam ddt / t) and redoes the
    // step lengths.  (A check that passes costs IR alone: IS and F3 return at the top.)
    // (F2 advanced iter: the step's factorization has the parity of iter - 1.)
    // (kPhIRP / kPhLqChk: HPIPM's lq_fact 1 check of the predictor step -- IR's residual of the
    // predictor's system, then the switch -- for the QPs still on the Cholesky factorization)
    constexpr bool kPred = PH == kPhIRP || PH == kPhLqChk;
    if constexpr (kPred) {
      if (a.lq_fact != 1 || qs[kQsForceLq] != real(0.0)) return;
    } else if (qs[kQsItDone] != real(0.0)) {
      return;
    }
    // parity of the step's factorization: this iteration's (the predictor, before F2 advanced
    // iter) or the previous count's (after it); the other slot takes the residual
    const int fpar = kPred ? (iter & 1) : ((iter - 1) & 1);
    real* const next = !kPred && a.stat && lane == 0
                           ? a.stat + ((size_t)qp * a.stat_rows + iter) * kStatCols
                           : nullptr;
    if constexpr (PH == kPhLqChk) {
      // the predictor's linear residual above 1e-5 (or NaN): refactorize this iteration by LQ
      // and keep LQ for the rest of the solve (d_ocp_qp_ipm_solve, lq_fact 1); the redo launch
      // recomputes RB -> F1 from the same iterate (no step applied: alpha 0)
      real ng = real(0.0), nb = real(0.0);
      for (int k0 = 0; k0 <= N; k0 += kGroup) {
        const int k = k0 + lane;
        const real* slot = c.st(k <= N ? k : N) + (fpar ^ 1) * kRecSize;
        const real g1 = slot[36], b1 = slot[37];
        if (k <= N) {
          ng = fmax(ng, g1);
          nb = fmax(nb, b1);
        }
      }
      const real nga = gmax(ng), nba = gmax(nb);
      if (!(nga <= kLqSwitch) || !(nba <= kLqSwitch)) {
        if (lane == 0) {
          qs[kQsForceLq] = real(1.0);
          qs[kQsLqRedo] = real(1.0);
          qs[kQsAlphaP] = real(0.0);
          qs[kQsAlphaD] = real(0.0);
        }
      }
      return;
    } else if constexpr (PH == kPhIR || PH == kPhIRP) {
      // one 12 x 12 LDS block per QP group (A, B, S in turn): 18 KB per workgroup, so the
      // sweep runs at its register occupancy (RB's three blocks would cap it at 2 waves/SIMD)
      __shared__ real ir_lds[(256 / kGroup) * 144];
      real* const blk = ir_lds + (threadIdx.x / kGroup) * 144;
      real ng = real(0.0), nb = real(0.0);
      {
        const int k = kst;
        real* stk = c.st(k);
        const real* stn = c.st(k < N ? k + 1 : k);
        // the stage's element-owned loads first (valid addresses on every lane, masked after)
        const real du_ld = stk[kStStep + li], dx_ld = stk[kStStep + 12 + li], dpi_ld = stk[kStStep + 24 + li];
        const real dpin_ld = stn[kStStep + 24 + li], dxn_ld = stn[kStStep + 12 + li];
        const real rgu = stk[kStRes + li], rgx = stk[kStRes + 12 + li], rbk = stk[kStRes + 24 + li];
        const BarStep bdu = c.bstep(stk, 0, li), bdx = c.bstep(stk, 1, li);
        const Side su = c.side_u(k, lane), sx = c.side_x(k, lane);
        const bool el = lane < kMaxDim;
        const real duv = el && uel && k < N ? du_ld : real(0.0);
        const real dxv = el && xel && k > 0 ? dx_ld : real(0.0);
        const real dpinv = el && xel && k < N ? dpin_ld : real(0.0);
        real ru = rgu + su.mu * bdu.dlu - su.ml * bdu.dll;
        real rx = rgx + sx.mu * bdx.dlu - sx.ml * bdx.dll - dpi_ld;
        real rb = rbk - dxn_ld;
        if constexpr (GEN) {
          // the rows' multiplier steps: + D'(dlam_u - dlam_l) on the u rows, C'(..) on x
          for (int ch = 0; ch < c.nch; ++ch) {
            const real* g = c.gs(k, ch);
            const Side sg = c.side_g(k, ch, lane);
            const BarStep d = load_gstep(g, li);
            const real dl = lane < kMaxDim ? sg.mu * d.dlu - sg.ml * d.dll : real(0.0);
            real Cc[12], Dc[12];
            c.g_col(k, ch, col, Cc, Dc);
            ru = dot_bcast(Dc, dl, ru);
            if constexpr (GEN == 2) rx = dot_bcast(Cc, dl, rx);
          }
        }
        real Ac[12], Bc[12];
        if (k < N) {
          c.col(c.A() + (size_t)k * c.nxx(), nx, col, xel, Ac);
          c.col(c.B() + (size_t)k * c.nxu(), nx, col, uel, Bc);
          real Sc[12];
          c.col(c.S() + (size_t)k * c.nxu(), nu, col, xel, Sc);
          rx = dot_bcast(Ac, dpinv, rx);  // + A'dpi_{k+1}
          ru = dot_bcast(Bc, dpinv, ru);  // + B'dpi_{k+1}
          rx = dot_bcast(Sc, duv, rx);    // + S'du
          real M[12];
          lds_put_col(blk, lane, Ac);
          lds_wave_fence();
          lds_get_row(blk, li, M);
          rb = dot_bcast(M, dxv, rb);  // + A dx
          lds_wave_fence();
          lds_put_col(blk, lane, Bc);
          lds_wave_fence();
          lds_get_row(blk, li, M);
          rb = dot_bcast(M, duv, rb);  // + B du
          lds_wave_fence();
          lds_put_col(blk, lane, Sc);
          lds_wave_fence();
          lds_get_row(blk, li, M);
          ru = dot_bcast(M, dxv, ru);  // + S dx
          lds_wave_fence();
          real Rc[12];
          c.col(c.R() + (size_t)k * c.nuu(), nu, col, uel, Rc);
          ru = dot_bcast(Rc, duv, ru);  // + R du
        }
        {
          real Qc[12];
          c.col(c.Q() + (size_t)k * c.nxx(), nx, col, xel, Qc);
          rx = dot_bcast(Qc, dxv, rx);  // + Q dx
        }
        if (!(el && uel && k < N)) ru = real(0.0);
        if (!(el && xel && k > 0)) rx = real(0.0);  // (x_0 is fixed)
        if (!(el && xel && k < N)) rb = real(0.0);
        ng = fmax(ng, fmax(nabs(ru), nabs(rx)));
        nb = fmax(nb, nabs(rb));
        // the residual waits for the correction's recursion (kPhIS) and F3 in the other
        // parity's record slot (the previous factorization's, dead until the next RB
        // overwrites it): r_b, r_u, r_x
        // the stage's norms (slot[36], slot[37]) wait for IS, which decides
        const real ngk = gmax(ng), nbk = gmax(nb);
        real* slot = stk + (fpar ^ 1) * kRecSize;
        if (el) {
          slot[lane] = rb;
          slot[12 + lane] = ru;
          slot[24 + lane] = rx;
        }
        if (lane == 0) {
          slot[36] = ngk;
          slot[37] = nbk;
        }
      }
      return;
    } else if constexpr (PH == kPhIS) {
      // ---- the check's verdict: the stages' norms (lane l: stages l, l + 16, ...) ----
      real ng = real(0.0), nb = real(0.0);
      for (int k0 = 0; k0 <= N; k0 += kGroup) {
        const int k = k0 + lane;
        const real* slot = c.st(k <= N ? k : N) + (fpar ^ 1) * kRecSize;
        const real g1 = slot[36], b1 = slot[37];
        if (k <= N) {
          ng = fmax(ng, g1);
          nb = fmax(nb, b1);
        }
      }
      const real nga = gmax(ng), nba = gmax(nb);
      const int cnt = (int)qs[kQsItCnt];
      const real n0g = cnt == 0 ? nga : qs[kQsItN0g], n0b = cnt == 0 ? nba : qs[kQsItN0b];
      const bool small = (nga < a.tol_stat || nga < real(1e-3) * n0g) &&
                         (nba < a.tol_eq || nba < real(1e-3) * n0b);
      if (lane == 0) {
        if (cnt == 0) {
          qs[kQsItN0g] = nga;
          qs[kQsItN0b] = nba;
        }
        if (small) qs[kQsItDone] = real(1.0);
      }
      if (next) {  // HPIPM stat: lin_res_stat, lin_res_eq (the dt / dlam rows are exact)
        next[14] = nga;
        next[15] = nba;
      }
      if (small) return;  // (F3 returns on the flag)
      // ---- IS: the correction's backward recursion (B2's, right-hand side r_u, r_x, r_b) ----
      real pnext = real(0.0);
      for (int k = N; k >= 0; --k) {
        real* stk = c.st(k);
        real* rec = stk + fpar * kRecSize;
        const real* slot = stk + (fpar ^ 1) * kRecSize;
        const bool el = lane < kMaxDim;
        const real rb = el ? slot[li] : real(0.0), ru = el ? slot[12 + li] : real(0.0);
        const real rx = el ? slot[24 + li] : real(0.0);
        if (k == N) {
          pnext = rx;  // p_N = q~_N (the terminal P_N carries Q_N + Gamma)
          if (el) rec[kRecPv + lane] = pnext;
          continue;
        }
        real Ac[12], Bc[12];
        c.col(c.A() + (size_t)k * c.nxx(), nx, col, xel, Ac);
        c.col(c.B() + (size_t)k * c.nxu(), nx, col, uel, Bc);
        const real* recn = c.st(k + 1) + fpar * kRecSize;
        const real w = rec_P_mul(recn, rb, pnext);
        real g = ru, f = rx;
        dot_bcast2(Bc, Ac, w, g, f);
        if (lane >= kMaxDim) g = real(0.0);
        real Kc[12];
        load12(rec + kRecK + col * 12, Kc);
        const real pv = dot_bcast(Kc, g, f);
        real Lr[12], Lc[12];
        load_packed_lrow(rec + kRecL, li, Lr);
        load_packed_lcol(rec + kRecL, col, Lc);
        const real rs = rec[kRecRs + li];
        real y = g;
        sfor<0, 12>([&](auto kk) {
          constexpr int K = decltype(kk)::value;
          const real yk = bc<K>(apply_rs(y, rs));
          if (lane == K) y = yk;
          if (lane > K) y = fmadd(-Lr[K], yk, y);
        });
        sfor_down<0, 12>([&](auto kk) {
          constexpr int K = decltype(kk)::value;
          const real zk = bc<K>(apply_rs(y, rs));
          if (lane == K) y = zk;
          if (lane < K) y = fmadd(-Lc[K], zk, y);
        });
        const real kv = el && uel ? -y : real(0.0);
        if (el) {
          rec[kRecKv + lane] = kv;
          rec[kRecPv + lane] = xel ? pv : real(0.0);
        }
        pnext = xel ? pv : real(0.0);
      }
      return;
    } else {
      // ---- F3: the correction (forward, row-owned), added to the step ----
      real ap = real(1e30), ad = real(1e30);
      bool bad = false;
      real dxc = real(0.0);  // correction of dx_0: 0 (x0 fixed)
      // dt / dlam are linear in the primal step: ddt = +-ddv, ddlam = -lam ddt / t
      auto upd = [&](const Side& sd, const Bar& b, BarStep& d, real dv) {
        if (sd.ml != real(0.0)) {
          d.dtl += dv;
          d.dll -= b.ll * dv / b.tl;
        }
        if (sd.mu != real(0.0)) {
          d.dtu -= dv;
          d.dlu += b.lu * dv / b.tu;
        }
      };
      for (int k = 0; k <= N; ++k) {
        real* stk = c.st(k);
        const real* rec = stk + fpar * kRecSize;
        const real dpc = k > 0 ? rec_P_mul(rec, dxc, rec[kRecPv + li]) : real(0.0);
        real duc = real(0.0), dxn = real(0.0);
        if (k < N) {
          real Kr[12], Ar[12];
          sfor<0, 12>([&](auto j) {
            constexpr int J = decltype(j)::value;
            Kr[J] = rec[kRecK + J * 12 + li];
          });
          c.row(c.A() + (size_t)k * c.nxx(), nx, nx, li, xel, Ar);
          duc = rec[kRecKv + li];
          dxn = stk[(fpar ^ 1) * kRecSize + li];
          dot_bcast2(Kr, Ar, dxc, duc, dxn);
          if (!uel) duc = real(0.0);
          real Br[12];
          c.row(c.B() + (size_t)k * c.nxu(), nx, nu, li, xel, Br);
          dxn = dot_bcast(Br, duc, dxn);
        }
        if (!uel || k == N) duc = real(0.0);
        real dpcv = dpc;
        if (!xel) {
          dxn = real(0.0);
          dpcv = real(0.0);
        }
        if constexpr (GEN) {
          // the rows' steps: ddv = C ddx + D ddu
          for (int ch = 0; ch < c.nch; ++ch) {
            real* g = c.gs(k, ch);
            real Cr[12], Dr[12];
            c.g_row(k, ch, lane, Cr, Dr);
            const real dv = dot_bcast(Dr, duc, GEN == 2 ? dot_bcast(Cr, dxc, real(0.0)) : real(0.0));
            if (lane < kMaxDim) {
              const Side sg = c.side_g(k, ch, lane);
              const Bar bg = load_gbar(g, lane);
              BarStep d = load_gstep(g, lane);
              upd(sg, bg, d, dv);
              bad |= huge(d.dtl) || huge(d.dtu) || huge(d.dll) || huge(d.dlu);
              ratio(sg, bg, d, ap, ad);
              store_gstep(g, lane, d);
            }
          }
        }
        if (lane < kMaxDim) {
          const Side su = c.side_u(k, lane), sx = c.side_x(k, lane);
          const Bar bu = c.bar(stk, 0, lane), bx = c.bar(stk, 1, lane);
          BarStep nu_ = c.bstep(stk, 0, lane), nx_ = c.bstep(stk, 1, lane);
          const real du = stk[kStStep + lane] + duc, dx = stk[kStStep + 12 + lane] + dxc;
          const real dpi = k > 0 ? stk[kStStep + 24 + lane] + dpcv : real(0.0);
          upd(su, bu, nu_, k < N ? duc : real(0.0));
          upd(sx, bx, nx_, dxc);
          ratio(su, bu, nu_, ap, ad);
          ratio(sx, bx, nx_, ap, ad);
          bad |= huge(du) || huge(dx) || huge(dpi) || huge(nu_.dtl) || huge(nu_.dtu) || huge(nu_.dll) ||
                 huge(nu_.dlu);
          c.put_bstep(stk, 0, lane, nu_);
          c.put_bstep(stk, 1, lane, nx_);
          stk[kStStep + lane] = du;
          stk[kStStep + 12 + lane] = dx;
          stk[kStStep + 24 + lane] = dpi;
        }
        dxc = dxn;
      }
      ap = gmin(lane < kMaxDim ? ap : real(1e30));
      ad = gmin(lane < kMaxDim ? ad : real(1e30));
      if (gmax((lane < kMaxDim && bad) ? real(1.0) : real(0.0)) > real(0.0)) {
        ap = real(0.0);
        ad = real(0.0);
      }
      if (!a.split_step) {
        ap = fmin(ap, ad);
        ad = ap;
      }
      const real alpha_p_new = fmin(real(1.0), kStepTau * ap);
      const real alpha_d_new = fmin(real(1.0), kStepTau * ad);
      const int cnt = (int)qs[kQsItCnt] + 1;
      if (lane == 0) {
        qs[kQsAlphaP] = alpha_p_new;
        qs[kQsAlphaD] = alpha_d_new;
        qs[kQsLastAmin] = fmin(alpha_p_new, alpha_d_new);
        qs[kQsItCnt] = (real)cnt;
      }
      if (next) {
        next[3] = alpha_p_new;
        next[4] = alpha_d_new;
        next[13] = (real)cnt;  // HPIPM stat: itref_corr
      }
      return;
    }
  }
  const real mu = qs[kQsMu], musum_all = qs[kQsMuSum];
  real sigma_mu = qs[kQsSigmaMu];
  if constexpr (PH == kPhB2) {
        // ---- B2: corrector vectors (element-owned recursion) ----
        real pnext = real(0.0);  // p_{k+1}, element-owned
        {
          real* stN = c.st(N);
          const Side sx = c.side_x(N, lane);
          const real xv = xel && c.has_bars(1) ? c.x()[(size_t)N * nx + lane] : real(0.0);
          real G = real(0.0), g = real(0.0);
          if (lane < kMaxDim) {
            const BarStep dx = c.bstep(stN, 1, lane);
            gamma_of(sx, c.bar(stN, 1, lane), xv, dx.dll * dx.dtl, dx.dlu * dx.dtu, sigma_mu, G, g);
          }
          pnext = lane < kMaxDim && xel ? stN[kStRes + 12 + lane] + g : real(0.0);
          if constexpr (GEN == 2) {
            // (C = NULL: the terminal stage has no general-row gradient, D_N is absent)
            real ra, qa;
            g_grad(N, true, sigma_mu, ra, qa);
            if (lane < kMaxDim && xel) pnext += qa;
          }
          if (lane < kMaxDim) stN[par * kRecSize + kRecPv + lane] = pnext;
        }
        for (int k = N - 1; k >= 0; --k) {
          tstamp(40);
          real* stk = c.st(k);
          real* rec = stk + par * kRecSize;
          [[maybe_unused]] const real* recn = c.st(k + 1) + par * kRecSize;
          // the stage's element-owned loads, all issued before any is waited for (valid
          // addresses on every lane, masked after; a load under a lane condition would be a
          // branch that waits for it)
          const Side su = c.side_u(k, lane), sx = c.side_x(k, lane);
          const int iu = li < nu ? li : 0, ix = li < nx ? li : 0;
          const real u_ld = c.u()[(size_t)k * nu + iu], x_ld = c.x()[(size_t)k * nx + ix];
          const Bar bu = c.bar(stk, 0, li), bx = c.bar(stk, 1, li);
          const BarStep du = c.bstep(stk, 0, li), dx = c.bstep(stk, 1, li);
          const real r_ld = stk[kStRes + li], q_ld = stk[kStRes + 12 + li], b_ld = stk[kStRes + 24 + li];
          real gv_ld = real(0.0);
          if constexpr (GEN == 1) {
            // D'gamma_corr = D'gamma_pred + sigma mu D'e + D'z (gamma is affine in both)
            const real* v = c.gv(k);
            gv_ld = v[li] + v[24 + li] + sigma_mu * v[12 + li];
          }
          // x, u enter only through the barrier terms of the bound families present
          const real uv = uel && c.has_bars(0) ? u_ld : real(0.0);
          const real xv = xel && c.has_bars(1) ? x_ld : real(0.0);
          real Gu = real(0.0), gu = real(0.0), Gx = real(0.0), gx = real(0.0);
          if (lane < kMaxDim) {
            gamma_of(su, bu, uv, du.dll * du.dtl, du.dlu * du.dtu, sigma_mu, Gu, gu);
            gamma_of(sx, bx, xv, dx.dll * dx.dtl, dx.dlu * dx.dtu, sigma_mu, Gx, gx);
          }
          real rt = lane < kMaxDim && uel ? r_ld + gu : real(0.0);
          real qt = lane < kMaxDim && xel ? q_ld + gx : real(0.0);
          if constexpr (GEN == 1) {
            if (lane < kMaxDim && uel) rt += gv_ld;
          } else if constexpr (GEN) {
            real ra, qa;
            g_grad(k, true, sigma_mu, ra, qa);
            if (lane < kMaxDim && uel) rt += ra;
            if (lane < kMaxDim && xel) qt += qa;
          }
          [[maybe_unused]] const real bt = lane < kMaxDim ? b_ld : real(0.0);
          // w = P_{k+1} b~ + p_{k+1} (P_{k+1} b~ from RB, classical Riccati)
          real w;
          if constexpr (kRecPbOn<SQRT>) {
            w = rec[kRecPb + li] + pnext;
          } else {
            w = rec_P_mul(recn, bt, pnext);
          }
          // g = r~ + B'w ; f = q~ + A'w
          real Bc[12], Ac[12];
          c.col(c.B() + (size_t)k * c.nxu(), nx, col, uel, Bc);
          c.col(c.A() + (size_t)k * c.nxx(), nx, col, xel, Ac);
          real g = rt, f = qt;
          dot_bcast2(Bc, Ac, w, g, f);
          if (lane >= kMaxDim) g = real(0.0);
          // p = f + K'g  (K column-owned: lane j holds K[:, j])
          real Kc[12];
          load12(rec + kRecK + col * 12, Kc);
          const real pv = dot_bcast(Kc, g, f);
          // y = L^-1 g (row-owned L), then z = L^-T y (column-owned L), k = -z
          real Lr[12], Lc[12];
          load_packed_lrow(rec + kRecL, li, Lr);
          load_packed_lcol(rec + kRecL, col, Lc);
          const real rs = rec[kRecRs + li];
          real y = g;
          sfor<0, 12>([&](auto kk) {
            constexpr int K = decltype(kk)::value;
            const real yk = bc<K>(apply_rs(y, rs));
            if (lane == K) y = yk;
            if (lane > K) y = fmadd(-Lr[K], yk, y);
          });
          sfor_down<0, 12>([&](auto kk) {
            constexpr int K = decltype(kk)::value;
            const real zk = bc<K>(apply_rs(y, rs));
            if (lane == K) y = zk;
            if (lane < K) y = fmadd(-Lc[K], zk, y);
          });
          const real kv = lane < kMaxDim && uel ? -y : real(0.0);
          if (lane < kMaxDim) {
            rec[kRecKv + lane] = kv;
            rec[kRecPv + lane] = xel ? pv : real(0.0);
          }
          pnext = xel ? pv : real(0.0);
        }
    return;
  }
  if constexpr (PH == kPhF1 || PH == kPhF2) {
    constexpr bool corr = PH == kPhF2;
    // F1 with C-free general rows: D'z goes through the group's first LDS block
    real* const f1_lds_grp = group_lds_blocks<GEN>();
    real ap = real(1e30), ad = real(1e30);
    real s1 = real(0.0), s2 = real(0.0);  // predictor sums lam dt + t dlam, dlam dt (element-owned)
    bool bad = false;  // a non-finite component in the final step (fp32 breakdown)
    // the step is kept (kStStep): the final one (F2, or F1 without corrector), or the
    // predictor whose linear residual decides HPIPM's lq_fact 1 switch (kPhIRP / kPhLqChk)
    const bool final_step = corr || !a.pred_corr;
    const bool lq_chk = !corr && a.lq_fact == 1 && !a.lq_redo && qs[kQsForceLq] == real(0.0);
    const bool keep_step = final_step || lq_chk;
      // ---- forward step (F1 predictor / F2 corrector), row-owned ----
      ap = real(1e30);
      ad = real(1e30);
      real dxk = real(0.0);  // dx_0 = 0 (x0 fixed)
      for (int k = 0; k <= N; ++k) {
        tstamp(corr ? 31 : 30);
        real* stk = c.st(k);
        const real* rec = stk + par * kRecSize;
        // dpi = P dx + p is part of the final step only (F2, or F1 without corrector)
        real dpi = real(0.0);
        if (keep_step) dpi = rec_P_mul(rec, dxk, rec[kRecPv + li]);
        real du = real(0.0), dxn = real(0.0);
        if (k < N) {
          // du = K dx + k, dx+ = A dx + B du + b~ (open loop: the QP's own A, B; b~ = res_b,
          // unchanged between predictor and corrector)
          real Kr[12], Ar[12];
          sfor<0, 12>([&](auto j) {
            constexpr int J = decltype(j)::value;
            Kr[J] = rec[kRecK + J * 12 + li];
          });
          c.row(c.A() + (size_t)k * c.nxx(), nx, nx, li, xel, Ar);
          du = rec[kRecKv + li];
          dxn = stk[kStRes + 24 + li];
          dot_bcast2(Kr, Ar, dxk, du, dxn);
          if (!uel) du = real(0.0);
          real Br[12];
          c.row(c.B() + (size_t)k * c.nxu(), nx, nu, li, xel, Br);
          dxn = dot_bcast(Br, du, dxn);
        }
        if (!uel || k == N) du = real(0.0);
        if (!xel) {
          dxn = real(0.0);
          dpi = real(0.0);
        }
        if constexpr (GEN) {
          // general rows: dv = C dx + D du, dt / dlam, step ratios
          // (GEN == 1, F1: z_i = ml dlam_l dt_l / t_l - mu dlam_u dt_u / t_u and D'z, the
          // predictor-product part of the corrector's D'gamma, for B2)
          constexpr bool kZ = GEN == 1 && !corr;
          real gza = real(0.0);
          for (int ch = 0; ch < c.nch; ++ch) {
            real* g = c.gs(k, ch);
            real Cr[12], Dr[12];
            c.g_row(k, ch, lane, Cr, Dr);
            const real dv = dot_bcast(Dr, du, GEN == 2 ? dot_bcast(Cr, dxk, real(0.0)) : real(0.0));
            real z = real(0.0);
            if (lane < kMaxDim) {
              const Side sg = c.side_g(k, ch, lane);
              const Bar bg = load_gbar(g, lane);
              real el = real(0.0), eu = real(0.0), sm = real(0.0);
              if (corr) {
                const BarStep pd = load_gstep(g, lane);
                el = pd.dll * pd.dtl;
                eu = pd.dlu * pd.dtu;
                sm = sigma_mu;
              }
              const BarStep d = bar_step(sg, bg, g[kGenVal + lane], dv, el, eu, sm);
              bad |= huge(d.dtl) || huge(d.dtu) || huge(d.dll) || huge(d.dlu);
              ratio(sg, bg, d, ap, ad);
              if (!corr) aff_sums(sg, bg, d, s1, s2);
              store_gstep(g, lane, d);
              if constexpr (kZ) {
                if (sg.ml != real(0.0)) z += d.dll * d.dtl / bg.tl;
                if (sg.mu != real(0.0)) z -= d.dlu * d.dtu / bg.tu;
              }
            }
            if constexpr (kZ) {
              // (D'z)_j = sum_i D[i][j] z_i: row i's products through this group's LDS
              // block, summed down column j by lane j
              real Y[12], M[12];
              sfor<0, 12>([&](auto j) { Y[decltype(j)::value] = Dr[decltype(j)::value] * z; });
              lds_put_col(f1_lds_grp, lane, Y);
              lds_wave_fence();
              lds_get_row(f1_lds_grp, li, M);
              sfor<0, 12>([&](auto i) { gza += M[decltype(i)::value]; });
              lds_wave_fence();
            }
          }
          if constexpr (kZ) {
            if (lane < kMaxDim) c.gv(k)[24 + lane] = gza;
          }
        }
        if (lane < kMaxDim) {
          const Side su = c.side_u(k, lane), sx = c.side_x(k, lane);
          const Bar bu = c.bar(stk, 0, lane), bx = c.bar(stk, 1, lane);
          const real uv = (uel && k < N && c.has_bars(0)) ? c.u()[(size_t)k * nu + lane] : real(0.0);
          const real xv = xel && c.has_bars(1) ? c.x()[(size_t)k * nx + lane] : real(0.0);
          real eul = real(0.0), euu = real(0.0), exl = real(0.0), exu = real(0.0), smu = real(0.0);
          if (corr) {
            const BarStep pu = c.bstep(stk, 0, lane), px = c.bstep(stk, 1, lane);
            eul = pu.dll * pu.dtl;
            euu = pu.dlu * pu.dtu;
            exl = px.dll * px.dtl;
            exu = px.dlu * px.dtu;
            smu = sigma_mu;
          }
          const BarStep nu_ = bar_step(su, bu, uv, du, eul, euu, smu);
          const BarStep nx_ = bar_step(sx, bx, xv, dxk, exl, exu, smu);
          ratio(su, bu, nu_, ap, ad);
          ratio(sx, bx, nx_, ap, ad);
          if (!corr) {
            aff_sums(su, bu, nu_, s1, s2);
            aff_sums(sx, bx, nx_, s1, s2);
          }
          c.put_bstep(stk, 0, lane, nu_);
          c.put_bstep(stk, 1, lane, nx_);
          if (final_step)
            bad |= huge(du) || huge(dxk) || huge(dpi) || huge(nu_.dtl) || huge(nu_.dtu) ||
                   huge(nu_.dll) || huge(nu_.dlu);
          if (keep_step) {  // (otherwise the predictor's du / dx / dpi are not used)
            stk[kStStep + lane] = du;
            stk[kStStep + 12 + lane] = dxk;
            stk[kStStep + 24 + lane] = k > 0 ? dpi : real(0.0);
          }
        }
        dxk = dxn;
      }
    real* const next = a.stat && lane == 0
                             ? a.stat + ((size_t)qp * a.stat_rows + iter + 1) * kStatCols
                             : nullptr;  // HPIPM stores step kk in row kk+1
    if (!corr) {
      // alpha_aff, mu_aff, sigma: sum (lam + a dlam)(t + a dt) = S0 + a S1 + a^2 S2
      const real aa = fmin(real(1.0), fmin(gmin(ap), gmin(ad)));
      const real S1 = gsum(lane < kMaxDim ? s1 : real(0.0)), S2 = gsum(lane < kMaxDim ? s2 : real(0.0));
      const real mu_aff = (musum_all + aa * (S1 + aa * S2)) * nc_inv;
      real sg = mu > real(0.0) ? mu_aff / mu : real(0.0);
      sg = sg * sg * sg;
      if (sg > real(1.0)) sg = real(1.0);
      if (lane == 0) qs[kQsSigmaMu] = sg * mu;
      if (next && a.pred_corr) {
        next[0] = aa;
        next[1] = mu_aff;
        next[2] = sg;
      }
      if (next) next[11] = qs[kQsForceLq] != real(0.0) ? real(1.0) : real(0.0);  // HPIPM stat: lq_fact
      if (a.lq_redo && lane == 0) qs[kQsLqRedo] = real(0.0);
    }
    if (corr || !a.pred_corr) {
      // ---- step length of the iteration ----
      ap = gmin(lane < kMaxDim ? ap : real(1e30));
      ad = gmin(lane < kMaxDim ? ad : real(1e30));
      // A step with a NaN component, or one whose square overflows the precision (an
      // fp32 factorization that broke down on a barrier Hessian of ~1e10), is not a
      // direction: take none, so the iterate stays finite and the next exit test stops
      // with MinStepLengthReached.
      if (gmax((lane < kMaxDim && bad) ? real(1.0) : real(0.0)) > real(0.0)) {
        ap = real(0.0);
        ad = real(0.0);
      }
      if (!a.split_step) {
        ap = fmin(ap, ad);
        ad = ap;
      }
      const real alpha_p_new = fmin(real(1.0), kStepTau * ap);
      const real alpha_d_new = fmin(real(1.0), kStepTau * ad);
      if (lane == 0) {
        qs[kQsAlphaP] = alpha_p_new;
        qs[kQsAlphaD] = alpha_d_new;
        qs[kQsLastAmin] = fmin(alpha_p_new, alpha_d_new);
        qs[kQsIter] = (real)(iter + 1);
        qs[kQsItCnt] = real(0.0);  // this step's refinement (kPhIR / kPhF3) starts afresh
        qs[kQsItDone] = real(0.0);
      }
      if (next) {
        next[3] = alpha_p_new;
        next[4] = alpha_d_new;
      }
    }
  }
}


// fp64: 2 workgroups per CU (<= 256 VGPRs); fp32 boxes / C-free rows: 3 (<= 168 VGPRs, 3 waves
// per SIMD -- the fp32 RB sweep sits just under that cliff and a free allocator crosses it:
// cone 175 -> 194 ms; with the fp64 stage factorization of C-free rows the sweep needs 178
// and spills 60-76 B at 168, still faster than 2 waves: cone 188.6 vs 205.7 ms); fp32 rows
// with C need 216 and stay at 2
template <int GEN>
constexpr int kIpmMinBlocks = sizeof(real) == 4 && GEN < 2 ? 3 : 2;

// Live-QP report after an RB sweep (ProblemArgsT::ctl): one count per workgroup with a QP
// still running; the workgroup that finishes last marks the solve done when none is left.
// Every thread of the workgroup reaches this (the phase functions return, the kernels do not).
__device__ __forceinline__ void report_running(const ProblemArgsT<real>& a) {
  if (!a.ctl) return;
  const int qp = group_qp(a);
  bool run = false;
  if ((threadIdx.x & (kGroup - 1)) == 0 && qp >= 0)  // the lane that wrote the status
    run = a.ws[(size_t)qp * a.ws_qp + kQsStatus] < real(0.0);
  const int any = __syncthreads_or(run);
  if (threadIdx.x == 0) {
    int* cnt = a.ctl + 2 * a.launch_it;
    if (any) atomicAdd(cnt, 1);
    __threadfence();
    if (atomicAdd(cnt + 1, 1) == (int)gridDim.x - 1) {
      __threadfence();
      if (atomicAdd(cnt, 0) == 0)  // no workgroup has a QP still running
        __hip_atomic_store(a.ctl + kCtlDone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// A sweep launched after every QP of the solve has exited returns at once (a uniform load of
// one control word; the launch costs its dispatch only).
__device__ __forceinline__ bool solve_done(const ProblemArgsT<real>& a) {
  return a.ctl && __atomic_load_n(a.ctl + kCtlDone, __ATOMIC_RELAXED) != 0;
}

template <bool FULL, int GEN, int PH, bool SQRT = false, int LQ = 0>
__global__ void __launch_bounds__(256, FULL ? kIpmMinBlocks<GEN> : 1) ipm_phase_kernel(ProblemArgsT<real> a) {
  if constexpr (PH == kPhInit) {  // this solve's live-QP counters and control words start at 0
    if (a.ctl)
      for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kCtlInts; i += gridDim.x * blockDim.x)
        a.ctl[i] = i == kCtlCur ? (int)gridDim.x : 0;  // cur: the full grid
  }
  if constexpr (PH != kPhInit && PH != kPhOut)
    if (solve_done(a)) return;
  ipm_phase<FULL, GEN, PH, SQRT, LQ>(a);
  if constexpr (PH == kPhRB && LQ != 3) report_running(a);  // (3: counted by the 1 launch)
}

// Two consecutive sweeps of one iteration in one launch (RB -> F1, B2 -> F2):
// the forward sweep starts on the stages the backward sweep touched last, while
// their records are still in L2 / the Infinity Cache, and the launch count halves.
// The second phase re-reads the per-QP state the first one wrote (same wave:
// visible after the workgroup-scope fence).
template <bool FULL, int GEN, int PH1, int PH2, bool SQRT = false, int LQ = 0>
__global__ void __launch_bounds__(256, FULL ? kIpmMinBlocks<GEN> : 1) ipm_phase2_kernel(ProblemArgsT<real> a) {
  if (solve_done(a)) return;
  ipm_phase<FULL, GEN, PH1, SQRT, LQ>(a);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  ipm_phase<FULL, GEN, PH2, SQRT, LQ>(a);
  if constexpr (PH1 == kPhRB && LQ != 3)  // (lq_fact 1: the LQ launch's QPs are counted, as
    if (!a.lq_redo) report_running(a);   // running, by the Cholesky launch before it)
}

// Active-QP compaction, decided on the device after the RB sweep of iteration `it`: when the
// workgroups with a live QP are at most 3/4 of the workgroups the current grid (or list) keeps
// busy, the list is rebuilt and the later sweeps run on it.  compact_decide_kernel (one
// thread) decides and clears the list's count; compact_running_kernel then lists every QP
// whose status is still "running", in no particular order (a QP's arithmetic does not depend
// on its place in the grid), the count at buf[batch], one atomic add per wave.
__global__ void __launch_bounds__(64) compact_decide_kernel(int* __restrict__ ctl, int it, int* __restrict__ buf,
                                                           int batch) {
  if (threadIdx.x != 0) return;
  const int live = ctl[2 * it], cur = ctl[kCtlCur];
  const bool rebuild = ctl[kCtlDone] == 0 && live > 0 && 4 * (long long)live <= 3 * (long long)cur;
  ctl[kCtlRebuild] = rebuild;
  if (rebuild) {
    buf[batch] = 0;
    ctl[kCtlListOn] = 1;
    ctl[kCtlCur] = live;
  }
}
__global__ void __launch_bounds__(256) compact_running_kernel(const real* __restrict__ ws, size_t ws_qp,
                                                              int batch, int* __restrict__ buf,
                                                              const int* __restrict__ ctl) {
  if (ctl[kCtlRebuild] == 0) return;
  const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const bool run = q < batch && ws[(size_t)q * ws_qp + kQsStatus] < real(0.0);
  const unsigned long long m = __ballot(run);
  const int lane = (int)(threadIdx.x & 63);
  int base = 0;
  if (lane == 0 && m) base = atomicAdd(buf + batch, __popcll(m));
  base = __shfl(base, 0);
  if (run) buf[base + __popcll(m & ((1ull << lane) - 1))] = q;
}

// diagnostic builds (-DSRBD_IPM_SPLIT=1, scripts/profile_ipm.sh): every sweep its own launch
#ifndef SRBD_IPM_SPLIT
#define SRBD_IPM_SPLIT 0
#endif
constexpr bool kIpmSplit = SRBD_IPM_SPLIT != 0;

template <bool FULL, int GEN, bool SQRT, int LQ>
static hipError_t launch_phases(const ProblemArgsT<real>& a, hipStream_t stream) {
  const int threads = 256;
  const long long lanes = (long long)a.batch * kGroup;
  const dim3 full_grid((unsigned)((lanes + threads - 1) / threads)), block(threads);
  const dim3 grid = full_grid;
  // Each sweep is its own launch, so every kernel gets the registers (and occupancy) of its
  // own phase; QPs that have exited return at the top of every later launch.  iter_max + 1
  // factorization sweeps at most: the last one always decides (converged or MaxIterReached).
  // The whole sequence is enqueued at once and the host never waits (the call is
  // asynchronous on `stream`): the stop decision lives on the device (ProblemArgsT::ctl):
  // once an RB sweep leaves no QP running, every later sweep returns at its first
  // instruction, so a finished solve's remaining launches cost their dispatch only.
  const bool ctl = a.ctl && a.iter_max < a.ctl_cap;

  ProblemArgsT<real> b = a;
  if (!ctl) b.ctl = nullptr;
  b.launch_it = 0;
  // Active-QP compaction (compact_decide_kernel): once the workgroups with a live QP are at
  // most 3/4 of the ones the grid keeps busy, the sweeps run on a list of the running QPs
  // (the grid keeps its size: groups past the list's count return at the top).  A wave then
  // carries four live QPs instead of the one or two a thinned-out batch leaves it.  Only for
  // grids large enough to thin out (>= 64 workgroups, 1024 QPs); smaller solves skip the
  // two launches per iteration.
  const bool compact = ctl && a.qp_buf && full_grid.x >= 64;
  // (init covers every QP and clears the control words: no list, whatever they held before)
  b.qp_list = nullptr;
  hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhInit>), grid, block, 0, stream, b);
  b.qp_list = compact ? a.qp_buf : nullptr;
  // (SQRT changes RB and how B2, F1, F2 and the outputs apply the record's P)
  for (int it = 0;; ++it) {
    b.launch_it = it;
    if (it >= a.iter_max) {
      if (!a.skip_last_rb) {
        hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhRB, SQRT, LQ>), grid, block, 0, stream, b);
        if constexpr (LQ == 1)  // (lq_fact 1: the switched QPs' RB by LQ)
          hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhRB, SQRT, 3>), grid, block, 0, stream, b);
      }
      break;
    }
    if (kIpmSplit) {  // diagnostic schedule: one launch per sweep
      hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhRB, SQRT, LQ>), grid, block, 0, stream, b);
      hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhF1, SQRT, LQ>), grid, block, 0, stream, b);
    } else {
      hipLaunchKernelGGL((ipm_phase2_kernel<FULL, GEN, kPhRB, kPhF1, SQRT, LQ>), grid, block, 0, stream, b);
    }
    if constexpr (LQ == 1) {
      // HPIPM lq_fact 1: RB -> F1 by LQ of the QPs switched in an earlier iteration, then the
      // predictor step's linear residual of the others (stage-parallel, IR's arithmetic), the
      // switch, and RB -> F1 again by LQ for the QPs it switched (from the same iterate)
      hipLaunchKernelGGL((ipm_phase2_kernel<FULL, GEN, kPhRB, kPhF1, SQRT, 3>), grid, block, 0, stream, b);
      hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhIRP, SQRT>), dim3(grid.x * (unsigned)(a.N + 1)), block,
                         0, stream, b);
      hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhLqChk, SQRT>), grid, block, 0, stream, b);
      ProblemArgsT<real> r = b;
      r.lq_redo = 1;
      hipLaunchKernelGGL((ipm_phase2_kernel<FULL, GEN, kPhRB, kPhF1, SQRT, 3>), grid, block, 0, stream, r);
    }
    if (compact) {  // RB(it) has counted its live workgroups: compact for the rest of the solve?
      hipLaunchKernelGGL(compact_decide_kernel, dim3(1), dim3(64), 0, stream, a.ctl, it, a.qp_buf, a.batch);
      hipLaunchKernelGGL(compact_running_kernel, dim3((unsigned)((a.batch + 255) / 256)), dim3(256), 0, stream,
                         a.ws, a.ws_qp, a.batch, a.qp_buf, a.ctl);
    }
    if (a.pred_corr && kIpmSplit) {
      hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhB2, SQRT>), grid, block, 0, stream, b);
      hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhF2, SQRT>), grid, block, 0, stream, b);
    } else if (a.pred_corr) {
      hipLaunchKernelGGL((ipm_phase2_kernel<FULL, GEN, kPhB2, kPhF2, SQRT>), grid, block, 0, stream, b);
    }
    // HPIPM's iterative refinement of the corrector step (Balance / Robust): at
    // most itref_corr_max corrections, each after a check of the step's linear residual; a
    // QP whose check passed returns at the top of the later ones
    if (a.pred_corr)
      for (int r = 0; r < a.itref_corr_max; ++r) {
        hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhIR, SQRT>), dim3(grid.x * (unsigned)(a.N + 1)),
                           block, 0, stream, b);
        hipLaunchKernelGGL((ipm_phase2_kernel<FULL, GEN, kPhIS, kPhF3, SQRT>), grid, block, 0, stream, b);
      }
  }
  b.qp_list = nullptr;  // outputs for every QP
  hipLaunchKernelGGL((ipm_phase_kernel<FULL, GEN, kPhOut, SQRT>), full_grid, block, 0, stream, b);
  return hipGetLastError();
}

// HPIPM's lq_fact (the C-ABI derives it from the mode, with ric_alg != 0 only)
template <bool FULL, int GEN>
static hipError_t launch_alg(const ProblemArgsT<real>& a, hipStream_t stream) {
  if (!a.ric_alg) return launch_phases<FULL, GEN, false, 0>(a, stream);
  if (a.lq_fact == 2) return launch_phases<FULL, GEN, true, 2>(a, stream);
  if (a.lq_fact == 1) return launch_phases<FULL, GEN, true, 1>(a, stream);
  return launch_phases<FULL, GEN, true, 0>(a, stream);
}

hipError_t launch(const ProblemArgsT<real>& a, hipStream_t stream) {
  if (a.batch <= 0) return hipSuccess;
  // 12 x 12 stages only: smaller problems arrive embedded by pad.hip
  if (a.nx != 12 || a.nu != 12) return hipErrorInvalidValue;
  // general rows: GEN 2 with C, GEN 1 when C is absent (NULL = 0, e.g. the friction
  // cone, SRBD_model.cpp:237-260, which constrains u only)
  if (a.ng > 0 && a.C) return launch_alg<true, 2>(a, stream);
  if (a.ng > 0) return launch_alg<true, 1>(a, stream);
  return launch_alg<true, 0>(a, stream);
}

}  // namespace SRBD_NS
}  // namespace srbd
