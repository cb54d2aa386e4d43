// riccati_unconstr_impl.h -- body of the unconstrained batched solve, instantiated
// per precision by riccati_unconstr.hip (SRBD_REAL, SRBD_NS).  No include guard.
//
// Two kernels share one per-QP body (solve_qp), differing only in where a QP's stage
// blocks and forward records live:
//   riccati_unconstr_kernel      (HbmSrc)  large batches: 16 lanes per QP, 16 QPs per
//                                          workgroup; blocks streamed from HBM, records
//                                          in the stage-major HBM workspace (fp64: each
//                                          wave writes its four records through an LDS
//                                          image as whole 16-byte pieces).
//   riccati_unconstr_lds_kernel  (LdsSrc)  small batches (the reference's one QP per
//                                          solve() call): one QP per workgroup; the whole
//                                          QP is first copied into an LDS image with
//                                          global->LDS DMA, the records overwrite the
//                                          stage slots they were computed from.  The
//                                          per-stage memory latency (three dependent HBM
//                                          round trips per backward stage) becomes an
//                                          LDS latency.
// Same instructions on the same values: the two kernels' outputs are bit-identical
// (tests/test_gpu_riccati.py::test_latency_kernel_bit_identical).
namespace srbd {
namespace SRBD_NS {

using real = SRBD_REAL;

// ---- where a QP's blocks and records are ----

// HBM, the C-ABI layout: QP-major ([batch][stage][blk], Eigen order) or stage-major
// ([stage][batch][blk]).  Records stage-major across the batch: stage k of QP q at
// ws[(k * batch + q) * kWsStage], so a wavefront's four QPs write / read one
// contiguous block per stage.
struct HbmSrc {
  const ProblemArgsT<real>& a;
  int qp;
  __device__ const real* at(const real* base, int nstage, int blk, int k) const {
    return a.layout == 1 ? base + ((size_t)k * a.batch + qp) * blk
                         : base + ((size_t)qp * nstage + k) * blk;
  }
  __device__ const real* A(int k) const { return at(a.A, a.N, 144, k); }
  __device__ const real* B(int k) const { return at(a.B, a.N, 144, k); }
  __device__ const real* b(int k) const { return at(a.b, a.N, 12, k); }
  __device__ const real* Q(int k) const { return at(a.Q, a.N + 1, 144, k); }
  __device__ const real* S(int k) const { return at(a.S, a.N, 144, k); }
  __device__ const real* R(int k) const { return at(a.R, a.N, 144, k); }
  __device__ const real* q(int k) const { return at(a.q, a.N + 1, 12, k); }
  __device__ const real* r(int k) const { return at(a.r, a.N, 12, k); }
  __device__ real* rec(int k) const { return a.ws + ((size_t)k * a.batch + qp) * kWsStage; }
  // fp64 large-batch kernel: the wave's LDS image of its four QPs' records (null: plain
  // stores)
  real* img = nullptr;  // the wave's image base: group g's record at img + g * kWsStage
  int gq = 0;           // QP group in the wave
  // stage k's record, `store` writing it at a given base (defined after store_rec below)
  template <class StoreRec>
  __device__ void store_stage(int k, StoreRec&& store) const;
};

// LDS image of one QP: stage slot k (k = 0..N) holds the stage's blocks at the offsets
// below (slot N: Q and q only); after the backward sweep has used slot k's Q, S, R, the
// stage's forward record (kernels.h kWs*, 246 reals) is written over them (A, B, b stay
// for the forward sweep's x+ = A x + B u + b).
constexpr int kImgA = 0, kImgB = 144, kImgb = 288, kImgQ = 300, kImgS = 444, kImgR = 588,
              kImgq = 732, kImgr = 744, kImgStage = 756, kImgRec = kImgQ;
static_assert(kImgRec + kWsStage <= kImgStage, "a record fits its stage slot past A, B, b");

struct LdsSrc {
  real* img;
  // records in the HBM workspace instead of over the image's Q, S, R (the fused-residual
  // kernel, whose residual pass reads those blocks after the forward sweep): stage-major
  // like HbmSrc, null = in the image
  real* grec = nullptr;
  int batch = 0, qp = 0;
  __device__ real* slot(int k) const { return img + k * kImgStage; }
  __device__ const real* A(int k) const { return slot(k) + kImgA; }
  __device__ const real* B(int k) const { return slot(k) + kImgB; }
  __device__ const real* b(int k) const { return slot(k) + kImgb; }
  __device__ const real* Q(int k) const { return slot(k) + kImgQ; }
  __device__ const real* S(int k) const { return slot(k) + kImgS; }
  __device__ const real* R(int k) const { return slot(k) + kImgR; }
  __device__ const real* q(int k) const { return slot(k) + kImgq; }
  __device__ const real* r(int k) const { return slot(k) + kImgr; }
  __device__ real* rec(int k) const {
    return grec ? grec + ((size_t)k * batch + qp) * kWsStage : slot(k) + kImgRec;
  }
};

// ---- stage records ----
// The terminal record (P_N, p_N) and, in solve_qp, every stage record by plain stores:
// column owner j stores K[i][j] at row i's slot j, the vector lane k[i] at slot 12
// (kernels.h kWs*); P by packed columns (rows >= j), p on the vector lane.
__device__ __forceinline__ void store_rec_P(real* rec, int lane, const real (&P)[12]) {
  if (lane < kMaxDim) store_packed_col(rec + kWsP, lane, P);
  if (lane == kVecLane) store12(rec + kWsp, P);
}
__device__ __forceinline__ void store_rec(real* rec, int lane, const real (&Kc)[12], const real (&P)[12]) {
  const bool isv = lane == kVecLane;
  if (lane < kMaxDim || isv) {
    const int c = isv ? kMaxDim : lane;
    sfor<0, 12>([&](auto m) {
      constexpr int M = decltype(m)::value;
      rec[kWsK + M * kWsRow + c] = Kc[M];
    });
  }
  store_rec_P(rec, lane, P);
}

constexpr int kRecHotStages = 4;

// A stage record by plain stores, or (img set) through the wave's LDS image: the four
// groups write their records into the image, then the wave stores the four records, which
// are contiguous in the stage-major workspace, as whole 16-byte pieces in lane order.
template <class StoreRec>
__device__ void HbmSrc::store_stage(int k, StoreRec&& store) const {
  if (!img) {
    store(rec(k));
    return;
  }
  store(img + gq * kWsStage);
  // the copy below reads other groups' parts of the image: LDS executes the wave's
  // instructions in order, so only the compiler must not move accesses across this point
  lds_wave_fence();
  const int qp0 = qp - gq;
  const int nq = a.batch - qp0 < 4 ? a.batch - qp0 : 4;  // live groups (the wave's first nq)
  constexpr int kPiecesPerRec = kWsStage * (int)sizeof(real) / 16;
  const int pieces = nq * kPiecesPerRec;
  typedef double d2 __attribute__((ext_vector_type(2)));
  const d2* src = reinterpret_cast<const d2*>(img);
  d2* dst = reinterpret_cast<d2*>(a.ws + ((size_t)k * a.batch + qp0) * kWsStage);
  // Records of stages >= kRecHotStages are written non-temporally (streamed past the caches):
  // between its write and its read in the forward sweep the chip moves ~(2k + 1) x 55 MB,
  // so only the last-written stages can still be cache-resident when they are read, and
  // write-allocating the rest only evicts them (3.43 -> 3.21 ms, same-box A/B).
  const int l = (int)(threadIdx.x & 63);
  if (k >= kRecHotStages) {
    for (int p = l; p < pieces; p += 16 * nq) __builtin_nontemporal_store(src[p], &dst[p]);
  } else {
    for (int p = l; p < pieces; p += 16 * nq) dst[p] = src[p];
  }
  lds_wave_fence();  // the next stage's writes into the image stay after these reads
}

// optional outputs of the backward sweep (hpipm-cpp getRiccati*): P_k, p_k, K_k, k_k
__device__ __forceinline__ void store_riccati_out(const ProblemArgsT<real>& a, int qp, int k, int lane,
                                                  const real (&F)[12], const real (&Kc)[12]) {
  const int N = a.N;
  const bool own = lane < kMaxDim, isv = lane == kVecLane;
  // (vector stores: the C-ABI requires 16-byte aligned base pointers, include/srbd_qp.h)
  if (a.P && own) store12(a.P + ((size_t)qp * (N + 1) + k) * 144 + (size_t)lane * 12, F);
  if (a.p && isv) store12(a.p + ((size_t)qp * (N + 1) + k) * 12, F);
  if (k < N) {
    if (a.K && own) store12(a.K + ((size_t)qp * N + k) * 144 + (size_t)lane * 12, Kc);
    if (a.k && isv) store12(a.k + ((size_t)qp * N + k) * 12, Kc);
  }
}

// ---- forward sweep (row-owned), shared by every unconstrained kernel ----
// u = K x + k, pi = P x + p, x+ = A x + B u + b (A, B, b row-owned from the QP data: the
// closed-loop Acl = A + B K is not formed in the backward sweep, which saves it 12 FMA blocks
// per stage and the record 156 reals).  The record and data rows of stage k+1 are loaded
// while stage k computes (the loads do not depend on x), so each stage pays one memory
// latency less.
// so (optional, the fused-residual kernel): an LDS copy of the solution, x [N+1][12], then
// u [N][12], then pi [N+1][12], for the residual pass that follows in the same kernel.
template <class Src>
__device__ __forceinline__ void fwd_sweep(const ProblemArgsT<real>& a, const Src& src, const int qp,
                                          const int lane, real* so = nullptr) {
  constexpr int nx = 12, nu = 12;
  const int N = a.N;
  const bool own = lane < kMaxDim;
  const int row = own ? lane : kMaxDim - 1;
  real xv = own ? a.x0[(size_t)qp * nx + lane] : real(0.0);
  bool bad = false;
  real* xo = a.x + (size_t)qp * (N + 1) * nx;
  real* uo = a.u + (size_t)qp * N * nu;
  real* po = a.pi + (size_t)qp * (N + 1) * nx;
  real Pr[12], Kr[12], Ar[12], pv, kv, bv;
  auto load_rows = [&](int k, real (&P_)[12], real (&K_)[12], real (&A__)[12], real& p_, real& k_,
                       real& b_) {
    const real* rec = src.rec(k);
    load_packed_sym(rec + kWsP, row, P_);
    p_ = rec[kWsp + row];
    if (k < N) {
      const real* kr = rec + kWsK + row * kWsRow;
      const real* Ab = src.A(k);
      sfor<0, 12>([&](auto j) {
        constexpr int J = decltype(j)::value;
        K_[J] = kr[J];
        A__[J] = Ab[J * 12 + row];  // column-major block: row `row` at stride 12
      });
      k_ = kr[12];
      b_ = src.b(k)[row];
    }
  };
  load_rows(0, Pr, Kr, Ar, pv, kv, bv);
#pragma unroll 1
  for (int k = 0; k <= N; ++k) {
    // this stage's B row (used last: its load overlaps P x, K x, A x), then stage k+1's rows
    real Br[12];
    if (k < N) {
      const real* Bb = src.B(k);
      sfor<0, 12>([&](auto j) { Br[decltype(j)::value] = Bb[decltype(j)::value * 12 + row]; });
    }
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
    if (own) {
      xo[(size_t)k * nx + lane] = xv;
      po[(size_t)k * nx + lane] = pp;
      if (so) {
        so[k * nx + lane] = xv;
        so[(2 * N + 1) * nx + k * nx + lane] = pp;
      }
    }
    if (k == N) break;
    real uu = kv, xn = bv;
    sfor<0, 12>([&](auto j) {
      constexpr int J = decltype(j)::value;
      uu = fmadd(Kr[J], bx[J], uu);
      xn = fmadd(Ar[J], bx[J], xn);
    });
    if (own) {
      uo[(size_t)k * nu + lane] = uu;
      if (so) so[(N + 1) * nx + k * nu + lane] = uu;
    }
    xn = dot_bcast(Br, uu, xn);  // + B u (u element-owned, broadcast inside the FMAs)
    bad |= own && (!(uu == uu) || !(xn == xn));
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

// ---- the solve of one QP by its 16-lane group, blocks and records through `src` ----
// SQRT: ric_alg = 1, the square-root recursion (riccati.h riccati_step_sqrt); the records
// and outputs are the same (P_k = F - Y'Y of the stage, which Lx factors).
template <bool SQRT, class Src>
__device__ __forceinline__ void solve_qp(const ProblemArgsT<real>& a, const Src& src, const int qp,
                                         const int lane, real* so = nullptr) {
  const int N = a.N;
  const bool isv = lane == kVecLane;
  const bool own = lane < kMaxDim;  // lane owns a block column
  const int col = own ? lane : kMaxDim - 1;
  const real reg = a.reg;

  // ---------------- terminal stage: P_N = Q_N, p_N = q_N ----------------
  real P[12];
  if (isv) {
    load12(src.q(N), P);
  } else {
    load12(src.Q(N) + col * 12, P);
  }
  store_rec_P(src.rec(N), lane, P);
  store_riccati_out(a, qp, N, lane, P, P);
  if constexpr (SQRT) sqrt_factor(P, lane);

  // ---------------- backward sweep ----------------
  real A_[12], B_[12];
#pragma unroll 1
  for (int k = N - 1; k >= 0; --k) {
    // A, B (VL: b) of stage k, column-owned
    if (isv) {
      load12(src.b(k), A_);
      sfor<0, 12>([&](auto i) { B_[decltype(i)::value] = real(0.0); });
    } else {
      load12(src.A(k) + col * 12, A_);
      load12(src.B(k) + col * 12, B_);
    }
    auto loadR = [&](real (&Rc)[12]) {
      if (isv) {
        sfor<0, 12>([&](auto i) { Rc[decltype(i)::value] = real(0.0); });
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
    tstamp(0);
    if constexpr (SQRT) {
      riccati_step_sqrt<1, false>(P, A_, B_, loadR, loadSQ, lane, reg, f);
    } else {
      riccati_step<1, false>(P, A_, B_, loadR, loadSQ, lane, reg, f);
    }
    if constexpr (std::is_same_v<Src, HbmSrc>) {
      src.store_stage(k, [&](real* r) { store_rec(r, lane, f.Kc, f.F); });
    } else {
      store_rec(src.rec(k), lane, f.Kc, f.F);
    }
    tstamp(11);
    store_riccati_out(a, qp, k, lane, f.F, f.Kc);
    sfor<0, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      P[I] = f.F[I];
    });
    if constexpr (SQRT) sqrt_factor(P, lane);
  }
  tstamp(12);
  fwd_sweep(a, src, qp, lane, so);
  tstamp(13);
}

// Large batches: 16 QPs per 256-thread workgroup, 2 workgroups per CU (the kernel needs
// 217-224 VGPRs; memory-bound with the compute overlapped).  fp64: each
// wave's stage records go out through its 12.6 KiB LDS image (HbmSrc::store_stage).
template <bool SQRT>
__global__ void __launch_bounds__(256, 2) riccati_unconstr_kernel(ProblemArgsT<real> a) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int qp = gid >> 4;
  if (qp >= a.batch) return;
  if constexpr (sizeof(real) == 8) {  // fp64 records are whole 16-byte pieces per QP
    __shared__ __attribute__((aligned(16))) real rec_img[16 * kWsStage];
    HbmSrc src{a, qp};
    src.gq = (threadIdx.x >> 4) & 3;
    src.img = rec_img + (threadIdx.x >> 6) * 4 * kWsStage;
    solve_qp<SQRT>(a, src, qp, threadIdx.x & (kGroup - 1));
  } else {
    solve_qp<SQRT>(a, HbmSrc{a, qp}, qp, threadIdx.x & (kGroup - 1));
  }
}

// Small batches: one QP per workgroup.  kLdsCopyThreads lanes (8 waves) copy the QP into the
// LDS image with 16-byte global->LDS DMA (one wave-instruction fills 1 KiB of the image; each
// lane gathers its own 16 bytes from the QP-major buffers), then lanes 0-15 solve.  One wave
// issuing the whole copy took ~40 us of the ~160 us single-QP solve (the DMA issue rate of a
// wave, scripts/dev/latency_breakdown.py); eight issue it in parallel.
constexpr int kRealsPerDma = 16 / (int)sizeof(real);
constexpr int kLdsCopyThreads = 512;

__device__ __forceinline__ const real* img_source(const ProblemArgsT<real>& a, int qp, int e) {
  const int N = a.N;
  const int k = e / kImgStage, o = e - k * kImgStage;
  const size_t s = (size_t)qp * N + k, s1 = (size_t)qp * (N + 1) + k;
  if (o >= kImgQ && o < kImgS) return a.Q + s1 * 144 + (o - kImgQ);
  if (o >= kImgq && o < kImgr) return a.q + s1 * 12 + (o - kImgq);
  if (k >= N) return nullptr;  // slot N holds Q_N and q_N only
  if (o < kImgB) return a.A + s * 144 + o;
  if (o < kImgb) return a.B + s * 144 + (o - kImgB);
  if (o < kImgQ) return a.b + s * 12 + (o - kImgb);
  if (o < kImgR) return a.S + s * 144 + (o - kImgS);
  if (o < kImgq) return a.R + s * 144 + (o - kImgR);
  return a.r + s * 12 + (o - kImgr);
}

// The QP's blocks into the LDS image by every thread of the workgroup (global->LDS DMA;
// the source may be device memory or mapped host memory), waited for and fenced.
// Image elements [e0, e1) (e0 even) issued by nthr threads (whole waves; t = 0..nthr-1 the
// thread's rank among them); not waited for.
__device__ __forceinline__ void lds_copy_range(const ProblemArgsT<real>& a, real* img, int qp, int e0, int e1,
                                               int t, int nthr) {
  const int wave_off = (t >> 6) * 64 * kRealsPerDma;  // this wave's 1 KiB of each round
  for (int c0 = e0; c0 < e1; c0 += nthr * kRealsPerDma) {
    const int e = c0 + t * kRealsPerDma;
    const real* g = e < e1 ? img_source(a, qp, e) : nullptr;
    if (g)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                       (__attribute__((address_space(3))) void*)(img + c0 + wave_off), 16,
                                       0, 0);
  }
}
__device__ __forceinline__ void lds_copy_qp(const ProblemArgsT<real>& a, real* img, int qp) {
  lds_copy_range(a, img, qp, 0, (a.N + 1) * kImgStage, threadIdx.x, kLdsCopyThreads);
  tstamp(14);  // (kernel entry is the first stamp of a launch: the copy into LDS ends here)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  tstamp(15);
}

template <bool SQRT>
__global__ void __launch_bounds__(kLdsCopyThreads, 1) riccati_unconstr_lds_kernel(ProblemArgsT<real> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  real* img = reinterpret_cast<real*>(lds_raw);
  const int qp = blockIdx.x;
  tstamp(16);
  lds_copy_qp(a, img, qp);
  if (threadIdx.x >= kGroup) return;
  solve_qp<SQRT>(a, LdsSrc{img}, qp, threadIdx.x);
}

size_t lds_image_bytes(int N) { return (size_t)(N + 1) * kImgStage * sizeof(real); }
// the fused-residual kernel's LDS: the image plus the solution copy x, u, pi
size_t lds_res_bytes(int N) { return lds_image_bytes(N) + (size_t)(3 * N + 2) * 12 * sizeof(real); }


// KKT residuals and objective of an unconstrained solution: HPIPM's
// d_ocp_qp_res_compute (hpipm_d_ocp_qp_res.h:57-67) for nc = 0, as the oracle's
// compute_residuals states it (oracle/ocp_qp_oracle.c):
//   res_stat = max( |R u + S x + r + B'pi_{k+1}| (k < N), |Q x + S'u + q + A'pi_{k+1} - pi_k| (k >= 1) )
//   res_eq   = max |A x + B u + b - x_{k+1}|,   res_ineq = res_comp = 0,
//   obj      = sum_k u'(R u / 2 + r + S x) (k < N) + x'(Q x / 2 + q) (k >= 1).
// Run only when the caller asks for res / obj / stat.  One 256-thread workgroup per QP,
// thread t on (stage t / 12 (+21 j), row t % 12): every row's dot products are
// independent, so a single QP (the reference's call pattern) costs a few memory latencies
// rather than a serial walk over its stages.  Any dims (padded problems are checked
// unpadded).
constexpr int kResThreads = 256;
constexpr int kResStages = kResThreads / 12;  // 21 stages per pass
constexpr int kResWavesMax = 8;                // (the fused single-QP kernel: 512 threads)

__device__ __forceinline__ void max_nan(real& m, real v) {
  v = v < real(0) ? -v : v;
  if (v > m || v != v) m = v;  // NaN propagates
}

// Where the residual pass finds a QP's blocks and its solution: the C-ABI buffers (QP-major
// or stage-major, any nx <= 12, nu <= 12), or (the fused single-QP kernel) the LDS image of
// riccati_unconstr_lds_kernel and its LDS copy of x, u, pi (12 x 12 stages).
struct ResGlobal {
  const ProblemArgsT<real>& a;
  int qp;
  __device__ const real* at(const real* base, int nstage, size_t blk, int k) const {
    return a.layout == 1 ? base + ((size_t)k * a.batch + qp) * blk : base + ((size_t)qp * nstage + k) * blk;
  }
  __device__ const real* A(int k) const { return at(a.A, a.N, (size_t)a.nx * a.nx, k); }
  __device__ const real* B(int k) const { return at(a.B, a.N, (size_t)a.nx * a.nu, k); }
  __device__ const real* b(int k) const { return at(a.b, a.N, a.nx, k); }
  __device__ const real* Q(int k) const { return at(a.Q, a.N + 1, (size_t)a.nx * a.nx, k); }
  __device__ const real* S(int k) const { return at(a.S, a.N, (size_t)a.nx * a.nu, k); }
  __device__ const real* R(int k) const { return at(a.R, a.N, (size_t)a.nu * a.nu, k); }
  __device__ const real* q(int k) const { return at(a.q, a.N + 1, a.nx, k); }
  __device__ const real* r(int k) const { return at(a.r, a.N, a.nu, k); }
  __device__ const real* x() const { return a.x + (size_t)qp * (a.N + 1) * a.nx; }
  __device__ const real* u() const { return a.u + (size_t)qp * a.N * a.nu; }
  __device__ const real* pi() const { return a.pi + (size_t)qp * (a.N + 1) * a.nx; }
};
struct ResLds : LdsSrc {
  const real* so;  // x [N+1][12], u [N][12], pi [N+1][12]
  int N;
  __device__ const real* x() const { return so; }
  __device__ const real* u() const { return so + (N + 1) * 12; }
  __device__ const real* pi() const { return so + (2 * N + 1) * 12; }
};

// The residual pass of one QP by the whole workgroup (every thread calls it: it ends with a
// workgroup reduction).  Threads >= kResStages * 12 only take part in the reduction, so a
// 512-thread workgroup sums the same partial results in the same order as a 256-thread one.
// (t: the thread's index in the workgroup, passed in so a caller can make it opaque; DIM > 0:
// nx = nu = DIM known at compile time, the same sums in the same order, unrolled)
template <class Acc, int DIM = 0>
__device__ __forceinline__ void unconstr_residuals_body(const ProblemArgsT<real>& a, const Acc& acc, int qp, int t) {
  const int N = a.N, nx = DIM ? DIM : a.nx, nu = DIM ? DIM : a.nu;
  if (a.stat) {  // the QP's stat table is cleared here (no separate memset), row 0 filled below
    real* tab = a.stat + (size_t)qp * a.stat_rows * kStatCols;
    for (int i = t; i < a.stat_rows * kStatCols; i += blockDim.x) tab[i] = real(0);
  }
  const real* x = acc.x();
  const real* u = acc.u();
  const real* pi = acc.pi();
  const int i = t % 12;
  real mg = real(0), mb = real(0), ob = real(0);
  for (int k = t / 12; t < kResStages * 12 && k <= N; k += kResStages) {
    const real* xk = x + (size_t)k * nx;
    if (k < N) {
      const real* uk = u + (size_t)k * nu;
      const real* xn = x + (size_t)(k + 1) * nx;
      const real* pn = pi + (size_t)(k + 1) * nx;
      const real* A = acc.A(k);
      const real* B = acc.B(k);
      if (i < nu) {  // column-major blocks: M[i][j] = M[j * rows + i]
        const real* S = acc.S(k);
        const real* R = acc.R(k);
        const real* r = acc.r(k);
        real ru = real(0), sx = real(0), bp = real(0);
        for (int j = 0; j < nu; ++j) ru += R[(size_t)j * nu + i] * uk[j];
        for (int j = 0; j < nx; ++j) sx += S[(size_t)j * nu + i] * xk[j];
        for (int j = 0; j < nx; ++j) bp += B[(size_t)i * nx + j] * pn[j];
        max_nan(mg, ru + sx + r[i] + bp);
        ob += uk[i] * (real(0.5) * ru + r[i] + sx);
      }
      if (i < nx) {
        const real* b = acc.b(k);
        real v = b[i] - xn[i];
        for (int j = 0; j < nx; ++j) v += A[(size_t)j * nx + i] * xk[j];
        for (int j = 0; j < nu; ++j) v += B[(size_t)j * nx + i] * uk[j];
        max_nan(mb, v);
      }
    }
    if (k > 0 && i < nx) {
      const real* Q = acc.Q(k);
      const real* q = acc.q(k);
      real qx = real(0), g = q[i] - pi[(size_t)k * nx + i];
      for (int j = 0; j < nx; ++j) qx += Q[(size_t)j * nx + i] * xk[j];
      g += qx;
      if (k < N) {
        const real* uk = u + (size_t)k * nu;
        const real* pn = pi + (size_t)(k + 1) * nx;
        const real* A = acc.A(k);
        const real* S = acc.S(k);
        for (int j = 0; j < nu; ++j) g += S[(size_t)i * nu + j] * uk[j];
        for (int j = 0; j < nx; ++j) g += A[(size_t)i * nx + j] * pn[j];
      }
      max_nan(mg, g);
      ob += xk[i] * (real(0.5) * qx + q[i]);
    }
  }
  // workgroup reduction: max (NaN-propagating) of mg, mb; sum of ob
  for (int m = 32; m >= 1; m >>= 1) {
    const real og = __shfl_xor(mg, m), obb = __shfl_xor(mb, m);
    if (og > mg || og != og) mg = og;
    if (obb > mb || obb != obb) mb = obb;
    ob += __shfl_xor(ob, m);
  }
  __shared__ real part[3][kResWavesMax];
  const int w = t / 64;
  if ((t & 63) == 0) {
    part[0][w] = mg;
    part[1][w] = mb;
    part[2][w] = ob;
  }
  __syncthreads();
  if (t == 0) {
    // (waves past the stage-parallel ones hold 0 and add nothing)
    mg = part[0][0], mb = part[1][0], ob = part[2][0];
    for (int j = 1; j < kResThreads / 64; ++j) {
      if (part[0][j] > mg || part[0][j] != part[0][j]) mg = part[0][j];
      if (part[1][j] > mb || part[1][j] != part[1][j]) mb = part[1][j];
      ob += part[2][j];
    }
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

__global__ void __launch_bounds__(kResThreads) unconstr_residuals_kernel(ProblemArgsT<real> a) {
  unconstr_residuals_body(a, ResGlobal{a, (int)blockIdx.x}, (int)blockIdx.x, (int)threadIdx.x);
}

// The reference's call pattern in one launch (one QP per workgroup, the C-ABI's small
// batches with res / obj / stat requested): the copy into LDS, the solve (records in the HBM
// workspace, so the image keeps Q, S, R for the residual pass; x, u, pi also into LDS), then
// the residual pass over the image by the whole workgroup -- the same arithmetic as
// riccati_unconstr_lds_kernel followed by unconstr_residuals_kernel, without the second
// launch and its re-read of the QP (which may live in mapped host memory: the C-ABI's
// host-buffer path hands its pinned staging buffer straight to this kernel).
template <bool SQRT>
__global__ void __launch_bounds__(kLdsCopyThreads, 1) riccati_unconstr_lds_res_kernel(ProblemArgsT<real> a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  real* img = reinterpret_cast<real*>(lds_raw);
  real* so = img + (a.N + 1) * kImgStage;
  const int qp = blockIdx.x;
  tstamp(16);
  lds_copy_qp(a, img, qp);
  LdsSrc src{img};
  src.grec = a.ws;
  src.batch = a.batch;
  src.qp = qp;
  if (threadIdx.x < kGroup) solve_qp<SQRT>(a, src, qp, threadIdx.x, so);
  __syncthreads();  // the solution copy is complete
  ResLds acc{};
  acc.img = img;
  acc.so = so;
  acc.N = a.N;
  unconstr_residuals_body(a, acc, qp, (int)threadIdx.x);
}

// The same residuals for large batches, on the solve's layout: one 16-lane group per QP
// (16 QPs per workgroup), lane j < 12 owning column j of every stage block (16-byte column
// loads, as the solve reads them), the QP's stages in order.  The column-shaped products
// (A'pi, B'pi, S'u) are DPP dot products; the row-shaped ones (A x + B u, R u + S x, Q x)
// are formed column by column and summed across the group through its 12 x 12 LDS block.
// The objective uses u'Sx = x'(S'u) and takes u'(Ru + Sx) from the row sums: the same
// quantities as the oracle's, summed in another order.  FULL: nx = nu = 12.
template <bool FULL>
__global__ void __launch_bounds__(256) unconstr_residuals_group_kernel(ProblemArgsT<real> a) {
  __shared__ __attribute__((aligned(16))) real tb_all[(256 / kGroup) * 144];
  const int qp = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 4);
  const int lane = threadIdx.x & (kGroup - 1);
  if (qp >= a.batch) return;
  real* const tb = tb_all + (threadIdx.x >> 4) * 144;
  const int N = a.N, nx = FULL ? 12 : a.nx, nu = FULL ? 12 : a.nu;
  if (a.stat) {  // the QP's stat table is cleared here, row 0 filled below
    real* tab = a.stat + (size_t)qp * a.stat_rows * kStatCols;
    for (int i = lane; i < a.stat_rows * kStatCols; i += kGroup) tab[i] = real(0);
  }
  const bool smaj = a.layout == 1;
  auto at = [&](const real* base, int nstage, size_t blk, int k) -> const real* {
    return smaj ? base + ((size_t)k * a.batch + qp) * blk : base + ((size_t)qp * nstage + k) * blk;
  };
  const size_t nxx = (size_t)nx * nx, nxu = (size_t)nx * nu, nuu = (size_t)nu * nu;
  const real* x = a.x + (size_t)qp * (N + 1) * nx;
  const real* u = a.u + (size_t)qp * N * nu;
  const real* pi = a.pi + (size_t)qp * (N + 1) * nx;
  const int li = lane < kMaxDim ? lane : 0;
  const bool xl = lane < nx, ul = lane < nu;
  // column j (= lane) of a rows x cols column-major block, zero past the block
  auto colv = [&](const real* blk, int rows, int cols, real (&v)[12]) {
    if constexpr (FULL) {
      load12(blk + li * 12, v);
    } else {
      load_col_pad(blk + (size_t)li * rows, rows, lane < cols, v);
    }
  };
  // lane i <- sum over columns j of T_j[i] (lane j holds T_j)
  auto row_sum = [&](const real (&T)[12]) -> real {
    lds_wave_fence();  // the previous sum's reads are done
    if (lane < kMaxDim) store12(tb + lane * 12, T);
    lds_wave_fence();
    real s = real(0);
    sfor<0, 12>([&](auto j) { s += tb[decltype(j)::value * 12 + li]; });
    return s;
  };
  real mg = real(0), mb = real(0), ob = real(0);
#pragma unroll 1
  for (int k = 0; k <= N; ++k) {
    const real xk = xl ? x[(size_t)k * nx + lane] : real(0);
    real T[12];
    real gx = real(0);  // x-row stationarity residual (k >= 1)
    if (k > 0) {
      real Qc[12];
      colv(at(a.Q, N + 1, nxx, k), nx, nx, Qc);
      sfor<0, 12>([&](auto i) { T[decltype(i)::value] = Qc[decltype(i)::value] * xk; });
      const real qx = row_sum(T);  // (Q x)_i
      const real qk = xl ? at(a.q, N + 1, nx, k)[lane] : real(0);
      gx = qx + qk - (xl ? pi[(size_t)k * nx + lane] : real(0));
      if (xl) ob += xk * (real(0.5) * qx + qk);
    }
    if (k < N) {
      const real uk = ul ? u[(size_t)k * nu + lane] : real(0);
      const real xn = xl ? x[(size_t)(k + 1) * nx + lane] : real(0);
      const real pin = xl ? pi[(size_t)(k + 1) * nx + lane] : real(0);
      real Ac[12], Bc[12];
      colv(at(a.A, N, nxx, k), nx, nx, Ac);
      colv(at(a.B, N, nxu, k), nx, nu, Bc);
      const real atp = dot_bcast(Ac, pin, real(0));  // (A'pi_{k+1})_j
      const real btp = dot_bcast(Bc, pin, real(0));  // (B'pi_{k+1})_j
      sfor<0, 12>([&](auto i) {
        constexpr int I = decltype(i)::value;
        T[I] = fmadd(Ac[I], xk, Bc[I] * uk);
      });
      const real axbu = row_sum(T);  // (A x + B u)_i
      if (xl) max_nan(mb, axbu + at(a.b, N, nx, k)[lane] - xn);
      real Sc[12], Rc[12];
      colv(at(a.S, N, nxu, k), nu, nx, Sc);
      colv(at(a.R, N, nuu, k), nu, nu, Rc);
      const real stu = dot_bcast(Sc, uk, real(0));  // (S'u)_j
      sfor<0, 12>([&](auto i) {
        constexpr int I = decltype(i)::value;
        T[I] = fmadd(Rc[I], uk, Sc[I] * xk);
      });
      const real rusx = row_sum(T);  // (R u + S x)_i
      const real rk = ul ? at(a.r, N, nu, k)[lane] : real(0);
      if (ul) {
        max_nan(mg, rusx + rk + btp);
        ob += uk * (real(0.5) * rusx + rk);
      }
      if (xl) ob += real(0.5) * xk * stu;
      gx += stu + atp;
    }
    if (k > 0 && xl) max_nan(mg, gx);
  }
  // group reduction: NaN-propagating max of mg, mb; sum of ob (lanes >= 12 hold 0)
  sfor<0, 4>([&](auto s) {
    constexpr int M = 8 >> decltype(s)::value;
    const real og = __shfl_xor(mg, M, kGroup), obb = __shfl_xor(mb, M, kGroup);
    if (og > mg || og != og) mg = og;
    if (obb > mb || obb != obb) mb = obb;
    ob += __shfl_xor(ob, M, kGroup);
  });
  if (lane == 0) {
    if (a.res) {
      a.res[(size_t)qp * 4 + 0] = mg;
      a.res[(size_t)qp * 4 + 1] = mb;
      a.res[(size_t)qp * 4 + 2] = real(0);
      a.res[(size_t)qp * 4 + 3] = real(0);
    }
    if (a.obj) a.obj[qp] = ob;
    if (a.stat) {
      real* row = a.stat + (size_t)qp * a.stat_rows * kStatCols;
      row[6] = mg;
      row[7] = mb;
      row[10] = ob;
    }
    if (a.status && (mg != mg || mb != mb)) a.status[qp] = 3;  // NaNDetected
  }
}

// small batches (the reference's one QP per call): the stage-parallel kernel above, whose
// latency is a few memory round trips; large ones: the group kernel (one pass over the data)
constexpr int kResGroupMin = 256;

hipError_t launch_residuals(const ProblemArgsT<real>& a, hipStream_t stream) {
  if (a.batch <= 0) return hipSuccess;
  if (a.batch <= kResGroupMin) {
    hipLaunchKernelGGL(unconstr_residuals_kernel, dim3((unsigned)a.batch), dim3(kResThreads), 0, stream, a);
    return hipGetLastError();
  }
  const unsigned blocks = (unsigned)(((long long)a.batch * kGroup + 255) / 256);
  if (a.nx == 12 && a.nu == 12) {
    hipLaunchKernelGGL(unconstr_residuals_group_kernel<true>, dim3(blocks), dim3(256), 0, stream, a);
  } else {
    hipLaunchKernelGGL(unconstr_residuals_group_kernel<false>, dim3(blocks), dim3(256), 0, stream, a);
  }
  return hipGetLastError();
}

// QP-major batches of at most this many QPs (one per CU) take the LDS kernel when the
// image fits a workgroup's LDS (fp64: N <= 26, fp32: N <= 53)
constexpr int kLdsBatchMax = 256;
constexpr size_t kLdsBytesMax = 160 * 1024;
constexpr size_t kLdsResStatic = 1024;  // >= sizeof(part) of unconstr_residuals_body

bool use_lds_kernel(const ProblemArgsT<real>& a) {
  return a.layout == 0 && a.batch <= kLdsBatchMax && lds_image_bytes(a.N) <= kLdsBytesMax;
}

// The fp64 classical solve of small batches runs on the matrix-core latency kernel
// (riccati_latency_impl.h).
#if SRBD_WITH_LATENCY
#include "riccati_latency_impl.h"
bool lat_eligible(const ProblemArgsT<real>& a) { return use_lds_kernel(a) && lat_fits(a.N); }
#else
bool lat_eligible(const ProblemArgsT<real>&) { return false; }
#endif

// the single-QP kernel computes the residuals itself (one launch, one read of the data)
bool fused_residuals(const ProblemArgsT<real>& a) {
  return a.fuse_res && (a.res || a.obj || a.stat) && a.nx == 12 && a.nu == 12 && use_lds_kernel(a) &&
         lds_res_bytes(a.N) + kLdsResStatic <= kLdsBytesMax;  // (+ the reduction's static LDS)
}
// the launch reads each QP's data once, into LDS, and nothing else reads it
bool reads_once(const ProblemArgsT<real>& a) {
  return a.nx == 12 && a.nu == 12 && use_lds_kernel(a) &&
         (fused_residuals(a) || !(a.res || a.obj || a.stat));
}

template <bool SQRT>
static hipError_t launch_alg(const ProblemArgsT<real>& a, hipStream_t stream) {
#if SRBD_WITH_LATENCY
  if (!SQRT && lat_eligible(a)) {
    if (fused_residuals(a)) {
      hipLaunchKernelGGL(riccati_latency_kernel<true>, dim3((unsigned)a.batch), dim3(kLatThreads),
                         lat_lds_bytes(a.N), stream, a);
    } else {
      hipLaunchKernelGGL(riccati_latency_kernel<false>, dim3((unsigned)a.batch), dim3(kLatThreads),
                         lat_lds_bytes(a.N), stream, a);
    }
    return hipGetLastError();
  }
#endif
  if (fused_residuals(a)) {
    hipLaunchKernelGGL(riccati_unconstr_lds_res_kernel<SQRT>, dim3((unsigned)a.batch), dim3(kLdsCopyThreads),
                       lds_res_bytes(a.N), stream, a);
    return hipGetLastError();
  }
  if (use_lds_kernel(a)) {
    // (the > 64 KiB dynamic-LDS attribute is set on the handle's device by srbd_qp_create:
    // prepare_device below)
    const size_t bytes = lds_image_bytes(a.N);
    hipLaunchKernelGGL(riccati_unconstr_lds_kernel<SQRT>, dim3((unsigned)a.batch), dim3(kLdsCopyThreads), bytes,
                       stream, a);
    return hipGetLastError();
  }
  const int threads = 256;
  const long long lanes = (long long)a.batch * kGroup;
  const int blocks = (int)((lanes + threads - 1) / threads);
  hipLaunchKernelGGL(riccati_unconstr_kernel<SQRT>, dim3(blocks), dim3(threads), 0, stream, a);
  return hipGetLastError();
}

#if SRBD_WITH_LATENCY
// the launch of `a` is one latency-kernel workgroup that reads its QP once (the resident
// server can take it: one QP, classical Riccati, residuals fused or not asked for)
bool server_ok(const ProblemArgsT<real>& a) {
  return a.batch == 1 && !a.ric_alg && lat_eligible(a) && reads_once(a);
}
hipError_t launch_server(const ProblemArgsT<real>& a, LatMailbox* mb, int epoch, int last_done,
                         long long idle_ticks, long long life_ticks, hipStream_t stream) {
  if (!server_ok(a)) return hipErrorInvalidValue;
  if (fused_residuals(a))
    hipLaunchKernelGGL(riccati_latency_server_kernel<true>, dim3(1), dim3(kLatThreads), lat_lds_bytes(a.N), stream,
                       a, mb, epoch, last_done, idle_ticks, life_ticks);
  else
    hipLaunchKernelGGL(riccati_latency_server_kernel<false>, dim3(1), dim3(kLatThreads), lat_lds_bytes(a.N), stream,
                       a, mb, epoch, last_done, idle_ticks, life_ticks);
  return hipGetLastError();
}
#endif

// Per-device launch attributes, set on the current device (srbd_qp_create calls this
// after selecting the handle's device; hipFuncSetAttribute is per device, and every
// handle sets it, so concurrent handles on any device need no shared flag).
hipError_t prepare_device() {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&riccati_unconstr_lds_kernel<false>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytesMax);
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&riccati_unconstr_lds_kernel<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytesMax);
  // (the fused kernel also has the residual reduction's static LDS: kLdsResStatic at most)
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&riccati_unconstr_lds_res_kernel<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytesMax - kLdsResStatic));
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&riccati_unconstr_lds_res_kernel<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytesMax - kLdsResStatic));
#if SRBD_WITH_LATENCY
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&riccati_latency_kernel<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytesMax - kLdsResStatic));
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&riccati_latency_kernel<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytesMax - kLdsResStatic));
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&riccati_latency_server_kernel<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytesMax - kLdsResStatic));
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&riccati_latency_server_kernel<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsBytesMax - kLdsResStatic));
#endif
  return e;
}

hipError_t launch(const ProblemArgsT<real>& a, hipStream_t stream) {
  if (a.batch <= 0) return hipSuccess;
  // 12 x 12 stages only: smaller problems arrive embedded by pad.hip
  if (a.nx != 12 || a.nu != 12) return hipErrorInvalidValue;
  return a.ric_alg ? launch_alg<true>(a, stream) : launch_alg<false>(a, stream);
}

}  // namespace SRBD_NS
}  // namespace srbd
