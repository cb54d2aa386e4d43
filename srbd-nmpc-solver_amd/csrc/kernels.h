// kernels.h -- launch interface between the C-ABI (srbd_qp_capi.hip) and the
// HIP kernels.  Internal; not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace srbd {

// Forward-pass record of one stage, written by the backward sweep and read
// back (row-owned) by the forward sweep.  [K | k] is 12 rows of 13: row i =
// (K[i][0..11], k[i]), so the backward sweep's column owners (lane j) and its
// vector lane (k: "column 12") store element (i, j) at one common stride per
// row i, and lane i of the forward pass loads row i and its affine term as 13
// contiguous values.  The symmetric P is packed (lower triangle by columns, 78
// values: qp_group.h packed_col), followed by p.  The forward sweep takes
// x+ = A x + B u + b from the QP data itself (no closed-loop Acl in the record).
constexpr int kWsRow = 13;   // [K | k] row length
constexpr int kWsK = 0;      // [K | k]     [12][13]
constexpr int kWsP = 156;    // P   packed lower triangle, 78
constexpr int kWsp = 234;    // p   [12]
constexpr int kWsStage = 246;  // doubles per stage record (16-byte multiple)

// Arguments of every launch; T = double (srbd_qp_solve_f64) or float
// (srbd_qp_solve_f32).  Workspace offsets below count elements of T.
template <typename T>
struct ProblemArgsT {
  int batch, N, nx, nu, ng;
  int layout;  // 0: QP-major inputs, 1: stage-major (srbd_qp_dims.layout)
  // unconstrained solves: the single-QP (LDS) kernel may compute res / obj / stat itself
  // (set by the C-ABI when the problem is not embedded; unconstr_fused_residuals says
  // whether the launch did, so the separate residual pass is skipped)
  int fuse_res;
  // QP data (device)
  const T *A, *B, *b, *Q, *S, *R, *q, *r, *x0;
  const T *lbu, *ubu, *lbu_mask, *ubu_mask;
  const T *lbx, *ubx, *lbx_mask, *ubx_mask;
  const T *C, *D, *lg, *ug, *lg_mask, *ug_mask;
  // solution (device)
  T *x, *u, *pi, *P, *p, *K, *k;
  int *status, *iter;
  T *res, *obj;
  T* stat;  // [batch][iter_max+2][kStatCols] or null
  // workspace
  T* ws;
  size_t ws_qp;  // elements per QP
  T reg;
  // IPM settings (hpipm-cpp OcpQpIpmSolverSettings semantics)
  int iter_max, pred_corr, split_step, warm_start;
  int ric_alg;    // 0: classical Riccati, else the square-root recursion (riccati.h)
  int stat_rows;  // rows per QP of `stat` (the caller's iter_max + 2)
  // iterative refinement of the corrector step (HPIPM itref_corr_max; the C-ABI derives it
  // from settings.mode: Balance 2, Robust 4, else 0).
  int itref_corr_max;
  // HPIPM's lq_fact (square-root Riccati only; the C-ABI derives it from settings.mode:
  // Balance 1, Robust 2, else 0): 2 = every stage factorization by LQ, 1 = Cholesky until a
  // predictor step's linear residual exceeds 1e-5, LQ from then on (ipm_box_impl.h).
  // lq_redo: internal, set on the launch that redoes an iteration's RB -> F1 by LQ.
  int lq_fact, lq_redo;
  // warm_start 2 only (internal: the fp64 continuation of srbd_qp_settings.f64_rescue):
  // per QP and stage the barrier state [kStLam block 96][nch chunks x 48], see ipm_box.hip
  const T* warm_bars;
  // internal (srbd_qp_solve_host_cb_f64, zero-copy single-QP path): mapped host flags [batch]
  // the latency kernel sets to 1 once P, p, K, k of that QP are in host memory (system
  // scope), while its forward sweep still runs; null = those outputs are written at the end
  int* factors_ready;
  // internal (srbd_qp_settings.f32_iters): end the IPM launch loop after the last corrector
  // step without the sweep that would apply it; the step is handed to the fp64 continuation
  int skip_last_rb;
  T alpha_min, mu0, tol_stat, tol_eq, tol_ineq, tol_comp;
  // Live-QP control of the IPM launch sequence, decided on the device (the handle's; ctl
  // NULL = off).  The host enqueues every launch of a solve up front and never waits.  After
  // the RB sweep of launch iteration it, ctl[2 it] counts the workgroups with a QP still
  // running and ctl[2 it + 1] the workgroups done; the last one sets ctl[kCtlDone] when no
  // QP is left, and every later sweep of the solve returns at its first instruction.  The
  // compaction kernels (ipm_box_impl.h) switch the sweeps to the active-QP list once the
  // live workgroups are at most 3/4 of the grid the list last covered.
  int* ctl;
  int ctl_cap;    // ctl_cap: iterations the counter arrays hold
  int launch_it;  // set per launch
  // Active-QP list of the IPM sweeps (the handle's; capacity + 1 ints, the count last).
  // qp_list set for a launch and ctl[kCtlListOn] set: QP group g of the grid works on QP
  // qp_list[g] if g < count.
  int* qp_buf;
  const int* qp_list;
  // internal (the latency IPM, ric_alg 1 with lq_fact 1): device word the kernel sets to 1 when a
  // QP's predictor check asks for the LQ factorization (HPIPM's switch), which only the batched
  // kernels have: the C-ABI then solves the batch there (srbd_qp_capi.hip solve_impl).  (Last:
  // the other fields keep their kernel-argument offsets.)
  int* lat_lq_flag;
};
// iterations of the live-QP counter arrays (iter_max >= this runs without the control)
constexpr int kCtlCap = 257;
// control words after the per-iteration counters: every later sweep returns at once
// (done), the sweeps read the active-QP list (list on), the compaction kernel of this
// iteration rebuilds the list (rebuild), the workgroups the current grid covers (cur)
constexpr int kCtlDone = 2 * kCtlCap, kCtlListOn = kCtlDone + 1, kCtlRebuild = kCtlDone + 2,
              kCtlCur = kCtlDone + 3, kCtlInts = kCtlDone + 4;
using ProblemArgs = ProblemArgsT<double>;

constexpr int kStatCols = 18;  // HPIPM ws->stat row width

// IPM per-stage workspace layout (doubles), see ipm_box.hip.  Two factor
// records per stage (ping-pong by iteration parity: the iteration that exits
// still reports the previous iteration's Riccati factors, like HPIPM's
// getters), then the iterate's barrier state.
// The forward sweeps step x+ = A x + B u + b~ with the QP's own A, B (open loop), so the
// record holds no closed-loop Acl = A + B K.
constexpr int kRecL = 0;     // L packed lower triangle (78)
constexpr int kRecK = 78;    // K [12][12], column j contiguous
constexpr int kRecP = 222;   // P packed lower triangle (78)
constexpr int kRecRs = 300;  // 1 / diag(L)
constexpr int kRecKv = 312;  // k
constexpr int kRecPv = 324;  // p
constexpr int kRecPb = 336;  // P_{k+1} b~_k (classical Riccati: B2's right-hand side, from RB)
constexpr int kRecSize = 348;
constexpr int kStLam = 2 * kRecSize;  // 8 x 12: lam_l,u / lam_u,u / t_l,u / t_u,u / same for x
constexpr int kStRes = kStLam + 96;   // 3 x 12: res_g,u / res_g,x / res_b
constexpr int kStStep = kStRes + 36;  // 3 x 12: du / dx / dpi
constexpr int kStDlt = kStStep + 36;  // 8 x 12: dt_l,u dt_u,u dlam_l,u dlam_u,u (u), same (x)
constexpr int kIpmStage = kStDlt + 96;
static_assert(kIpmStage % 2 == 0, "16-byte aligned stages");
// general constraints (ng > 0): per stage and 12-row chunk, appended after
// kIpmStage: bars lam_l / lam_u / t_l / t_u [4][12], steps [4][12], row values
// C x + D u [12], 4 pad
constexpr int kGenChunk = 112;
// general rows, per stage after the chunks: the corrector's u-gradient D'gamma in
// parts (C = NULL kernels): D'gamma_pred [12] (RB), D'e [12] with e = d gamma / d(sigma mu)
// (RB), D'z [12] with z the predictor-product term of gamma_corr (F1)
constexpr int kGenVec = 36;

size_t ws_doubles_ipm(int N, int ng);  // elements per QP (either precision)
// The one-launch latency IPM (ipm_latency.hip): fp64, both Riccati forms, HPIPM's refinement, up
// to max_batch QPs (one workgroup each).  ipm_latency_ok says whether `a` runs there;
// launch_ipm_box_batched always takes the batched kernels.
constexpr int kIpmLatencyMaxBatch = 512;
int ipm_latency_max_batch();
bool ipm_latency_ok(const ProblemArgsT<double>& a, int max_batch);
hipError_t launch_ipm_latency(const ProblemArgsT<double>& a, hipStream_t stream);
hipError_t prepare_ipm_latency_device();  // srbd_qp_create, on the handle's device
template <typename T>
hipError_t launch_ipm_box(const ProblemArgsT<T>& a, hipStream_t stream);
hipError_t launch_ipm_box_batched(const ProblemArgsT<double>& a, hipStream_t stream);

// Workspace doubles per QP needed by the unconstrained solve.
size_t ws_doubles_unconstr(int N);

template <typename T>
hipError_t launch_riccati_unconstr(const ProblemArgsT<T>& a, hipStream_t stream);
// per-device launch attributes of the unconstrained kernels, on the current device
// (srbd_qp_create, after selecting the handle's device)
hipError_t prepare_riccati_device();
// KKT residual norms / objective of an unconstrained solution into a.res / a.obj
template <typename T>
hipError_t launch_unconstr_residuals(const ProblemArgsT<T>& a, hipStream_t stream);
// true when launch_riccati_unconstr(a) computes res / obj / stat in its own kernel
template <typename T>
bool unconstr_fused_residuals(const ProblemArgsT<T>& a);
// true when launch_riccati_unconstr(a) reads each QP's data exactly once, in one kernel
// (the single-QP kernel's copy into LDS): the data may then live in mapped host memory
template <typename T>
bool unconstr_reads_once(const ProblemArgsT<T>& a);

// The one-QP host call's resident server (riccati_latency_impl.h): the mailbox lives in
// mapped, coherent host memory; the host writes seq / quit, the kernel done / exited.
struct alignas(8) LatMailbox {
  int seq;     // host: number of the request posted last
  int flags;   // host: kLatQuit (leave now), kLatArm (this request writes the early factors and
               // sets factors_ready, the launch's fixed flags pointer); seq and flags are one
               // 8-byte word the server polls, a post writes both at once
  int done;    // device: number of the request finished last
  int exited;  // device: epoch of the server launch that has left
};
constexpr int kLatQuit = 1, kLatArm = 2;
// the latency IPM's status for a QP whose lq_fact 1 check asked for the LQ factorization: the
// C-ABI solves it again on the batched kernels (never returned to a caller)
constexpr int kLatNeedsLq = 4;
// true when launch_riccati_unconstr(a) would be one latency-kernel workgroup reading its QP
// once (batch 1, classical Riccati, N <= 20): the server can take the call instead
bool latency_server_ok(const ProblemArgsT<double>& a);
// the server on `stream` (dedicated: it stays until quit, idle_ticks of wall clock with no
// request, or the first answer after life_ticks since its launch); the first mailbox seq that
// differs from last_done is served
hipError_t launch_latency_server(const ProblemArgsT<double>& a, LatMailbox* mb, int epoch, int last_done,
                                 long long idle_ticks, long long life_ticks, hipStream_t stream);

// nx < 12 or nu < 12: embed the problem in 12 x 12 stages (pad.hip).  pad_elems
// is the pad buffer size (elements of T); pad_problem fills it from `a` and
// returns the padded arguments in `o` (solution pointers into the buffer);
// unpad_solution copies the solution back into `a`'s buffers.
size_t pad_elems(int batch, int N, int ng);
template <typename T>
hipError_t pad_problem(const ProblemArgsT<T>& a, T* buf, ProblemArgsT<T>& o, hipStream_t s);
template <typename T>
hipError_t unpad_solution(const ProblemArgsT<T>& a, const ProblemArgsT<T>& o, hipStream_t s);

}  // namespace srbd
#include "../../include/srbd_qp.h"
namespace srbd {
hipError_t launch_srbd_linesearch(const srbd_model_params& p, const srbd_linesearch_params& ls,
                                  int batch, int N, double* xs, double* us, const double* dx,
                                  const double* du, double* alpha, double* merit, int* converged,
                                  hipStream_t stream, const int* done = nullptr);
hipError_t launch_nmpc_prep(int batch, int N, int it, const double* xs, const double* x0,
                            double* dx0, int* done, int* sqp_iter, int* converged,
                            hipStream_t stream);
hipError_t launch_nmpc_after(int batch, int it, const int* conv, int* done, int* sqp_iter,
                             int* converged, int* active, hipStream_t stream);
hipError_t launch_srbd_linearize(const srbd_model_params& p, int batch, int N, int mode,
                                 const double* xs, const double* us,
                                 const srbd_qp_data_f64& out, hipStream_t stream);

// rescue.hip (srbd_qp_settings.f64_rescue / f32_iters): list the QPs with status >=
// min_status in batch order, widen / narrow QP-major rows of `elems` values between fp32 and fp64
hipError_t launch_select_unsolved(const int* status, int batch, int min_status, int* idx, int* count,
                                  hipStream_t s);
hipError_t launch_gather_widen(const float* src, double* dst, const int* idx, int rows, size_t elems,
                               hipStream_t s);
hipError_t launch_scatter_narrow(const double* src, float* dst, const int* idx, int rows, size_t elems,
                                 hipStream_t s);
hipError_t launch_scatter_int(const int* src, int* dst, const int* idx, int rows, hipStream_t s);
hipError_t launch_gather_rows(const double* src, double* dst, const int* idx, int rows, size_t elems,
                              hipStream_t s);
hipError_t launch_scatter_rows(const double* src, double* dst, const int* idx, int rows, size_t elems,
                               hipStream_t s);
hipError_t launch_narrow(const double* src, float* dst, size_t n, hipStream_t s);
hipError_t launch_widen(const float* src, double* dst, size_t n, hipStream_t s);
// ipm_box.hip: the barrier state of the fp32 IPM workspace rows idx[0..rows) (idx NULL: rows
// 0..rows), widened into the warm_bars layout of ProblemArgsT (rows x (N+1) x (96 + nch*48))
// ipm_box.hip (f32_iters): the fp32 pass's whole iterate, widened, with the step it computed
// last applied (QPs still running, fp32 status < 0): x, u, pi into the fp64 outputs, the barrier
// state into the warm_bars layout
hipError_t launch_gather_warm_apply(const float* ws32, size_t ws_qp, int N, int ng, int batch,
                                    const float* x32, const float* u32, const float* pi32, double* x,
                                    double* u, double* pi, double* bars, hipStream_t s);
hipError_t launch_gather_warm_bars(const float* ws32, size_t ws_qp, int N, int ng, const int* idx,
                                   int rows, double* dst, hipStream_t s);

}  // namespace srbd
