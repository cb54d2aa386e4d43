/*
 * srbd_qp.h -- C-ABI of the MI355X-native batched OCP-QP solver (libsrbd_qp.so).
 *
 * This is the drop-in boundary for the reference's hot path: everything
 * hpipm::OcpQpIpmSolver::solve() does below the Eigen marshalling
 * (hpipm-cpp/src/ocp_qp_ipm_solver.cpp:181-414) -- d_ocp_qp_set_all (:283),
 * d_ocp_qp_ipm_solve (:334, decl hpipm_d_ocp_qp_ipm.h:238), the solution and
 * Riccati getters (:337-346) and the stage-0 rebuild (:347-373) -- batched
 * over thousands of independent QPs and run by hand-written HIP kernels for
 * gfx950.  Plain C types only; no exceptions cross this boundary.
 *
 * Entry point -> reference interface it replaces:
 *   srbd_qp_create       OcpQpIpmSolver(qp, settings) ctor + resize()
 *                        (ocp_qp_ipm_solver.cpp:60-68, :120-178): dims check,
 *                        workspace sizing (d_ocp_qp_ipm_ws_create).
 *   srbd_qp_solve_f64    OcpQpIpmSolver::solve (ocp_qp_ipm_solver.cpp:181-414)
 *                        on a batch of device-resident QPs, asynchronous.
 *   srbd_qp_solve_host_f64  the same from host buffers, synchronous (what the
 *                        hpipm-cpp shim calls for one QP or a small batch).
 *   srbd_qp_solve_f32 / _host_f32  the fp32 twins (HPIPM's s_ocp_qp_ipm_solve,
 *                        hpipm_s_ocp_qp_ipm.h:238).
 *   srbd_qp_destroy      ~OcpQpIpmSolver (d_ocp_qp_*_wrapper frees).
 *   srbd_qp_status_string  hpipm::to_string(HpipmStatus) (:19-33).
 * The steps either side of the solve in the reference's SQP iteration, batched:
 *   srbd_qp_srbd_linearize_f64   NMPCSolver::prepareQpStructures (NMPC_solver.cpp:276-314)
 *   srbd_qp_srbd_linesearch_f64  NMPCSolver::linearSearch (NMPC_solver.cpp:149-274)
 *   srbd_qp_srbd_nmpc_f64        the SQP loop of NMPCSolver::controlLoop
 *                                (NMPC_solver.cpp:362-372) around all three.
 *
 * ------------------------------------------------------------------------
 * Problem (per QP, stages k = 0..N), identical to hpipm::OcpQp
 * (hpipm-cpp/include/hpipm-cpp/ocp_qp.hpp:15-177):
 *   min  sum_k 1/2 x'Q x + u'S x + 1/2 u'R u + q'x + r'u
 *   s.t. x[k+1] = A x[k] + B u[k] + b,  x[0] = x0,
 *        lbu <= u <= ubu, lbx <= x <= ubx (k >= 1), lg <= C x + D u <= ug.
 * x0 is embedded like hpipm-cpp does it (nx[0] = nbx[0] = 0,
 * ocp_qp_ipm_solver.cpp:128-130): box-x bounds and C at stage 0 are ignored.
 *
 * Memory layout (every pointer may be host or device memory as the entry
 * point says; 16-byte aligned base pointers are required for the fast path):
 *   batch-major, then stage-major, then one dense block per stage.  Matrix
 *   blocks are column-major (Eigen's default, what d_ocp_qp_set_all reads):
 *     A [batch][N  ][nx*nx]   B [batch][N][nx*nu]   b [batch][N][nx]
 *     Q [batch][N+1][nx*nx]   S [batch][N][nu*nx]   R [batch][N][nu*nu]
 *     q [batch][N+1][nx]      r [batch][N][nu]      x0 [batch][nx]
 *   Box constraints are dense per variable: one bound per variable plus an
 *   optional 0/1 mask per bound (a NULL mask means "all bounds active"; a
 *   masked bound is absent, exactly like hpipm's d_ocp_qp_set_l*_mask).  The
 *   reference's index form (idxbu/idxbx) maps onto this by setting mask 0 for
 *   variables not in the index list (the hpipm-cpp shim does this).
 *     lbu, ubu, lbu_mask, ubu_mask [batch][N][nu]        (NULL lbu: no box)
 *     lbx, ubx, lbx_mask, ubx_mask [batch][N+1][nx]      (NULL lbx: no box)
 *   General constraints (ng rows per stage, pad with masked rows):
 *     C [batch][N+1][ng*nx]  D [batch][N][ng*nu]  lg, ug, lg_mask, ug_mask [batch][N+1][ng]
 *   C = NULL means C = 0 (rows on u only, e.g. the friction cone) and selects
 *   the kernels without the C products; D = NULL means D = 0.
 * Outputs:
 *     x [batch][N+1][nx]  u [batch][N][nu]  pi [batch][N+1][nx]   (required)
 *     P [batch][N+1][nx*nx]  p [batch][N+1][nx]  K [batch][N][nu*nx]  k [batch][N][nu]
 *     status [batch] (HpipmStatus codes)  iter [batch]  res [batch][4]  obj [batch]
 *     stat [batch][iter_max+2][18]
 *   Conventions (ocp_qp_ipm_solver.cpp:337-373, test/ocp_qp_ipm_solver.cpp:60-109):
 *     x[0] = x0; pi[k] is the multiplier of x[k] = A x[k-1] + ... (hpipm pi[k-1]),
 *     pi[k] = P[k] x[k] + p[k]; u[k] = K[k] x[k] + k[k]; stage 0 as rebuilt.
 *
 * Dimensions: 1 <= nx, nu <= 12, 1 <= N <= 1024, 0 <= ng <= 64.  nx = nu = 12
 * (the SRBD model) takes the fast path; smaller problems are zero-padded
 * inside the kernel (exact: padded states stay 0, padded inputs get R = 1).
 */
#ifndef SRBD_QP_H_
#define SRBD_QP_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRBD_QP_ABI_VERSION 12
#define SRBD_QP_MAX_NX 12
#define SRBD_QP_MAX_NU 12
#define SRBD_QP_MAX_NG 64

/* error codes (returned by every entry point) */
enum {
  SRBD_QP_OK = 0,
  SRBD_QP_EINVAL = -1,      /* NULL / inconsistent argument                 */
  SRBD_QP_EDIM = -2,        /* dimensions outside the supported range        */
  SRBD_QP_ENOMEM = -3,      /* device allocation failed                      */
  SRBD_QP_EDEVICE = -4,     /* HIP runtime error / no GPU                     */
  SRBD_QP_ECAPACITY = -5,   /* batch larger than the handle's capacity        */
  SRBD_QP_ESETTINGS = -6    /* settings rejected (checkSettings rules)        */
};

/* per-QP solver status, same codes as hpipm::HpipmStatus
 * (hpipm-cpp/include/hpipm-cpp/ocp_qp_ipm_solver.hpp:24-30)                */
enum {
  SRBD_QP_SUCCESS = 0,
  SRBD_QP_MAX_ITER = 1,
  SRBD_QP_MIN_STEP = 2,
  SRBD_QP_NAN_SOL = 3,
  SRBD_QP_UNKNOWN_FAILURE = 4
};

/* hpipm::HpipmMode (ocp_qp_ipm_solver_settings.hpp:10-15) */
enum { SRBD_QP_MODE_SPEED_ABS = 0, SRBD_QP_MODE_SPEED = 1, SRBD_QP_MODE_BALANCE = 2,
       SRBD_QP_MODE_ROBUST = 3 };

typedef struct srbd_qp_dims {
  int N;          /* horizon                                                */
  int nx, nu;     /* uniform state / input dimensions                        */
  int ng;         /* general constraints per stage (0 = none)                */
  int has_box_u;  /* 1 if lbu/ubu will be passed                             */
  int has_box_x;  /* 1 if lbx/ubx will be passed                             */
  int layout;     /* SRBD_QP_LAYOUT_QP_MAJOR (0, default) or _STAGE_MAJOR (1) */
} srbd_qp_dims;

/* Input layouts.  QP-major: every array [batch][stage][block] (Eigen order,
 * what the hpipm-cpp shim packs).  Stage-major: [stage][batch][block], so the
 * QPs of one wavefront are adjacent in HBM (longer contiguous streams); the
 * unconstrained solve reads it (the IPM and the linearisation write / read
 * QP-major only for now: srbd_qp_create rejects stage-major with
 * constraints).  Outputs are always QP-major.                              */
enum { SRBD_QP_LAYOUT_QP_MAJOR = 0, SRBD_QP_LAYOUT_STAGE_MAJOR = 1 };

/* hpipm::OcpQpIpmSolverSettings (ocp_qp_ipm_solver_settings.hpp:26-86);
 * srbd_qp_default_settings() gives the same defaults.                     */
typedef struct srbd_qp_settings {
  int mode;       /* HpipmMode: 0 SpeedAbs, 1 Speed, 2 Balance, 3 Robust; selects
                  * itref_corr_max 0 / 0 / 2 / 4             */
  int iter_max;
  double alpha_min;
  double mu0;
  double tol_stat, tol_eq, tol_ineq, tol_comp;
  double reg_prim;
  int warm_start;   /* 1: x/u output buffers hold the primal warm start     */
  int pred_corr;
  int ric_alg;      /* 0: classical Riccati; else the square-root recursion  */
  int split_step;
  int compute_residuals; /* unconstrained QPs (nc = 0): 1 (default) = res/obj, when
                          * given, hold the solution's KKT residual norms and
                          * objective (HPIPM's comp_res_exit; one extra pass over
                          * the QP data); 0 = they are zero-filled              */
  int f64_rescue;   /* fp32 solves with constraints only (ignored otherwise):
                     * 0 (default) = HPIPM's s_ocp_qp_ipm behaviour; n > 0 =
                     * the fp32 pass runs min(n, iter_max) iterations, then
                     * every QP it left with status != Success continues in
                     * fp64 (iter_max as given) on its data widened to fp64,
                     * starting from the fp32 iterate (x, u, pi, lam, t; cold
                     * when nx or nu < 12 or the iterate is not finite), and
                     * its outputs (x, u, pi, P, p, K, k, status, iter, res,
                     * obj, stat) are the fp64 solve's, narrowed.  The call
                     * then waits for the fp32 pass (it counts the QPs to
                     * re-solve on the host).                               */
  int f32_iters;    /* fp64 solves with constraints on 12 x 12 stages and
                     * iter_max >= 2 only (ignored otherwise): 0 (default) =
                     * fp64 throughout; n > 0 = a mixed-precision IPM: the data
                     * is narrowed once to fp32, the first m = min(n,
                     * iter_max - 1) iterations run in fp32 (half the bytes per
                     * sweep), and the fp64 IPM continues from that iterate (x,
                     * u, pi, lam, t) on the caller's fp64 data to the fp64
                     * tolerances for at most iter_max - m iterations; iter and
                     * stat count the fp64 iterations.  Contract: the mixed path
                     * never ends a QP worse than the fp64 path.  Every QP the
                     * continuation does not end with Success is solved again
                     * in fp64 exactly as the plain fp64 call would solve it
                     * (iter_max iterations, from the caller's x / u when
                     * warm_start is set, cold otherwise) and then carries that
                     * solve's outputs, bit for bit; the call waits once to
                     * count them.  Worst case per QP: iter_max iterations (m of
                     * them fp32) plus iter_max fp64 ones.                  */
  int lq_fact;      /* HPIPM's lq_fact (d_ocp_qp_ipm_arg_set "lq_fact",
                     * hpipm_d_ocp_qp_ipm.h:78,147), square-root Riccati only:
                     * -1 (default) = the mode's, as d_ocp_qp_ipm_arg_set_default
                     * sets it (Balance 1, Robust 2, else 0); 0 = Cholesky
                     * factorizations; 1 = Cholesky until a predictor step's
                     * linear residual exceeds 1e-5, then LQ for the rest of
                     * the solve; 2 = every stage factorization by LQ (the
                     * barrier Hessians are absorbed as columns, never summed).
                     * Ignored with ric_alg = 0. (ABI 11)                    */
} srbd_qp_settings;

typedef struct srbd_qp_data_f64 {
  const double *A, *B, *b, *Q, *S, *R, *q, *r;
  const double *lbu, *ubu, *lbu_mask, *ubu_mask;
  const double *lbx, *ubx, *lbx_mask, *ubx_mask;
  const double *C, *D, *lg, *ug, *lg_mask, *ug_mask;
  const double *x0;
} srbd_qp_data_f64;

typedef struct srbd_qp_solution_f64 {
  double *x, *u, *pi;      /* required                                     */
  double *P, *p, *K, *k;   /* optional Riccati outputs (may be NULL)        */
  int *status, *iter;      /* optional                                     */
  double *res;             /* optional [batch][4] max |res_stat|,|res_eq|,|res_ineq|,|res_comp| */
  double *obj;             /* optional [batch]                              */
  double *stat;            /* optional [batch][iter_max+2][18]: per-iteration
                            * statistics in HPIPM's ws->stat row layout, the
                            * rows hpipm-cpp copies into OcpQpIpmSolverStatistics
                            * (ocp_qp_ipm_solver.cpp:381-403): alpha_aff, mu_aff,
                            * sigma, alpha_prim, alpha_dual, mu, res_stat, res_eq,
                            * res_ineq, res_comp, obj, lq_fact (0: none),
                            * itref_pred (0), itref_corr (corrections of the
                            * step, mode Balance / Robust with boxes), then
                            * lin_res_stat, lin_res_eq of the last refinement
                            * check, lin_res_ineq, lin_res_comp (0: exact).    */
} srbd_qp_solution_f64;

/* fp32 twins (BASELINE config 5; HPIPM's s_ocp_qp_ipm, hpipm_s_ocp_qp_ipm.h:238):
 * same fields, same layout, float elements.  Tolerances below ~1e-6 are not
 * reachable in fp32; use the NMPC settings (1e-4). */
typedef struct srbd_qp_data_f32 {
  const float *A, *B, *b, *Q, *S, *R, *q, *r;
  const float *lbu, *ubu, *lbu_mask, *ubu_mask;
  const float *lbx, *ubx, *lbx_mask, *ubx_mask;
  const float *C, *D, *lg, *ug, *lg_mask, *ug_mask;
  const float *x0;
} srbd_qp_data_f32;

typedef struct srbd_qp_solution_f32 {
  float *x, *u, *pi;
  float *P, *p, *K, *k;
  int *status, *iter;
  float *res;
  float *obj;
  float *stat;
} srbd_qp_solution_f32;

typedef struct srbd_qp_handle_s* srbd_qp_handle;

/* Fill *s with hpipm-cpp's defaults (Speed, iter_max 15, tol 1e-8, mu0 100,
 * alpha_min 1e-8, reg_prim 1e-12, pred_corr 1, ric_alg 1, split_step 0).   */
void srbd_qp_default_settings(srbd_qp_settings* s);

/* Validate settings like OcpQpIpmSolverSettings::checkSettings
 * (ocp_qp_ipm_solver_settings.cpp:7-38); returns SRBD_QP_ESETTINGS with a
 * message retrievable by srbd_qp_last_error().                              */
int srbd_qp_check_settings(const srbd_qp_settings* s);

/* Create a solver for `dims` able to solve up to `batch_capacity` QPs per call
 * on HIP device `device`.  Allocates the device workspace and one stream.  */
int srbd_qp_create(const srbd_qp_dims* dims, int batch_capacity, int device,
                   srbd_qp_handle* out);

/* Device-resident batch solve, asynchronous on `stream` (a hipStream_t; NULL
 * = the handle's own stream): the call enqueues the whole solve and returns
 * without waiting -- the IPM's stop decision is taken on the device -- except
 * that settings->f64_rescue / f32_iters wait once for their first pass.
 * Every data/solution pointer is device memory.  With settings->warm_start the
 * x/u buffers are read as the warm start.  One handle serves one solve at a
 * time (its workspace); several handles run concurrently.
 * Cost of the asynchronous stop: the batched IPM enqueues all iter_max
 * iterations up front; the iterations after the device has stopped the solve
 * cost their dispatch only (about 2 to 6 launches per iteration, a few
 * microseconds each, so ~0.1 ms for the NMPC's iter_max 30).  fp64 solves of
 * up to 512 QPs with the classical Riccati (ric_alg 0), or the square root
 * without C rows (any mode: Balance / Robust refine in the same launch) run as
 * one launch instead (the latency IPM), which stops where it
 * converges.  With the square root and lq_fact 1 (Balance's) that call waits
 * for its stream once: a QP asking for the LQ factorization is solved again,
 * alone, on the batched kernels before the call returns.
 * SRBD_IPM_LATENCY_MAX (environment, QPs; 0 = off) moves that switch.     */
int srbd_qp_solve_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* settings,
                      const srbd_qp_data_f64* data, const srbd_qp_solution_f64* sol,
                      void* stream);

/* Host-buffer batch solve: copies to device, solves, copies back, waits.
 * Small unconstrained batches (<= 256 QPs, nx = nu = 12, N <= 26) are zero copy:
 * the kernel reads the handle's pinned staging buffer and writes the outputs
 * into it.  A single such QP with the classical Riccati (ric_alg 0, N <= 20:
 * the reference's call pattern) goes to the handle's resident server: a
 * one-workgroup kernel on its own stream that polls a mailbox in mapped host
 * memory, so a call costs no launch; it leaves its CU after 5 ms without a
 * request, after its first answer once it has been up 20 ms, or at
 * srbd_qp_destroy / process exit, and the next call relaunches it (also when
 * it left between the call's check and its post).  While it is up it holds
 * one CU, and a device-wide synchronize waits for it to leave.  Its stream
 * has the greatest priority: HIP maps a process's streams onto a few hardware
 * queues per priority that run their packets in order, so a kernel queued
 * behind the server on a shared queue would wait for it; default-priority
 * streams never share its queue, and another high-priority stream that does
 * waits at most the 20 ms lifetime.  SRBD_LAT_SERVER=0 (environment) launches
 * per call; SRBD_LAT_SERVER_IDLE_MS overrides the 5 ms (tests).          */
int srbd_qp_solve_host_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* settings,
                           const srbd_qp_data_f64* data, const srbd_qp_solution_f64* sol);

/* srbd_qp_solve_host_f64 that hands the caller the Riccati outputs early:
 * `on_factors(ctx)` runs at most once on the calling thread, before the call
 * returns, as soon as sol->P, p, K, k have been written to the caller's
 * buffers.  The call's return code and sol->status then decide whether they
 * are valid: the callback can run and the call still return an error (a
 * device failure after the factors were written) or a QP end with status 3
 * (NaN: the status is set after the callback), so a caller keeps what it
 * unpacked only on SRBD_QP_OK and status 0.  On the zero-copy single-QP path (above; fp64 classical
 * Riccati, N <= 20) that is while the kernel still runs its forward sweep,
 * u / pi and residual passes, so a caller can unpack the factors (the bulk of
 * the outputs) under the kernel's tail; elsewhere it runs after the solve.
 * The callback must not call into the handle.  Replaces the
 * d_ocp_qp_ipm_get_ric_P / _p / _K / _k reads of ocp_qp_ipm_solver.cpp:342-345
 * for the hpipm-cpp shim.  (ABI 12)                                          */
int srbd_qp_solve_host_cb_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* settings,
                              const srbd_qp_data_f64* data, const srbd_qp_solution_f64* sol,
                              void (*on_factors)(void* ctx), void* ctx);

/* The handle's pinned host staging for a srbd_qp_solve_host_f64 call of `batch`
 * QPs with `settings`: every field that *data / *sol have non-NULL (any value,
 * e.g. (void*)1: a marker) is replaced by its place in the staging buffer, the
 * others set NULL.  A caller that packs its QPs there and then passes the same
 * two structs to srbd_qp_solve_host_f64 saves both staging copies (the solve
 * skips a copy whose source already is its place); the outputs are left there.
 * The pointers are invalidated by the handle's destruction and by ANY later
 * srbd_qp_solve_host_* or srbd_qp_host_staging_* call on the handle that needs a
 * larger staging buffer (the old pinned buffer is freed): re-stage after such a
 * call, as the hpipm-cpp shim does on every solve.  SRBD_QP_ECAPACITY
 * when the call's buffers exceed the pinned staging size (8 MiB).  Replaces the
 * Eigen-pointer marshalling of ocp_qp_ipm_solver.cpp:226-289 for the shim.
 * (ABI 10)                                                                  */
int srbd_qp_host_staging_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* settings,
                             srbd_qp_data_f64* data, srbd_qp_solution_f64* sol);

/* fp32 twins of the two solve entry points (the handle serves both).      */
int srbd_qp_solve_f32(srbd_qp_handle h, int batch, const srbd_qp_settings* settings,
                      const srbd_qp_data_f32* data, const srbd_qp_solution_f32* sol,
                      void* stream);
int srbd_qp_solve_host_f32(srbd_qp_handle h, int batch, const srbd_qp_settings* settings,
                           const srbd_qp_data_f32* data, const srbd_qp_solution_f32* sol);

/* ------------------------------------------------------------------------
 * Device-side SRBD linearisation: the producer of the QP data, i.e.
 * NMPCSolver::prepareQpStructures (NMPC_solver.cpp:276-314) with the model of
 * dynamics/SRBD_model.cpp:75-295 (RK4 defect with Euler Jacobians, friction
 * cone as a relaxed log barrier in the cost), for a batch of linearisation
 * points, written straight into the solver's input buffers.
 * Parameters: config/mpc_option.yaml:2-18, NMPC_solver.cpp:53-82, :332-351.
 * ---------------------------------------------------------------------- */
typedef struct srbd_model_params {
  double Q[12], Qf[12];   /* diagonal state weights (mpc_option.yaml Q, Qf)    */
  double R;               /* input weight                                      */
  double dt;              /* discretisation step                               */
  double Lbody[3];        /* body inertia diagonal (the model stores L^-1)     */
  double mu_b, theta_b;   /* relaxed-barrier weight / threshold                */
  double mass;
  double foot_r[3], foot_l[3];  /* foot positions in the body frame          */
  double mu, Lfx, Lfz, fmax, fmin;  /* friction cone / torque limits         */
  double x_ref[12];       /* reference state                                   */
  double qf_scale;        /* terminal weight factor (<= 0: N, NMPC_solver.cpp:58) */
  double u_lo[12], u_hi[12];  /* box on u + du for SRBD_QP_SRBD_BOX_U         */
} srbd_model_params;

enum { SRBD_QP_SRBD_NONE = 0, SRBD_QP_SRBD_BOX_U = 1, SRBD_QP_SRBD_CONE = 2 };

/* mpc_option.yaml / setupDynamics defaults (box: (+-50, +-50, 0..300 N,
 * +-5 Nm) per foot). */
void srbd_qp_srbd_default_params(srbd_model_params* p);

/* Linearise `batch` SRBD trajectories on the handle's device and stream (or
 * `stream`): xs [batch][N+1][12], us [batch][N][12] (device).  Fills A, B, b,
 * Q, S, R, q, r of `out` and, per `constraints`, lbu/ubu (BOX_U) or D, lg,
 * ug, lg_mask, ug_mask (CONE: ng = 24, lg = -f(u), ug masked; C = 0 is
 * written only if out->C is given -- pass C = NULL to the solve).  The handle's
 * dims must be N, nx = nu = 12 (and ng = 24 for CONE).  Asynchronous.       */
int srbd_qp_srbd_linearize_f64(srbd_qp_handle h, int batch, const srbd_model_params* params,
                               int constraints, const double* xs, const double* us,
                               const srbd_qp_data_f64* out, void* stream);

/* Batched filter line search of the SQP iteration (NMPCSolver::linearSearch,
 * NMPC_solver.cpp:149-274): per QP, merit phi (cost + friction barrier) and
 * theta (shooting defect) at xs/us, trial steps alpha, beta alpha, ... along
 * the QP solution (dx [B][N+1][12], du [B][N][12]) until the filter accepts;
 * xs/us (device, in place) move to the accepted point.  alpha [B] is read and
 * written like the reference's persistent alpha_ (NMPC_solver.h:104); merit
 * [B][3] (phi, theta, dphi) and converged [B] (dphi > -1e-3 && theta < 1e-6)
 * are optional.  Constants: NMPC_solver.h:97-103.                         */
typedef struct srbd_linesearch_params {
  double theta_max, theta_min, eta, beta_phi, beta_theta, beta_alpha, alpha_min;
} srbd_linesearch_params;
void srbd_qp_srbd_default_linesearch(srbd_linesearch_params* p);
int srbd_qp_srbd_linesearch_f64(srbd_qp_handle h, int batch, const srbd_model_params* params,
                                const srbd_linesearch_params* ls, double* xs, double* us,
                                const double* dx, const double* du, double* alpha, double* merit,
                                int* converged, void* stream);

/* The SQP loop of NMPCSolver::controlLoop (NMPC_solver.cpp:362-372) for a batch
 * of robots: for it < sqp_max_loop (mpc_option.yaml sqp_max_loop):
 * prepareQpStructures (srbd_qp_srbd_linearize_f64 at xs, us), solveQpProblems
 * (srbd_qp_solve_f64 with settings and x0 - xs[:, 0], NMPC_solver.cpp:316-330),
 * checkConvergence = linearSearch (srbd_qp_srbd_linesearch_f64: xs, us move to
 * the accepted point, alpha persists); a robot whose line search reports
 * convergence stops there (`if (checkConvergence()) break;`) and is not changed
 * again.  xs [batch][N+1][12], us [batch][N][12] (in/out), x0 [batch][12],
 * alpha [batch] (in/out), sqp_iter [batch] (SQP iterations run) and converged
 * [batch] (out): device memory.  The QP data, solution and loop state live in
 * a scratch buffer of the handle (allocated on first use, capacity-sized).
 * Runs on the handle's stream and returns when every robot has stopped or
 * sqp_max_loop iterations ran (one 4-byte read-back per iteration).  The
 * handle's dims: N, nx = nu = 12, and has_box_u / ng = 24 per `constraints`. */
int srbd_qp_srbd_nmpc_f64(srbd_qp_handle h, int batch, const srbd_model_params* params,
                          const srbd_linesearch_params* ls, const srbd_qp_settings* settings,
                          int constraints, int sqp_max_loop, double* xs, double* us,
                          const double* x0, double* alpha, int* sqp_iter, int* converged);

/* ------------------------------------------------------------------------
 * One solver over several devices, driven from one host thread (SURVEY.md 5,
 * "one process, 8 devices"; BASELINE config 4: a batch sharded over 8 MI355X
 * with the solutions gathered to one device).  A handle per device; the
 * shards' solves are all queued before any is waited for, and x, u, pi are
 * gathered to the root device (devices[0]) by peer copies over xGMI, each
 * behind its shard's solve on that shard's stream.  (ABI 10)
 * ---------------------------------------------------------------------- */
typedef struct srbd_qp_multi_s* srbd_qp_multi;

/* A handle of `capacity_per_device` QPs on each of devices[0..ndev) (a device
 * may repeat: two shards on one GPU).  Peer access root <-> shard is enabled
 * where the devices support it.                                              */
int srbd_qp_multi_create(const srbd_qp_dims* dims, int capacity_per_device, const int* devices,
                         int ndev, srbd_qp_multi* out);
void srbd_qp_multi_destroy(srbd_qp_multi m);
/* Shard i's handle (its stream, workspace size, ...); NULL past the end.    */
srbd_qp_handle srbd_qp_multi_handle(srbd_qp_multi m, int i);
/* Shard i: batch[i] QPs with data[i] / sol[i] in devices[i]'s memory.  Every
 * shard is solved with `settings`; then, when root_x / root_u / root_pi are
 * given (root-device memory for sum(batch) QPs, the C-ABI layout), the shards'
 * x, u, pi land there in shard order.  Returns when all of it has finished. */
int srbd_qp_multi_solve_f64(srbd_qp_multi m, const int* batch, const srbd_qp_settings* settings,
                            const srbd_qp_data_f64* data, const srbd_qp_solution_f64* sol,
                            double* root_x, double* root_u, double* root_pi);
/* The fp32 twin (BASELINE config 5 sharded; HPIPM's s_ocp_qp_ipm), the same
 * contract with srbd_qp_solve_f32 on every shard.  (ABI 11)                   */
int srbd_qp_multi_solve_f32(srbd_qp_multi m, const int* batch, const srbd_qp_settings* settings,
                            const srbd_qp_data_f32* data, const srbd_qp_solution_f32* sol,
                            float* root_x, float* root_u, float* root_pi);

/* Blocks until all work queued on the handle's stream is done.            */
int srbd_qp_synchronize(srbd_qp_handle h);

/* The handle's hipStream_t (for event timing / stream interop).           */
void* srbd_qp_stream(srbd_qp_handle h);

/* Device workspace bytes the handle holds.                                */
size_t srbd_qp_workspace_bytes(srbd_qp_handle h);

/* Every byte the handle holds right now: the workspace plus the buffers it
 * allocates on first use (host-solve staging and its pinned host mirror, the
 * 12 x 12 embedding, the NMPC loop state, the f64_rescue / f32_iters
 * batches).  A pool of handles (hpipm-cpp's, which re-implements the
 * reference's construct-per-solve pattern, NMPC_solver.cpp:318-319) sizes
 * itself by this.  (ABI 9)                                                  */
size_t srbd_qp_memory_bytes(srbd_qp_handle h);

void srbd_qp_destroy(srbd_qp_handle h);

/* "HpipmStatus::Success" ... like hpipm::to_string (ocp_qp_ipm_solver.cpp:19-33) */
const char* srbd_qp_status_string(int status);
const char* srbd_qp_error_string(int err);
/* Message of the last error raised on this thread (never NULL).           */
const char* srbd_qp_last_error(void);

int srbd_qp_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SRBD_QP_H_ */
