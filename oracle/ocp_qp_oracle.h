/*
 * ocp_qp_oracle.h -- CPU restatement of the reference's OCP-QP solve path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle (and the bench's
 * `cpu_baseline` "port").  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path (libsrbd_qp.so) never links
 * or calls it.
 *
 * What it restates (reference = /root/reference, read as text only):
 *   - hpipm::OcpQpIpmSolver::solve() boundary conventions
 *       hpipm-cpp/src/ocp_qp_ipm_solver.cpp:181-414
 *       (x0 elimination :225,236 / nx[0]=0 :128-130, stage-0 rebuild :347-373)
 *   - the unconstrained Riccati recursion pinned by the reference test
 *       hpipm-cpp/test/ocp_qp_ipm_solver.cpp:67-90
 *   - HPIPM's relative-formulation Mehrotra predictor-corrector IPM
 *       (d_ocp_qp_ipm_solve, hpipm_d_ocp_qp_ipm.h:238; core ops
 *        hpipm_d_core_qp_ipm_aux.h:44-62; residuals hpipm_d_ocp_qp_res.h:57-67).
 *     HPIPM's C sources are NOT vendored in the reference (headers only), so
 *     the IPM is restated from the vendored declarations and the published
 *     algorithm; iteration traces are not claimed to match HPIPM, the
 *     solution and KKT residuals are (see DESIGN.md "Parity").
 *
 * Parity pins (tests/test_oracle.py):
 *   - textbook Riccati of test/ocp_qp_ipm_solver.cpp:67-90 (rel 1e-10)
 *   - OSQP golden trajectories sol0..14.txt of test/ocp_qp_ipm_solver.cpp:170-315
 *     (box-constrained quadcopter, masks, warm start; rel 1e-9)
 *   - numpy dense-KKT solve of the unconstrained QP.
 *
 * Data layout (identical to the C-ABI in include/srbd_qp.h, one QP):
 *   every matrix block is column-major (Eigen default), blocks are stacked
 *   stage after stage.  Box constraints are dense per variable with 0/1
 *   masks (a masked bound is absent); see include/srbd_qp.h.
 */
#ifndef SRBD_OCP_QP_ORACLE_H_
#define SRBD_OCP_QP_ORACLE_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_ocp_qp {
  int N, nx, nu, ng;
  const double *A, *B, *b;  /* N*nx*nx, N*nx*nu, N*nx                        */
  const double *Q, *S, *R;  /* (N+1)*nx*nx, N*nu*nx, N*nu*nu                */
  const double *q, *r;      /* (N+1)*nx, N*nu                               */
  /* dense box on u: N*nu each, or NULL (no box).  NULL mask => all ones.    */
  const double *lbu, *ubu, *lbu_mask, *ubu_mask;
  /* dense box on x: (N+1)*nx each, or NULL.  Stage 0 ignored (x0 fixed).    */
  const double *lbx, *ubx, *lbx_mask, *ubx_mask;
  /* general lg <= C x + D u <= ug : C (N+1)*ng*nx, D N*ng*nu, lg/ug (N+1)*ng.
   * C at stage 0 is ignored, mirroring hpipm-cpp's nx[0]=0 embedding.       */
  const double *C, *D, *lg, *ug, *lg_mask, *ug_mask;
} oracle_ocp_qp;

typedef struct oracle_settings {
  int iter_max;
  double alpha_min, mu0, tol_stat, tol_eq, tol_ineq, tol_comp, reg_prim;
  int warm_start, pred_corr, split_step;
  int ric_alg;  /* 0 classical Riccati; else square root: P_k = Lx Lx', with the
                 * stage products formed from chol(P_{k+1}) (HPIPM square_root_alg) */
  int itref_corr_max; /* iterative refinement steps of the final (corrector) step        */
  int lq_fact;  /* HPIPM lq_fact: 0 Cholesky; 2 LQ factorization of every stage (square-root
                 * form, Gamma as its square root beside the data); 1 Cholesky until a
                 * predictor step's linear residual exceeds 1e-5, LQ from then on.  HPIPM's
                 * Balance / Robust select 1 / 2; the oracle takes it only when asked (the HIP
                 * library does not build it: DESIGN.md 9)                                     */
} oracle_settings;

typedef struct oracle_result {
  int status;        /* 0 Success, 1 MaxIter, 2 MinStep, 3 NaN            */
  int iter;
  double res[4];     /* max |res_stat|, |res_eq|, |res_ineq|, |res_comp|    */
  double obj;
  int lq_iters;      /* iterations whose step came from the LQ factorization */
} oracle_result;

/* Solve one QP.  x ((N+1)*nx), u (N*nu): in = warm start (if enabled), out =
 * solution.  pi ((N+1)*nx).  P ((N+1)*nx*nx), p ((N+1)*nx), K (N*nu*nx),
 * k (N*nu) may be NULL.  Returns 0 on success, <0 on bad arguments.       */
int oracle_solve(const oracle_ocp_qp* qp, const oracle_settings* st,
                 const double* x0, double* x, double* u, double* pi,
                 double* P, double* p, double* K, double* k,
                 oracle_result* res);

/* Batch helper: QP i reads every pointer advanced by i times the per-QP
 * size; runs on `threads` POSIX threads (the CPU baseline).                */
int oracle_solve_batch(int batch, const oracle_ocp_qp* qp0,
                       const oracle_settings* st, const double* x0,
                       double* x, double* u, double* pi, int* status,
                       int* iters, int threads);

#ifdef __cplusplus
}
#endif
#endif
