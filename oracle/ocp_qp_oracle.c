/*
 * ocp_qp_oracle.c -- CPU restatement of the OCP-QP solve (parity oracle).
 *
 * TEST INFRASTRUCTURE ONLY (see ocp_qp_oracle.h).  Plain C99, scalar, one QP
 * at a time; oracle_solve_batch() spreads QPs over POSIX threads for the
 * bench's cpu_baseline ("port").
 *
 * Algorithm map (reference file:line):
 *   riccati_factor / riccati_vectors / riccati_forward
 *       textbook recursion of hpipm-cpp/test/ocp_qp_ipm_solver.cpp:67-90
 *       (P_N = Q_N, s_N = -q_N; F, H, G; K = -G^-1 H; P = F - K'GK; forward
 *       rollout :83-87; costate lmd = P x - s :90), written with p = -s so
 *       that pi_k = P_k x_k + p_k (hpipm-cpp convention, solution.hpp:12-48).
 *   x0 handling: x0 is fixed, stage-0 x-constraints and C_0 are dropped,
 *       mirroring nx[0]=nbx[0]=0 (src/ocp_qp_ipm_solver.cpp:128-130) and the
 *       b0/r0 fold (:225,236).
 *   stage-0 outputs: the rebuild of src/ocp_qp_ipm_solver.cpp:347-373.
 *   ipm(): relative-formulation Mehrotra predictor-corrector of HPIPM
 *       d_ocp_qp_ipm_solve (hpipm_d_ocp_qp_ipm.h:238), core ops of
 *       hpipm_d_core_qp_ipm_aux.h:44-62 (Gamma/gamma, alpha, update, mu_aff,
 *       centering correction), residuals of hpipm_d_ocp_qp_res.h:57-67,
 *       exit statuses of hpipm_common.h (SUCCESS/MAX_ITER/MIN_STEP/NAN_SOL).
 */
#include "ocp_qp_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#ifdef ORACLE_DEBUG
#include <stdio.h>
#endif

#define IPM_THR0 0.1      /* minimum initial slack (HPIPM init_var)          */
#define IPM_STEP_TAU 0.995 /* fraction-to-boundary factor                     */

/* ------------------------------------------------------------------ */
/* small dense helpers, column-major, leading dimension = rows          */
/* ------------------------------------------------------------------ */
#define M_(a, ld, i, j) ((a)[(size_t)(i) + (size_t)(j) * (size_t)(ld)])

/* C(m x n) = A(m x k) * B(k x n) */
static void mm(int m, int n, int k, const double* A, const double* B, double* C) {
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0.0;
      for (int l = 0; l < k; ++l) s += M_(A, m, i, l) * M_(B, k, l, j);
      M_(C, m, i, j) = s;
    }
}
/* C(m x n) = A(k x m)' * B(k x n) */
static void mtm(int m, int n, int k, const double* A, const double* B, double* C) {
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0.0;
      for (int l = 0; l < k; ++l) s += M_(A, k, l, i) * M_(B, k, l, j);
      M_(C, m, i, j) = s;
    }
}
/* y(m) = A(m x n) x */
static void mv(int m, int n, const double* A, const double* x, double* y) {
  for (int i = 0; i < m; ++i) {
    double s = 0.0;
    for (int j = 0; j < n; ++j) s += M_(A, m, i, j) * x[j];
    y[i] = s;
  }
}
/* y(n) = A(m x n)' x */
static void mtv(int m, int n, const double* A, const double* x, double* y) {
  for (int j = 0; j < n; ++j) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) s += M_(A, m, i, j) * x[i];
    y[j] = s;
  }
}
/* in-place lower Cholesky of a (n x n).  A non-positive pivot is not an
 * error: like BLASFEO's dpotrf_l (which HPIPM's Riccati calls)
 * the pivot and its column are zeroed and the solves skip that direction.
 * Returns the number of such pivots.                                       */
static int chol(int n, double* a) {
  int bad = 0;
  for (int j = 0; j < n; ++j) {
    double d = M_(a, n, j, j);
    for (int l = 0; l < j; ++l) d -= M_(a, n, j, l) * M_(a, n, j, l);
    double inv;
    if (d > 0.0) { d = sqrt(d); inv = 1.0 / d; } else { d = 0.0; inv = 0.0; ++bad; }
    M_(a, n, j, j) = d;
    for (int i = j + 1; i < n; ++i) {
      double s = M_(a, n, i, j);
      for (int l = 0; l < j; ++l) s -= M_(a, n, i, l) * M_(a, n, j, l);
      M_(a, n, i, j) = s * inv;
    }
    for (int i = 0; i < j; ++i) M_(a, n, i, j) = 0.0;
  }
  return bad;
}
/* solve (L L') x = b in place, L lower (n x n); zero pivots give zero */
static void chol_solve(int n, const double* L, double* b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int l = 0; l < i; ++l) s -= M_(L, n, i, l) * b[l];
    double d = M_(L, n, i, i);
    b[i] = d > 0.0 ? s / d : 0.0;
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int l = i + 1; l < n; ++l) s -= M_(L, n, l, i) * b[l];
    double d = M_(L, n, i, i);
    b[i] = d > 0.0 ? s / d : 0.0;
  }
}

/* ------------------------------------------------------------------ */
/* QP access                                                            */
/* ------------------------------------------------------------------ */
typedef struct {
  const oracle_ocp_qp* qp;
  int N, nx, nu, ng, n;
} dims_t;

static const double* qA(const dims_t* d, int k) { return d->qp->A + (size_t)k * d->nx * d->nx; }
static const double* qB(const dims_t* d, int k) { return d->qp->B + (size_t)k * d->nx * d->nu; }
static const double* qb(const dims_t* d, int k) { return d->qp->b + (size_t)k * d->nx; }
static const double* qQ(const dims_t* d, int k) { return d->qp->Q + (size_t)k * d->nx * d->nx; }
static const double* qS(const dims_t* d, int k) { return d->qp->S + (size_t)k * d->nu * d->nx; }
static const double* qR(const dims_t* d, int k) { return d->qp->R + (size_t)k * d->nu * d->nu; }
static const double* qq(const dims_t* d, int k) { return d->qp->q + (size_t)k * d->nx; }
static const double* qr(const dims_t* d, int k) { return d->qp->r + (size_t)k * d->nu; }

/* One inequality row of stage k over v_k = [u_k; x_k] (length n_k). */
typedef struct {
  int kind;          /* 0 box (single var), 1 general                      */
  int var;           /* box: index into v                                   */
  const double* Drow; /* general: D row (stride ng), may be NULL            */
  const double* Crow; /* general: C row (stride ng), may be NULL            */
  double lb, ub;
  int has_l, has_u;
  /* IPM state */
  double lam_l, lam_u, t_l, t_u;
  double rd_l, rd_u, rm_l, rm_u; /* res_d, res_m                            */
  double dlam_l, dlam_u, dt_l, dt_u;
  double aff_l, aff_u;           /* dlam_aff * dt_aff                        */
  double G;                      /* this iteration's barrier Hessian weight  */
  int gidx;                      /* general rows: the row's index in 0..ng-1  */
} row_t;

typedef struct {
  int nu_k;          /* nu at this stage (0 at N)                          */
  int nrow;
  row_t* rows;
} stage_rows_t;

static double row_dot(const dims_t* d, const row_t* rw, int nu_k, const double* u, const double* x) {
  if (rw->kind == 0) return rw->var < nu_k ? u[rw->var] : x[rw->var - nu_k];
  double s = 0.0;
  if (rw->Drow && nu_k > 0)
    for (int j = 0; j < d->nu; ++j) s += rw->Drow[(size_t)j * d->ng] * u[j];
  if (rw->Crow)
    for (int j = 0; j < d->nx; ++j) s += rw->Crow[(size_t)j * d->ng] * x[j];
  return s;
}
/* g[v] += c * row */
static void row_axpy(const dims_t* d, const row_t* rw, int nu_k, double c, double* gu, double* gx) {
  if (rw->kind == 0) {
    if (rw->var < nu_k) gu[rw->var] += c; else gx[rw->var - nu_k] += c;
    return;
  }
  if (rw->Drow && nu_k > 0)
    for (int j = 0; j < d->nu; ++j) gu[j] += c * rw->Drow[(size_t)j * d->ng];
  if (rw->Crow)
    for (int j = 0; j < d->nx; ++j) gx[j] += c * rw->Crow[(size_t)j * d->ng];
}
/* H[v,v] += c * row row'  (H is n_k x n_k, order [u; x]) */
static void row_syr(const dims_t* d, const row_t* rw, int nu_k, double c, double* H) {
  int n = nu_k + d->nx;
  if (rw->kind == 0) { M_(H, n, rw->var, rw->var) += c; return; }
  double vrow[64];
  for (int j = 0; j < n; ++j) vrow[j] = 0.0;
  if (rw->Drow && nu_k > 0)
    for (int j = 0; j < d->nu; ++j) vrow[j] = rw->Drow[(size_t)j * d->ng];
  if (rw->Crow)
    for (int j = 0; j < d->nx; ++j) vrow[nu_k + j] = rw->Crow[(size_t)j * d->ng];
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) M_(H, n, i, j) += c * vrow[i] * vrow[j];
}

static stage_rows_t* build_rows(const dims_t* d, int* nc_out) {
  const oracle_ocp_qp* qp = d->qp;
  stage_rows_t* st = (stage_rows_t*)calloc((size_t)d->N + 1, sizeof(stage_rows_t));
  int nc = 0;
  for (int k = 0; k <= d->N; ++k) {
    int nu_k = k < d->N ? d->nu : 0;
    int cap = (qp->lbu && k < d->N ? d->nu : 0) + (qp->lbx && k > 0 ? d->nx : 0) + (qp->lg ? d->ng : 0);
    st[k].nu_k = nu_k;
    st[k].rows = (row_t*)calloc((size_t)(cap > 0 ? cap : 1), sizeof(row_t));
    int nr = 0;
    if (qp->lbu && k < d->N) {
      for (int i = 0; i < d->nu; ++i) {
        size_t o = (size_t)k * d->nu + i;
        int hl = qp->lbu_mask ? qp->lbu_mask[o] != 0.0 : 1;
        int hu = qp->ubu_mask ? qp->ubu_mask[o] != 0.0 : 1;
        if (!hl && !hu) continue;
        row_t* rw = &st[k].rows[nr++];
        rw->kind = 0; rw->var = i; rw->lb = qp->lbu[o]; rw->ub = qp->ubu[o];
        rw->has_l = hl; rw->has_u = hu;
      }
    }
    if (qp->lbx && k > 0) {
      for (int i = 0; i < d->nx; ++i) {
        size_t o = (size_t)k * d->nx + i;
        int hl = qp->lbx_mask ? qp->lbx_mask[o] != 0.0 : 1;
        int hu = qp->ubx_mask ? qp->ubx_mask[o] != 0.0 : 1;
        if (!hl && !hu) continue;
        row_t* rw = &st[k].rows[nr++];
        rw->kind = 0; rw->var = nu_k + i; rw->lb = qp->lbx[o]; rw->ub = qp->ubx[o];
        rw->has_l = hl; rw->has_u = hu;
      }
    }
    if (qp->lg && d->ng > 0) {
      for (int c = 0; c < d->ng; ++c) {
        size_t o = (size_t)k * d->ng + c;
        int hl = qp->lg_mask ? qp->lg_mask[o] != 0.0 : 1;
        int hu = qp->ug_mask ? qp->ug_mask[o] != 0.0 : 1;
        if (!hl && !hu) continue;
        row_t* rw = &st[k].rows[nr++];
        rw->kind = 1;
        rw->gidx = c;
        rw->Drow = (k < d->N && qp->D) ? qp->D + (size_t)k * d->ng * d->nu + c : NULL;
        /* C_0 dropped: hpipm-cpp embeds x0 with nx[0]=0 (ocp_qp_ipm_solver.cpp:128) */
        rw->Crow = (k > 0 && qp->C) ? qp->C + (size_t)k * d->ng * d->nx + c : NULL;
        rw->lb = qp->lg[o]; rw->ub = qp->ug[o];
        rw->has_l = hl; rw->has_u = hu;
      }
    }
    st[k].nrow = nr;
    for (int i = 0; i < nr; ++i) nc += st[k].rows[i].has_l + st[k].rows[i].has_u;
  }
  *nc_out = nc;
  return st;
}

static void free_rows(const dims_t* d, stage_rows_t* st) {
  for (int k = 0; k <= d->N; ++k) free(st[k].rows);
  free(st);
}

/* ------------------------------------------------------------------ */
/* Riccati on a step problem with stage Hessians Ht_k ([u;x] order),    */
/* gradients gt_k, dynamics (A_k, B_k, bt_k) and a fixed x_0.            */
/* ------------------------------------------------------------------ */
typedef struct {
  double* Ht;  /* per stage n_k x n_k (stage N: nx x nx)                  */
  double* gt;  /* per stage n_k                                           */
  double* bt;  /* per stage nx (k < N)                                    */
  double* P;   /* (N+1) nx*nx */
  double* p;   /* (N+1) nx    */
  double* K;   /* N nu*nx     */
  double* kk;  /* N nu        */
  double* Lg;  /* N nu*nu (chol of G)                                     */
  size_t hstride, gstride;
  /* ric_alg != 0 (square root, HPIPM's form): the stage factors and y = Lu^-1 l_u    */
  double* Lf;  /* (N+1) n*n: stage k < N [Lu 0; Lxu Lx] (ld n), stage N Lx (ld nx)   */
  double* yv;  /* N nu                                                               */
  int sq;      /* 1 once the last factorization was the square-root one              */
  int sform;   /* 1: the vectors travel as s = Lx^-1 p (fact_solve), 0: p           */
} ric_ws_t;

/* ric_alg = 0: the textbook recursion (test/ocp_qp_ipm_solver.cpp:67-90): F, H, G from
 * P_{k+1}, K = -G^-1 H, P_k = F + H'K symmetrised (the square-root variant is
 * sqrt_factor below).                                                               */
static int riccati_factor(const dims_t* d, ric_ws_t* w, double reg) {
  const int nx = d->nx, nu = d->nu, n = nx + nu, N = d->N;
  double PA[32 * 32], PB[32 * 32], G[32 * 32], Hm[32 * 32], F[32 * 32];
  double* PN = w->P + (size_t)N * nx * nx;
  const double* HtN = w->Ht + (size_t)N * w->hstride;
  memcpy(PN, HtN, sizeof(double) * nx * nx);
  w->sq = 0;
  for (int k = N - 1; k >= 0; --k) {
    const double* A = qA(d, k);
    const double* B = qB(d, k);
    const double* P1 = w->P + (size_t)(k + 1) * nx * nx;
    const double* Ht = w->Ht + (size_t)k * w->hstride;
    mm(nx, nx, nx, P1, A, PA);
    mm(nx, nu, nx, P1, B, PB);
    mtm(nu, nu, nx, B, PB, G);
    mtm(nu, nx, nx, B, PA, Hm);
    mtm(nx, nx, nx, A, PA, F);
    for (int j = 0; j < nu; ++j)
      for (int i = 0; i < nu; ++i) M_(G, nu, i, j) += M_(Ht, n, i, j);
    for (int i = 0; i < nu; ++i) M_(G, nu, i, i) += reg;
    for (int j = 0; j < nx; ++j)
      for (int i = 0; i < nu; ++i) M_(Hm, nu, i, j) += M_(Ht, n, i, nu + j);
    for (int j = 0; j < nx; ++j)
      for (int i = 0; i < nx; ++i) M_(F, nx, i, j) += M_(Ht, n, nu + i, nu + j);
    double* L = w->Lg + (size_t)k * nu * nu;
    memcpy(L, G, sizeof(double) * nu * nu);
    chol(nu, L);
    /* K = -G^-1 H */
    double* K = w->K + (size_t)k * nu * nx;
    for (int j = 0; j < nx; ++j) {
      double col[32];
      for (int i = 0; i < nu; ++i) col[i] = M_(Hm, nu, i, j);
      chol_solve(nu, L, col);
      for (int i = 0; i < nu; ++i) M_(K, nu, i, j) = -col[i];
    }
    /* P = F + H'K, symmetrised */
    double* P = w->P + (size_t)k * nx * nx;
    for (int j = 0; j < nx; ++j)
      for (int i = 0; i < nx; ++i) {
        double s = M_(F, nx, i, j);
        for (int l = 0; l < nu; ++l) s += M_(Hm, nu, l, i) * M_(K, nu, l, j);
        M_(P, nx, i, j) = s;
      }
    for (int j = 0; j < nx; ++j)
      for (int i = j + 1; i < nx; ++i) {
        double s = 0.5 * (M_(P, nx, i, j) + M_(P, nx, j, i));
        M_(P, nx, i, j) = s; M_(P, nx, j, i) = s;
      }
  }
  return 0;
}

/* ric_alg != 0: HPIPM's square-root Riccati (square_root_alg, the hpipm-cpp default
 * ocp_qp_ipm_solver_settings.hpp:81) as its kkt routines form it (hpipm_d_ocp_qp_kkt.h:54-60;
 * restated, the source is not vendored).  The stage factor is carried, never re-formed from an
 * explicit P: with AL = [B'; A'] Lx_{k+1},
 *     L_k = [Lu 0; Lxu Lx] = chol(Ht_k + AL AL')           (dsyrk_dpotrf_ln_mn, one 24 x 24 factor)
 * so G = Lu Lu', H = Lxu Lu', P_k = Lx Lx' with Lx the trailing factor of the same elimination.
 * The Riccati vector travels in the two forms HPIPM's ws->valid_ric_p names
 * (hpipm_d_ocp_qp_ipm.h:134, "0 p*inv(L), 1 p"):
 *   sform 1 (d_ocp_qp_fact_solve_kkt_step / _unconstr: the factor's last row):
 *     m = Lx_{k+1}' b + s_{k+1}, l = g + AL m, y = Lu^-1 l_u, s_k = Lx^-1 (l_x - Lxu y)
 *   sform 0 (d_ocp_qp_solve_kkt_step: the corrector and the refinement):
 *     l = g + [B'; A'] (Lx_{k+1} (Lx_{k+1}' b) + p_{k+1}), y = Lu^-1 l_u, p_k = l_x - Lxu y
 * and the forward substitution never forms K or P:
 *     du = -Lu^-T (y + Lxu' dx), dx+ = A dx + B du + b, dpi = Lx (Lx' dx + s) | Lx (Lx' dx) + p.
 * The HIP library's square-root kernels (riccati.h riccati_step_sqrt, ipm_box_impl.h SQRT)
 * follow the same forms.                                                                     */
static const double* sq_L(const ric_ws_t* w, const dims_t* d, int k) {
  return w->Lf + (size_t)k * (size_t)d->n * d->n;
}
static int sqrt_factor(const dims_t* d, ric_ws_t* w, double reg) {
  const int nx = d->nx, nu = d->nu, n = nx + nu, N = d->N;
  double M[64 * 64], AL[64 * 32];
  w->sq = 1;
  {
    double* LN = w->Lf + (size_t)N * n * n;
    memcpy(LN, w->Ht + (size_t)N * w->hstride, sizeof(double) * nx * nx);
    chol(nx, LN);
  }
  for (int k = N - 1; k >= 0; --k) {
    const double* A = qA(d, k);
    const double* B = qB(d, k);
    const double* Ln = sq_L(w, d, k + 1);
    const int nun = k + 1 < N ? nu : 0, ldn = nun + nx; /* Lx_{k+1} = Ln[nun:, nun:] */
    for (int j = 0; j < nx; ++j) {
      for (int i = 0; i < nu; ++i) {
        double s = 0.0;
        for (int l = j; l < nx; ++l) s += M_(B, nx, l, i) * M_(Ln, ldn, nun + l, nun + j);
        M_(AL, n, i, j) = s;
      }
      for (int i = 0; i < nx; ++i) {
        double s = 0.0;
        for (int l = j; l < nx; ++l) s += M_(A, nx, l, i) * M_(Ln, ldn, nun + l, nun + j);
        M_(AL, n, nu + i, j) = s;
      }
    }
    const double* Ht = w->Ht + (size_t)k * w->hstride;
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) {
        double s = M_(Ht, n, i, j);
        for (int l = 0; l < nx; ++l) s += M_(AL, n, i, l) * M_(AL, n, j, l);
        M_(M, n, i, j) = s;
      }
    for (int i = 0; i < nu; ++i) M_(M, n, i, i) += reg;
    chol(n, M);
    memcpy(w->Lf + (size_t)k * n * n, M, sizeof(double) * n * n);
  }
  /* P = Lx Lx', Lg = Lu, K = -Lu^-T Lxu' for the getters (ocp_qp_ipm_solver.cpp:337-346) */
  for (int k = 0; k <= N; ++k) {
    const int nuk = k < N ? nu : 0, ld = nuk + nx;
    const double* L = sq_L(w, d, k);
    double* P = w->P + (size_t)k * nx * nx;
    for (int j = 0; j < nx; ++j)
      for (int i = 0; i < nx; ++i) {
        double s = 0.0;
        for (int l = 0; l < nx; ++l) s += M_(L, ld, nuk + i, nuk + l) * M_(L, ld, nuk + j, nuk + l);
        M_(P, nx, i, j) = s;
      }
    if (k == N) continue;
    double* Lg = w->Lg + (size_t)k * nu * nu;
    for (int j = 0; j < nu; ++j)
      for (int i = 0; i < nu; ++i) M_(Lg, nu, i, j) = M_(L, ld, i, j);
    double* K = w->K + (size_t)k * nu * nx;
    for (int j = 0; j < nx; ++j) {
      double col[32];
      for (int i = 0; i < nu; ++i) col[i] = M_(L, ld, nu + j, i);
      for (int i = nu - 1; i >= 0; --i) {
        double s = col[i];
        for (int l = i + 1; l < nu; ++l) s -= M_(L, ld, l, i) * col[l];
        const double dd = M_(L, ld, i, i);
        col[i] = dd > 0.0 ? s / dd : 0.0;
      }
      for (int i = 0; i < nu; ++i) M_(K, nu, i, j) = -col[i];
    }
  }
  return 0;
}
/* x := Lx^-1 x (the x block of a stage factor, ld ld, offset off); zero pivots give zero */
static void lx_solve(const double* L, int ld, int off, int nx, double* x) {
  for (int i = 0; i < nx; ++i) {
    double s = x[i];
    for (int l = 0; l < i; ++l) s -= M_(L, ld, off + i, off + l) * x[l];
    const double dd = M_(L, ld, off + i, off + i);
    x[i] = dd > 0.0 ? s / dd : 0.0;
  }
}
static void sqrt_vectors(const dims_t* d, ric_ws_t* w) {
  const int nx = d->nx, nu = d->nu, n = nx + nu, N = d->N;
  double* pN = w->p + (size_t)N * nx;
  memcpy(pN, w->gt + (size_t)N * w->gstride, sizeof(double) * nx);
  if (w->sform) lx_solve(sq_L(w, d, N), nx, 0, nx, pN);
  for (int k = N - 1; k >= 0; --k) {
    const double* A = qA(d, k);
    const double* B = qB(d, k);
    const double* Ln = sq_L(w, d, k + 1);
    const int nun = k + 1 < N ? nu : 0, ldn = nun + nx;
    const double* bt = w->bt + (size_t)k * nx;
    const double* pn = w->p + (size_t)(k + 1) * nx;
    const double* gt = w->gt + (size_t)k * w->gstride;
    double t[32], l_[64];
    for (int j = 0; j < nx; ++j) { /* Lx' b */
      double s = 0.0;
      for (int l = j; l < nx; ++l) s += M_(Ln, ldn, nun + l, nun + j) * bt[l];
      t[j] = s;
    }
    if (w->sform) {
      /* l = g + AL m, m = Lx' b + s, AL = [B'; A'] Lx */
      for (int j = 0; j < nx; ++j) t[j] += pn[j];
      for (int i = 0; i < n; ++i) {
        double acc = gt[i];
        for (int j = 0; j < nx; ++j) {
          double al = 0.0;
          for (int q = j; q < nx; ++q)
            al += (i < nu ? M_(B, nx, q, i) : M_(A, nx, q, i - nu)) * M_(Ln, ldn, nun + q, nun + j);
          acc += al * t[j];
        }
        l_[i] = acc;
      }
    } else {
      /* l = g + [B'; A'] (Lx (Lx' b) + p) */
      double tmp[32];
      for (int i = 0; i < nx; ++i) {
        double s = 0.0;
        for (int l = 0; l <= i; ++l) s += M_(Ln, ldn, nun + i, nun + l) * t[l];
        tmp[i] = s + pn[i];
      }
      mtv(nx, nu, B, tmp, l_);
      mtv(nx, nx, A, tmp, l_ + nu);
      for (int i = 0; i < n; ++i) l_[i] += gt[i];
    }
    const double* L = sq_L(w, d, k);
    double* y = w->yv + (size_t)k * nu;
    for (int i = 0; i < nu; ++i) {
      double s = l_[i];
      for (int q = 0; q < i; ++q) s -= M_(L, n, i, q) * y[q];
      const double dd = M_(L, n, i, i);
      y[i] = dd > 0.0 ? s / dd : 0.0;
    }
    double* pk = w->p + (size_t)k * nx;
    for (int i = 0; i < nx; ++i) {
      double s = l_[nu + i];
      for (int q = 0; q < nu; ++q) s -= M_(L, n, nu + i, q) * y[q];
      pk[i] = s;
    }
    if (w->sform) lx_solve(L, n, nu, nx, pk);
  }
}
static void sqrt_forward(const dims_t* d, const ric_ws_t* w, const double* xinit, double* x,
                         double* u, double* pi) {
  const int nx = d->nx, nu = d->nu, n = nx + nu, N = d->N;
  memcpy(x, xinit, sizeof(double) * nx);
  for (int k = 0; k < N; ++k) {
    const double* L = sq_L(w, d, k);
    const double* xk = x + (size_t)k * nx;
    double* uk = u + (size_t)k * nu;
    for (int i = 0; i < nu; ++i) { /* -(y + Lxu' x) */
      double s = w->yv[(size_t)k * nu + i];
      for (int l = 0; l < nx; ++l) s += M_(L, n, nu + l, i) * xk[l];
      uk[i] = -s;
    }
    for (int i = nu - 1; i >= 0; --i) { /* Lu^-T */
      double s = uk[i];
      for (int l = i + 1; l < nu; ++l) s -= M_(L, n, l, i) * uk[l];
      const double dd = M_(L, n, i, i);
      uk[i] = dd > 0.0 ? s / dd : 0.0;
    }
    double t1[32], t2[32];
    mv(nx, nx, qA(d, k), xk, t1);
    mv(nx, nu, qB(d, k), uk, t2);
    double* x1 = x + (size_t)(k + 1) * nx;
    for (int i = 0; i < nx; ++i) x1[i] = t1[i] + t2[i] + w->bt[(size_t)k * nx + i];
  }
  for (int k = 1; k <= N; ++k) {
    const double* L = sq_L(w, d, k);
    const int nuk = k < N ? nu : 0, ld = nuk + nx;
    const double* xk = x + (size_t)k * nx;
    const double* pk = w->p + (size_t)k * nx;
    double t[32];
    for (int j = 0; j < nx; ++j) { /* Lx' x (+ s) */
      double s = 0.0;
      for (int l = j; l < nx; ++l) s += M_(L, ld, nuk + l, nuk + j) * xk[l];
      t[j] = s + (w->sform ? pk[j] : 0.0);
    }
    for (int i = 0; i < nx; ++i) {
      double s = 0.0;
      for (int l = 0; l <= i; ++l) s += M_(L, ld, nuk + i, nuk + l) * t[l];
      pi[(size_t)k * nx + i] = s + (w->sform ? 0.0 : pk[i]);
    }
  }
}

/* LQ factorization with a positive diagonal of the n x m matrix M (column-major, ld n), in
 * place: afterwards the lower triangle of M[:, 0:n] holds L with M = L Q (Q orthogonal, not
 * formed).  One Householder reflection from the right per row maps row i's entries i..m-1 to
 * (||.||, 0, ..., 0): LAPACK's dgelqf with dlarfgp's positive beta, as HPIPM's dgelqf_pd
 * (restated: HPIPM / BLASFEO are not vendored).  A zero row stays zero.        */
static void lq_pd(int n, int m, double* M) {
  double v[512];
  for (int i = 0; i < n; ++i) {
    const double alpha = M_(M, n, i, i);
    double sigma = 0.0;
    for (int j = i + 1; j < m; ++j) sigma += M_(M, n, i, j) * M_(M, n, i, j);
    if (sigma == 0.0) {
      if (alpha < 0.0)
        for (int r = i; r < n; ++r) M_(M, n, r, i) = -M_(M, n, r, i);
      continue;
    }
    const double norm = sqrt(alpha * alpha + sigma);
    v[0] = alpha <= 0.0 ? alpha - norm : -sigma / (alpha + norm);
    for (int j = i + 1; j < m; ++j) v[j - i] = M_(M, n, i, j);
    const double vtv = v[0] * v[0] + sigma;
    for (int r = i; r < n; ++r) {
      double dot = 0.0;
      for (int j = i; j < m; ++j) dot += M_(M, n, r, j) * v[j - i];
      const double f = 2.0 * dot / vtv;
      for (int j = i; j < m; ++j) M_(M, n, r, j) -= f * v[j - i];
    }
    M_(M, n, i, i) = norm;
    for (int j = i + 1; j < m; ++j) M_(M, n, i, j) = 0.0;
  }
}

/* HPIPM's lq_fact factorization (d_ocp_qp_fact_lq_solve_kkt_step, hpipm_d_ocp_qp_kkt.h:58,
 * restated): the stage's barrier-augmented Hessian is never formed.  Stage k's factor
 * L_k = [Lu 0; Lxu Lx] ([u; x] order) is
 *   L_k = LQ([ chol(RSQ_k + Gamma_box + reg_u) | [B'; A'] Lx_{k+1} | sqrt(G_r) [D_r'; C_r'] ... ])
 * so L_k L_k' = RSQ_k + Gamma_k + reg + [B'; A'] P_{k+1} [B A] -- riccati_factor's matrix -- with
 * the dense terms (the cost-to-go and the general rows) entering as columns beside the data
 * instead of being added to it.  The columns are absorbed block by block (the cost-to-go, then
 * the general rows in chunks of 12 by row index), one positive-diagonal LQ (lq_pd) per block,
 * as the HIP library's riccati_step_lq does.  HPIPM keeps the box Gamma as a diagonal block
 * beside the Hessian factor (dgelqf_pd_lla); here, as on the GPU, it is added to the Hessian's
 * diagonal before its Cholesky (a diagonal addition cannot cancel).  The factor feeds the
 * square-root vector and forward routines (HPIPM's lq path solves with L exactly as the
 * Cholesky square root does); P, Lg, K are filled for the getters.                         */
static void fill_stage_H(const dims_t* d, int k, double* Ht, double* gt);
static int riccati_factor_lq(const dims_t* d, ric_ws_t* w, const stage_rows_t* st, double reg) {
  const int nx = d->nx, nu = d->nu, N = d->N, ng = d->ng;
  double* M = (double*)malloc(sizeof(double) * 64 * 128);
  double Hd[64 * 64], gdum[64], vrow[64];
  if (!M) return -1;
  w->sq = 1;
  for (int k = N; k >= 0; --k) {
    const int nu_k = st[k].nu_k, ns = nu_k + nx;
    fill_stage_H(d, k, Hd, gdum);
    for (int r = 0; r < st[k].nrow; ++r) {
      const row_t* rw = &st[k].rows[r];
      if (rw->kind == 0) M_(Hd, ns, rw->var, rw->var) += rw->G;
    }
    for (int j = 0; j < nu_k; ++j) M_(Hd, ns, j, j) += reg;
    chol(ns, Hd);
    for (int j = 0; j < ns; ++j)
      for (int i = 0; i < ns; ++i) M_(M, ns, i, j) = M_(Hd, ns, i, j);
    if (k < N) { /* the cost-to-go [B'; A'] Lx_{k+1} */
      const double* A = qA(d, k);
      const double* B = qB(d, k);
      const double* Ln = w->Lf + (size_t)(k + 1) * (size_t)d->n * d->n;
      const int nun = k + 1 < N ? nu : 0, ldn = nun + nx;
      for (int j = 0; j < nx; ++j) {
        for (int i = 0; i < nu; ++i) {
          double acc = 0.0;
          for (int l = j; l < nx; ++l) acc += M_(B, nx, l, i) * M_(Ln, ldn, nun + l, nun + j);
          M_(M, ns, i, ns + j) = acc;
        }
        for (int i = 0; i < nx; ++i) {
          double acc = 0.0;
          for (int l = j; l < nx; ++l) acc += M_(A, nx, l, i) * M_(Ln, ldn, nun + l, nun + j);
          M_(M, ns, nu + i, ns + j) = acc;
        }
      }
      lq_pd(ns, ns + nx, M);
    }
    for (int c0 = 0; c0 < ng; c0 += 12) { /* the general rows, 12 by row index */
      int m = ns;
      for (int r = 0; r < st[k].nrow; ++r) {
        const row_t* rw = &st[k].rows[r];
        if (rw->kind != 1 || rw->gidx < c0 || rw->gidx >= c0 + 12 || !(rw->G > 0.0)) continue;
        for (int i = 0; i < ns; ++i) vrow[i] = 0.0;
        row_axpy(d, rw, nu_k, sqrt(rw->G), vrow, vrow + nu_k);
        for (int i = 0; i < ns; ++i) M_(M, ns, i, m) = vrow[i];
        ++m;
      }
      if (m > ns) lq_pd(ns, m, M);
    }
    double* Lk = w->Lf + (size_t)k * (size_t)d->n * d->n;
    for (int j = 0; j < ns; ++j)
      for (int i = 0; i < ns; ++i) M_(Lk, ns, i, j) = i >= j ? M_(M, ns, i, j) : 0.0;
    double* P = w->P + (size_t)k * nx * nx;
    for (int j = 0; j < nx; ++j)
      for (int i = 0; i < nx; ++i) {
        double acc = 0.0;
        for (int l = 0; l < nx; ++l) acc += M_(Lk, ns, nu_k + i, nu_k + l) * M_(Lk, ns, nu_k + j, nu_k + l);
        M_(P, nx, i, j) = acc;
      }
    if (k == N) continue;
    double* L = w->Lg + (size_t)k * nu * nu;
    for (int j = 0; j < nu; ++j)
      for (int i = 0; i < nu; ++i) M_(L, nu, i, j) = M_(Lk, ns, i, j);
    double* K = w->K + (size_t)k * nu * nx;
    for (int j = 0; j < nx; ++j) { /* K[:, j] = -Lu^-T Lxu[j, :]' */
      double col[32];
      for (int i = 0; i < nu; ++i) col[i] = M_(Lk, ns, nu + j, i);
      for (int i = nu - 1; i >= 0; --i) {
        double sacc = col[i];
        for (int l = i + 1; l < nu; ++l) sacc -= M_(Lk, ns, l, i) * col[l];
        const double dd = M_(Lk, ns, i, i);
        col[i] = dd > 0.0 ? sacc / dd : 0.0;
      }
      for (int i = 0; i < nu; ++i) M_(K, nu, i, j) = -col[i];
    }
  }
  free(M);
  return 0;
}

/* p-vector recursion: p_N = gt_N; k_k = -G^-1 (r~ + B'(P b~ + p));
 * p_k = q~ + A'(P b~ + p) + K' (r~ + B'(P b~ + p)).                   */
static void riccati_vectors(const dims_t* d, ric_ws_t* w) {
  const int nx = d->nx, nu = d->nu, N = d->N;
  memcpy(w->p + (size_t)N * nx, w->gt + (size_t)N * w->gstride, sizeof(double) * nx);
  for (int k = N - 1; k >= 0; --k) {
    const double* A = qA(d, k);
    const double* B = qB(d, k);
    const double* P1 = w->P + (size_t)(k + 1) * nx * nx;
    const double* p1 = w->p + (size_t)(k + 1) * nx;
    const double* bt = w->bt + (size_t)k * nx;
    const double* gt = w->gt + (size_t)k * w->gstride;
    double Pb[32], g[32], f[32];
    mv(nx, nx, P1, bt, Pb);
    for (int i = 0; i < nx; ++i) Pb[i] += p1[i];
    mtv(nx, nu, B, Pb, g);
    for (int i = 0; i < nu; ++i) g[i] += gt[i];
    mtv(nx, nx, A, Pb, f);
    for (int i = 0; i < nx; ++i) f[i] += gt[nu + i];
    const double* K = w->K + (size_t)k * nu * nx;
    double* p = w->p + (size_t)k * nx;
    for (int j = 0; j < nx; ++j) {
      double s = f[j];
      for (int l = 0; l < nu; ++l) s += M_(K, nu, l, j) * g[l];
      p[j] = s;
    }
    double* kk = w->kk + (size_t)k * nu;
    memcpy(kk, g, sizeof(double) * nu);
    chol_solve(nu, w->Lg + (size_t)k * nu * nu, kk);
    for (int i = 0; i < nu; ++i) kk[i] = -kk[i];
  }
}

/* forward rollout from x_0 = xinit: u = K x + k, x+ = A x + B u + b~,
 * pi_k = P_k x_k + p_k for k >= 1 (pi_0 left to the caller).        */
static void riccati_forward(const dims_t* d, const ric_ws_t* w, const double* xinit,
                            double* x, double* u, double* pi) {
  const int nx = d->nx, nu = d->nu, N = d->N;
  memcpy(x, xinit, sizeof(double) * nx);
  for (int k = 0; k < N; ++k) {
    const double* xk = x + (size_t)k * nx;
    double* uk = u + (size_t)k * nu;
    mv(nu, nx, w->K + (size_t)k * nu * nx, xk, uk);
    for (int i = 0; i < nu; ++i) uk[i] += w->kk[(size_t)k * nu + i];
    double t1[32], t2[32];
    mv(nx, nx, qA(d, k), xk, t1);
    mv(nx, nu, qB(d, k), uk, t2);
    double* x1 = x + (size_t)(k + 1) * nx;
    for (int i = 0; i < nx; ++i) x1[i] = t1[i] + t2[i] + w->bt[(size_t)k * nx + i];
  }
  for (int k = 1; k <= N; ++k) {
    const double* xk = x + (size_t)k * nx;
    double* pk = pi + (size_t)k * nx;
    mv(nx, nx, w->P + (size_t)k * nx * nx, xk, pk);
    for (int i = 0; i < nx; ++i) pk[i] += w->p[(size_t)k * nx + i];
  }
}

/* stage Hessians / gradients of the original QP */
static void fill_stage_H(const dims_t* d, int k, double* Ht, double* gt) {
  const int nx = d->nx, nu = d->nu;
  if (k == d->N) {
    memcpy(Ht, qQ(d, k), sizeof(double) * nx * nx);
    memcpy(gt, qq(d, k), sizeof(double) * nx);
    return;
  }
  const int n = nx + nu;
  const double *R = qR(d, k), *S = qS(d, k), *Q = qQ(d, k);
  for (int j = 0; j < nu; ++j)
    for (int i = 0; i < nu; ++i) M_(Ht, n, i, j) = M_(R, nu, i, j);
  for (int j = 0; j < nx; ++j)
    for (int i = 0; i < nu; ++i) {
      M_(Ht, n, i, nu + j) = M_(S, nu, i, j);
      M_(Ht, n, nu + j, i) = M_(S, nu, i, j);
    }
  for (int j = 0; j < nx; ++j)
    for (int i = 0; i < nx; ++i) M_(Ht, n, nu + i, nu + j) = M_(Q, nx, i, j);
  memcpy(gt, qr(d, k), sizeof(double) * nu);
  memcpy(gt + nu, qq(d, k), sizeof(double) * nx);
}

/* The linear residual of the Newton system at the step (du, dx, dpi and the rows' dt, dlam), in
 * its full form: QP Hessian, the rows' multiplier steps, dynamics (HPIPM d_ocp_qp_res_compute_lin,
 * restated); the dt / dlam rows hold exactly by construction and are not formed.  Fills itg / itb
 * and returns the infinity norms of the stationarity and equality parts.                      */
static void lin_res(const dims_t* d, const stage_rows_t* st, const ric_ws_t* w, const double* rg,
                    const double* rb, const double* du, const double* dx, const double* dpi,
                    double* itg, double* itb, double* ng_out, double* nb_out) {
  const int nx = d->nx, nu = d->nu, N = d->N;
  double ng = 0.0, nb = 0.0;
  for (int s = 0; s <= N; ++s) {
    int nu_k = st[s].nu_k, ns = nu_k + nx;
    double H[64 * 64], gdum[64], v[64], r1[64];
    fill_stage_H(d, s, H, gdum);
    for (int i = 0; i < nu_k; ++i) v[i] = du[(size_t)s * nu + i];
    for (int i = 0; i < nx; ++i) v[nu_k + i] = dx[(size_t)s * nx + i];
    for (int i = 0; i < ns; ++i) {
      double acc = rg[(size_t)s * w->gstride + i];
      for (int j = 0; j < ns; ++j) acc += M_(H, ns, i, j) * v[j];
      r1[i] = acc;
    }
    for (int i = 0; i < st[s].nrow; ++i) {
      row_t* rw = &st[s].rows[i];
      double c = (rw->has_u ? rw->dlam_u : 0.0) - (rw->has_l ? rw->dlam_l : 0.0);
      row_axpy(d, rw, nu_k, c, r1, r1 + nu_k);
    }
    if (s < N) {
      double t[32];
      mtv(nx, nu, qB(d, s), dpi + (size_t)(s + 1) * nx, t);
      for (int i = 0; i < nu; ++i) r1[i] += t[i];
      mtv(nx, nx, qA(d, s), dpi + (size_t)(s + 1) * nx, t);
      for (int i = 0; i < nx; ++i) r1[nu_k + i] += t[i];
    }
    if (s > 0) for (int i = 0; i < nx; ++i) r1[nu_k + i] -= dpi[(size_t)s * nx + i];
    else for (int i = 0; i < nx; ++i) r1[nu_k + i] = 0.0;  /* x_0 fixed */
    for (int i = 0; i < ns; ++i) ng = fmax(ng, fabs(r1[i]));
    memcpy(itg + (size_t)s * w->gstride, r1, sizeof(double) * ns);
    if (s < N) {
      double t1[32], t2[32];
      mv(nx, nx, qA(d, s), dx + (size_t)s * nx, t1);
      mv(nx, nu, qB(d, s), du + (size_t)s * nu, t2);
      for (int i = 0; i < nx; ++i) {
        double rbi = rb[(size_t)s * nx + i] + t1[i] + t2[i] - dx[(size_t)(s + 1) * nx + i];
        itb[(size_t)s * nx + i] = rbi;
        nb = fmax(nb, fabs(rbi));
      }
    }
  }
  *ng_out = ng;
  *nb_out = nb;
}

/* ------------------------------------------------------------------ */
/* outputs: P, p, K, k, pi_0 (stage-0 rebuild, ocp_qp_ipm_solver.cpp:347-373) */
/* ------------------------------------------------------------------ */
static void write_outputs(const dims_t* d, const ric_ws_t* w, const double* x, const double* u,
                          double* pi, double* P, double* p, double* K, double* k) {
  const int nx = d->nx, nu = d->nu, N = d->N;
  /* p_k := pi_k - P_k x_k, k_k := u_k - K_k x_k (k >= 1); for an
   * unconstrained QP these are exactly the Riccati vectors.            */
  double pk_all[64 * 32];
  double* pp = (N + 1) * nx <= 64 * 32 ? pk_all : (double*)malloc(sizeof(double) * (N + 1) * nx);
  for (int s = 1; s <= N; ++s) {
    double Px[32];
    mv(nx, nx, w->P + (size_t)s * nx * nx, x + (size_t)s * nx, Px);
    for (int i = 0; i < nx; ++i) pp[(size_t)s * nx + i] = pi[(size_t)s * nx + i] - Px[i];
  }
  /* stage 0: k0 = u0 - K0 x0; p0 = q0 + A0'p1 + A0'P1 b0 + H0'k0; pi0 = p0 + P0 x0 */
  {
    const double* A0 = qA(d, 0);
    const double* B0 = qB(d, 0);
    const double* P1 = w->P + (size_t)1 * nx * nx;
    double k0[32], Kx[32];
    mv(nu, nx, w->K, x, Kx);
    for (int i = 0; i < nu; ++i) k0[i] = u[i] - Kx[i];
    double PA[32 * 32], H0[32 * 32];
    mm(nx, nx, nx, P1, A0, PA);
    mtm(nu, nx, nx, B0, PA, H0);
    const double* S0 = qS(d, 0);
    for (int j = 0; j < nx; ++j)
      for (int i = 0; i < nu; ++i) M_(H0, nu, i, j) += M_(S0, nu, i, j);
    double Pb[32], t[32];
    mv(nx, nx, P1, qb(d, 0), Pb);
    for (int i = 0; i < nx; ++i) Pb[i] += pp[(size_t)nx + i];
    mtv(nx, nx, A0, Pb, t);
    double t2[32];
    mtv(nu, nx, H0, k0, t2);
    const double* q0 = qq(d, 0);
    for (int i = 0; i < nx; ++i) pp[i] = q0[i] + t[i] + t2[i];
    double Px[32];
    mv(nx, nx, w->P, x, Px);
    for (int i = 0; i < nx; ++i) pi[i] = pp[i] + Px[i];
  }
  if (P) memcpy(P, w->P, sizeof(double) * (N + 1) * nx * nx);
  if (p) memcpy(p, pp, sizeof(double) * (N + 1) * nx);
  if (K) memcpy(K, w->K, sizeof(double) * N * nu * nx);
  if (k) {
    for (int s = 0; s < N; ++s) {
      double Kx[32];
      mv(nu, nx, w->K + (size_t)s * nu * nx, x + (size_t)s * nx, Kx);
      for (int i = 0; i < nu; ++i) k[(size_t)s * nu + i] = u[(size_t)s * nu + i] - Kx[i];
    }
  }
  if (pp != pk_all) free(pp);
}

/* ------------------------------------------------------------------ */
/* residuals at the current iterate                                    */
/* ------------------------------------------------------------------ */
static void compute_residuals(const dims_t* d, stage_rows_t* st, const double* x, const double* u,
                              const double* pi, double* rg, double* rb, double res[4],
                              double* obj, size_t gstride) {
  const int nx = d->nx, nu = d->nu, N = d->N;
  double rmax_g = 0.0, rmax_b = 0.0, rmax_d = 0.0, rmax_m = 0.0, ob = 0.0;
  for (int k = 0; k <= N; ++k) {
    const double* xk = x + (size_t)k * nx;
    const double* uk = u + (size_t)k * nu;
    double* gu = rg + (size_t)k * gstride;
    double* gx = gu + (k < N ? nu : 0);
    int nu_k = k < N ? nu : 0;
    if (k < N) {
      double t1[32], t2[32];
      mv(nu, nu, qR(d, k), uk, t1);
      mv(nu, nx, qS(d, k), xk, t2);
      for (int i = 0; i < nu; ++i) gu[i] = t1[i] + t2[i] + qr(d, k)[i];
      double o = 0.0;
      for (int i = 0; i < nu; ++i) o += uk[i] * (0.5 * t1[i] + qr(d, k)[i]);
      if (k == 0) for (int i = 0; i < nu; ++i) o += uk[i] * t2[i];
      ob += o;
      mtv(nx, nu, qB(d, k), pi + (size_t)(k + 1) * nx, t1);
      for (int i = 0; i < nu; ++i) gu[i] += t1[i];
    }
    {
      double t1[32], t2[32];
      mv(nx, nx, qQ(d, k), xk, t1);
      for (int i = 0; i < nx; ++i) gx[i] = t1[i] + qq(d, k)[i] - pi[(size_t)k * nx + i];
      if (k > 0) {
        double o = 0.0;
        for (int i = 0; i < nx; ++i) o += xk[i] * (0.5 * t1[i] + qq(d, k)[i]);
        if (k < N) { mv(nu, nx, qS(d, k), xk, t2); for (int i = 0; i < nu; ++i) o += uk[i] * t2[i]; }
        ob += o;
      }
      if (k < N) {
        mtv(nu, nx, qS(d, k), uk, t2);
        for (int i = 0; i < nx; ++i) gx[i] += t2[i];
        mtv(nx, nx, qA(d, k), pi + (size_t)(k + 1) * nx, t2);
        for (int i = 0; i < nx; ++i) gx[i] += t2[i];
      }
    }
    for (int i = 0; i < st[k].nrow; ++i) {
      row_t* rw = &st[k].rows[i];
      double val = row_dot(d, rw, nu_k, uk, xk);
      double c = (rw->has_l ? rw->lam_l : 0.0) - (rw->has_u ? rw->lam_u : 0.0);
      row_axpy(d, rw, nu_k, -c, gu, gx);
      if (rw->has_l) {
        rw->rd_l = val - rw->lb - rw->t_l;
        rw->rm_l = rw->lam_l * rw->t_l;
        if (fabs(rw->rd_l) > rmax_d) rmax_d = fabs(rw->rd_l);
        if (fabs(rw->rm_l) > rmax_m) rmax_m = fabs(rw->rm_l);
        if (isnan(rw->rd_l) || isnan(rw->rm_l)) rmax_d = NAN;
      }
      if (rw->has_u) {
        rw->rd_u = rw->ub - val - rw->t_u;
        rw->rm_u = rw->lam_u * rw->t_u;
        if (fabs(rw->rd_u) > rmax_d) rmax_d = fabs(rw->rd_u);
        if (fabs(rw->rm_u) > rmax_m) rmax_m = fabs(rw->rm_u);
        if (isnan(rw->rd_u) || isnan(rw->rm_u)) rmax_d = NAN;
      }
    }
    for (int i = 0; i < nu_k; ++i) { double a = fabs(gu[i]); if (a > rmax_g || isnan(a)) rmax_g = a; }
    if (k > 0) for (int i = 0; i < nx; ++i) { double a = fabs(gx[i]); if (a > rmax_g || isnan(a)) rmax_g = a; }
    if (k < N) {
      double t1[32], t2[32];
      mv(nx, nx, qA(d, k), xk, t1);
      mv(nx, nu, qB(d, k), uk, t2);
      double* rbk = rb + (size_t)k * nx;
      for (int i = 0; i < nx; ++i) {
        rbk[i] = t1[i] + t2[i] + qb(d, k)[i] - x[(size_t)(k + 1) * nx + i];
        double a = fabs(rbk[i]);
        if (a > rmax_b || isnan(a)) rmax_b = a;
      }
    }
  }
  res[0] = rmax_g; res[1] = rmax_b; res[2] = rmax_d; res[3] = rmax_m;
  if (obj) *obj = ob;
}

/* the factorization / vector / forward routines of the Riccati variant (ric_alg) */
static int factor(const dims_t* d, ric_ws_t* w, double reg, int ric_alg) {
  return ric_alg ? sqrt_factor(d, w, reg) : riccati_factor(d, w, reg);
}
static void vectors(const dims_t* d, ric_ws_t* w, int sform) {
  w->sform = sform;
  if (w->sq) sqrt_vectors(d, w); else riccati_vectors(d, w);
}
static void forward(const dims_t* d, const ric_ws_t* w, const double* xinit, double* x, double* u,
                    double* pi) {
  if (w->sq) sqrt_forward(d, w, xinit, x, u, pi); else riccati_forward(d, w, xinit, x, u, pi);
}

/* ------------------------------------------------------------------ */
/* main entry                                                          */
/* ------------------------------------------------------------------ */
int oracle_solve(const oracle_ocp_qp* qp, const oracle_settings* set, const double* x0,
                 double* x, double* u, double* pi, double* P, double* p, double* K,
                 double* k, oracle_result* res) {
  if (!qp || !set || !x0 || !x || !u || !pi || !res) return -1;
  if (qp->N < 1 || qp->nx < 1 || qp->nx > 32 || qp->nu < 1 || qp->nu > 31 || qp->ng < 0 || qp->ng > 64)
    return -2;
  dims_t d = {qp, qp->N, qp->nx, qp->nu, qp->ng, qp->nx + qp->nu};
  const int nx = d.nx, nu = d.nu, N = d.N, n = d.n;
  ric_ws_t w;
  w.hstride = (size_t)n * n;
  w.gstride = (size_t)n;
  w.Ht = (double*)calloc((size_t)(N + 1) * w.hstride, sizeof(double));
  w.gt = (double*)calloc((size_t)(N + 1) * w.gstride, sizeof(double));
  w.bt = (double*)calloc((size_t)N * nx, sizeof(double));
  w.P = (double*)calloc((size_t)(N + 1) * nx * nx, sizeof(double));
  w.p = (double*)calloc((size_t)(N + 1) * nx, sizeof(double));
  w.K = (double*)calloc((size_t)N * nu * nx, sizeof(double));
  w.kk = (double*)calloc((size_t)N * nu, sizeof(double));
  w.Lg = (double*)calloc((size_t)N * nu * nu, sizeof(double));
  w.Lf = (double*)calloc((size_t)(N + 1) * n * n, sizeof(double));
  w.yv = (double*)calloc((size_t)N * nu + 1, sizeof(double));
  w.sq = 0;
  w.sform = 0;
  double* rg = (double*)calloc((size_t)(N + 1) * w.gstride, sizeof(double));
  double* rb = (double*)calloc((size_t)N * nx, sizeof(double));
  double* dx = (double*)calloc((size_t)(N + 1) * nx, sizeof(double));
  double* du = (double*)calloc((size_t)N * nu + 1, sizeof(double));
  double* dpi = (double*)calloc((size_t)(N + 1) * nx, sizeof(double));
  double* zero = (double*)calloc((size_t)nx, sizeof(double));
  double* itg = (double*)calloc((size_t)(N + 1) * w.gstride, sizeof(double));
  double* itb = (double*)calloc((size_t)N * nx + 1, sizeof(double));
  double* cdx = (double*)calloc((size_t)(N + 1) * nx, sizeof(double));
  double* cdu = (double*)calloc((size_t)N * nu + 1, sizeof(double));
  double* cdpi = (double*)calloc((size_t)(N + 1) * nx, sizeof(double));
  int nc = 0;
  stage_rows_t* st = build_rows(&d, &nc);
  int rc = 0;
  memset(res, 0, sizeof(*res));

  if (nc == 0) {
    /* unconstrained: one Riccati factor + solve, iter = 0
     * (pinned by test/ocp_qp_ipm_solver.cpp:55-56)                   */
    for (int s = 0; s <= N; ++s) fill_stage_H(&d, s, w.Ht + s * w.hstride, w.gt + s * w.gstride);
    memcpy(w.bt, qp->b, sizeof(double) * N * nx);
    /* (d_ocp_qp_fact_solve_kkt_unconstr: the square root carries s = Lx^-1 p) */
    if (factor(&d, &w, set->reg_prim, set->ric_alg)) { res->status = 3; rc = 0; goto done_nan; }
    vectors(&d, &w, 1);
    forward(&d, &w, x0, x, u, pi);
    compute_residuals(&d, st, x, u, pi, rg, rb, res->res, &res->obj, w.gstride);
    write_outputs(&d, &w, x, u, pi, P, p, K, k);
    res->iter = 0;
    res->status = 0;
    for (int i = 0; i < 4; ++i) if (isnan(res->res[i])) res->status = 3;
    goto done;
  }

  /* ---------------- init (relative formulation, var_init_scheme 0) --- */
  if (!set->warm_start) {
    memset(u, 0, sizeof(double) * N * nu);
    memset(x, 0, sizeof(double) * (N + 1) * nx);
  }
  memcpy(x, x0, sizeof(double) * nx);
  memset(pi, 0, sizeof(double) * (N + 1) * nx);
  for (int s = 0; s <= N; ++s) {
    int nu_k = st[s].nu_k;
    double* us = u + (size_t)s * nu;
    double* xs = x + (size_t)s * nx;
    for (int i = 0; i < st[s].nrow; ++i) {
      row_t* rw = &st[s].rows[i];
      if (rw->kind == 0) {
        double* vp = rw->var < nu_k ? &us[rw->var] : &xs[rw->var - nu_k];
        double tl = *vp - rw->lb, tu = rw->ub - *vp;
        if (rw->has_l && rw->has_u) {
          if (tl < IPM_THR0) {
            if (tu < IPM_THR0) { *vp = 0.5 * (rw->lb + rw->ub); tl = tu = IPM_THR0; }
            else { tl = IPM_THR0; *vp = rw->lb + IPM_THR0; tu = rw->ub - *vp; }
          } else if (tu < IPM_THR0) { tu = IPM_THR0; *vp = rw->ub - IPM_THR0; tl = *vp - rw->lb; }
        } else if (rw->has_l) {
          if (tl < IPM_THR0) { tl = IPM_THR0; *vp = rw->lb + IPM_THR0; }
        } else if (tu < IPM_THR0) { tu = IPM_THR0; *vp = rw->ub - IPM_THR0; }
        rw->t_l = tl; rw->t_u = tu;
      }
    }
    for (int i = 0; i < st[s].nrow; ++i) {
      row_t* rw = &st[s].rows[i];
      if (rw->kind == 1) {
        double val = row_dot(&d, rw, nu_k, us, xs);
        rw->t_l = fmax(val - rw->lb, IPM_THR0);
        rw->t_u = fmax(rw->ub - val, IPM_THR0);
      }
      rw->lam_l = rw->has_l ? set->mu0 / rw->t_l : 0.0;
      rw->lam_u = rw->has_u ? set->mu0 / rw->t_u : 0.0;
    }
  }

  double alpha_prim = 1.0, alpha_dual = 1.0;
  int iter = 0;
  /* lq_fact applies to the square-root Riccati only ("for square_root_alg==1",
   * hpipm_d_ocp_qp_ipm.h:78); 1 switches for the rest of the solve */
  const int lqf = set->ric_alg ? set->lq_fact : 0;
  int force_lq = lqf == 2;
  for (;;) {
    compute_residuals(&d, st, x, u, pi, rg, rb, res->res, &res->obj, w.gstride);
    double mu = 0.0;
    for (int s = 0; s <= N; ++s)
      for (int i = 0; i < st[s].nrow; ++i) {
        row_t* rw = &st[s].rows[i];
        if (rw->has_l) mu += rw->rm_l;
        if (rw->has_u) mu += rw->rm_u;
      }
    mu /= (double)nc;
    int isn = 0;
    for (int i = 0; i < 4; ++i) if (isnan(res->res[i])) isn = 1;
    if (isnan(mu)) isn = 1;
    if (isn) { res->status = 3; break; }
    if (res->res[0] <= set->tol_stat && res->res[1] <= set->tol_eq &&
        res->res[2] <= set->tol_ineq && res->res[3] <= set->tol_comp) { res->status = 0; break; }
    if (iter >= set->iter_max) { res->status = 1; break; }
    if (iter > 0 && fmin(alpha_prim, alpha_dual) < set->alpha_min) { res->status = 2; break; }

    /* ---- predictor: Gamma = lam/t, gamma = (res_m + lam res_d)/t ---- */
    for (int s = 0; s <= N; ++s) {
      int nu_k = st[s].nu_k, ns = nu_k + nx;
      double* Ht = w.Ht + s * w.hstride;
      double* gt = w.gt + s * w.gstride;
      fill_stage_H(&d, s, Ht, gt);
      for (int i = 0; i < ns; ++i) gt[i] = rg[(size_t)s * w.gstride + i];
      for (int i = 0; i < st[s].nrow; ++i) {
        row_t* rw = &st[s].rows[i];
        double G = 0.0, gam = 0.0;
        if (rw->has_l) { G += rw->lam_l / rw->t_l; gam += (rw->rm_l + rw->lam_l * rw->rd_l) / rw->t_l; }
        if (rw->has_u) { G += rw->lam_u / rw->t_u; gam -= (rw->rm_u + rw->lam_u * rw->rd_u) / rw->t_u; }
        rw->G = G;
        row_syr(&d, rw, nu_k, G, Ht);
        row_axpy(&d, rw, nu_k, gam, gt, gt + nu_k);
      }
      if (s < N) memcpy(w.bt + (size_t)s * nx, rb + (size_t)s * nx, sizeof(double) * nx);
    }
    if (force_lq ? riccati_factor_lq(&d, &w, st, set->reg_prim)
                 : factor(&d, &w, set->reg_prim, set->ric_alg)) { res->status = 3; break; }
    /* predictor: d_ocp_qp_fact_solve_kkt_step (square root: s-form) */
    vectors(&d, &w, 1);
    forward(&d, &w, zero, dx, du, dpi);
#ifdef ORACLE_DEBUG
    {
      double tmin = 1e300, lmax = 0;
      for (int s = 0; s <= N; ++s)
        for (int i = 0; i < st[s].nrow; ++i) {
          row_t* rw = &st[s].rows[i];
          if (rw->has_l) { tmin = fmin(tmin, rw->t_l); lmax = fmax(lmax, rw->lam_l); }
          if (rw->has_u) { tmin = fmin(tmin, rw->t_u); lmax = fmax(lmax, rw->lam_u); }
        }
      fprintf(stderr, "it %d mu %.3e res %.3e %.3e %.3e %.3e ap %.3e ad %.3e tmin %.3e lmax %.3e\n", iter, mu,
              res->res[0], res->res[1], res->res[2], res->res[3], alpha_prim, alpha_dual, tmin, lmax);
    }
#endif

    double sigma_mu = 0.0;
    /* step on t / lam from dv */
#define STEP_TLAM()                                                                       \
    for (int s = 0; s <= N; ++s) {                                                        \
      int nu_k = st[s].nu_k;                                                              \
      for (int i = 0; i < st[s].nrow; ++i) {                                              \
        row_t* rw = &st[s].rows[i];                                                       \
        double dv = row_dot(&d, rw, nu_k, du + (size_t)s * nu, dx + (size_t)s * nx);      \
        if (rw->has_l) {                                                                  \
          rw->dt_l = rw->rd_l + dv;                                                       \
          rw->dlam_l = -(rw->rm_l - sigma_mu + rw->aff_l + rw->lam_l * rw->dt_l) / rw->t_l; \
        }                                                                                 \
        if (rw->has_u) {                                                                  \
          rw->dt_u = rw->rd_u - dv;                                                       \
          rw->dlam_u = -(rw->rm_u - sigma_mu + rw->aff_u + rw->lam_u * rw->dt_u) / rw->t_u; \
        }                                                                                 \
      }                                                                                   \
    }
    for (int s = 0; s <= N; ++s)
      for (int i = 0; i < st[s].nrow; ++i) { st[s].rows[i].aff_l = 0.0; st[s].rows[i].aff_u = 0.0; }
    STEP_TLAM();
    if (lqf == 1 && !force_lq) {
      /* HPIPM lq_fact 1: the predictor step's linear residual decides; above 1e-5 (or NaN) the
       * factorization is redone by LQ, and LQ stays for the rest of the solve */
      double ng = 0.0, nb = 0.0;
      lin_res(&d, st, &w, rg, rb, du, dx, dpi, itg, itb, &ng, &nb);
      if (!(ng <= 1e-5) || !(nb <= 1e-5)) {
        force_lq = 1;
        if (riccati_factor_lq(&d, &w, st, set->reg_prim)) { res->status = 3; break; }
        vectors(&d, &w, 1);
        forward(&d, &w, zero, dx, du, dpi);
        STEP_TLAM();
      }
    }
    res->lq_iters += force_lq;

    if (set->pred_corr) {
      /* alpha_aff, mu_aff, sigma = (mu_aff/mu)^3 */
      double ap = 1.0, ad = 1.0;
      for (int s = 0; s <= N; ++s)
        for (int i = 0; i < st[s].nrow; ++i) {
          row_t* rw = &st[s].rows[i];
          if (rw->has_l) {
            if (rw->dt_l < 0.0) ap = fmin(ap, -rw->t_l / rw->dt_l);
            if (rw->dlam_l < 0.0) ad = fmin(ad, -rw->lam_l / rw->dlam_l);
          }
          if (rw->has_u) {
            if (rw->dt_u < 0.0) ap = fmin(ap, -rw->t_u / rw->dt_u);
            if (rw->dlam_u < 0.0) ad = fmin(ad, -rw->lam_u / rw->dlam_u);
          }
        }
      double aa = fmin(ap, ad);
      double mu_aff = 0.0;
      for (int s = 0; s <= N; ++s)
        for (int i = 0; i < st[s].nrow; ++i) {
          row_t* rw = &st[s].rows[i];
          if (rw->has_l) mu_aff += (rw->lam_l + aa * rw->dlam_l) * (rw->t_l + aa * rw->dt_l);
          if (rw->has_u) mu_aff += (rw->lam_u + aa * rw->dlam_u) * (rw->t_u + aa * rw->dt_u);
        }
      mu_aff /= (double)nc;
      double sigma = mu_aff / mu;
      sigma = sigma * sigma * sigma;
      if (sigma > 1.0) sigma = 1.0;
      sigma_mu = sigma * mu;
      /* corrector: res_m <- lam t + dlam_aff dt_aff - sigma mu; same factors */
      for (int s = 0; s <= N; ++s) {
        int nu_k = st[s].nu_k, ns = nu_k + nx;
        double* gt = w.gt + s * w.gstride;
        for (int i = 0; i < ns; ++i) gt[i] = rg[(size_t)s * w.gstride + i];
        for (int i = 0; i < st[s].nrow; ++i) {
          row_t* rw = &st[s].rows[i];
          double gam = 0.0;
          if (rw->has_l) {
            rw->aff_l = rw->dlam_l * rw->dt_l;
            gam += (rw->rm_l + rw->aff_l - sigma_mu + rw->lam_l * rw->rd_l) / rw->t_l;
          }
          if (rw->has_u) {
            rw->aff_u = rw->dlam_u * rw->dt_u;
            gam -= (rw->rm_u + rw->aff_u - sigma_mu + rw->lam_u * rw->rd_u) / rw->t_u;
          }
          row_axpy(&d, rw, nu_k, gam, gt, gt + nu_k);
        }
      }
      /* corrector: d_ocp_qp_solve_kkt_step, same factors (square root: p-form) */
      vectors(&d, &w, 0);
      forward(&d, &w, zero, dx, du, dpi);
      STEP_TLAM();
    }
    /* iterative refinement of the final step (HPIPM itref_corr_max: Balance 2, Robust 4;
     * restated from HPIPM's d_ocp_qp_ipm_solve / d_ocp_qp_res_compute_lin, not vendored):
     * the linear residual of the Newton system at the step, in its full form (QP Hessian,
     * multiplier steps of the rows, dynamics); the dt / dlam rows hold exactly by
     * construction (STEP_TLAM), so they are not formed.  Each check stops the refinement
     * when the residual's infinity norms are below the tolerances (or below 1e-3 of the
     * first check's); otherwise the same factors solve for the correction, which is added.
     * ipm_box_impl.h kPhIR / kPhF3 restate the same for the HIP kernels.                */
    {
      double n0g = 0.0, n0b = 0.0;
      for (int ir = 0; ir < set->itref_corr_max; ++ir) {
        double ng = 0.0, nb = 0.0;
        lin_res(&d, st, &w, rg, rb, du, dx, dpi, itg, itb, &ng, &nb);
        if (ir == 0) { n0g = ng; n0b = nb; }
        if ((ng < set->tol_stat || ng < 1e-3 * n0g) && (nb < set->tol_eq || nb < 1e-3 * n0b)) break;
        /* correction: same factors, right-hand side = the residual */
        double* gkeep = w.gt; double* bkeep = w.bt;
        w.gt = itg; w.bt = itb;
        vectors(&d, &w, 0);
        forward(&d, &w, zero, cdx, cdu, cdpi);
        w.gt = gkeep; w.bt = bkeep;
        for (size_t i = 0; i < (size_t)(N + 1) * nx; ++i) { dx[i] += cdx[i]; if (i >= (size_t)nx) dpi[i] += cdpi[i]; }
        for (size_t i = 0; i < (size_t)N * nu; ++i) du[i] += cdu[i];
        STEP_TLAM();
      }
    }
#undef STEP_TLAM

    /* step lengths (fraction to boundary) */
    /* fraction to the boundary: alpha = min(1, tau * alpha_max), alpha_max
     * uncapped, so a step never lands exactly on t = 0 or lam = 0.        */
    double ap = 1e300, ad = 1e300;
    for (int s = 0; s <= N; ++s)
      for (int i = 0; i < st[s].nrow; ++i) {
        row_t* rw = &st[s].rows[i];
        if (rw->has_l) {
          if (rw->dt_l < 0.0) ap = fmin(ap, -rw->t_l / rw->dt_l);
          if (rw->dlam_l < 0.0) ad = fmin(ad, -rw->lam_l / rw->dlam_l);
        }
        if (rw->has_u) {
          if (rw->dt_u < 0.0) ap = fmin(ap, -rw->t_u / rw->dt_u);
          if (rw->dlam_u < 0.0) ad = fmin(ad, -rw->lam_u / rw->dlam_u);
        }
      }
    if (!set->split_step) { ap = fmin(ap, ad); ad = ap; }
    ap = fmin(1.0, IPM_STEP_TAU * ap);
    ad = fmin(1.0, IPM_STEP_TAU * ad);
    /* a step with a NaN component, or one too large to square (a factorization
     * that broke down), is not a direction: no step, and the next exit test
     * stops with MinStepLengthReached (the HIP kernel's rule, ipm_box_impl.h) */
    {
      int bad = 0;
#define HUGE_STEP(v) (!(fabs(v) < 1.3e150))
      for (int s = 0; s <= N; ++s) {
        for (int i = 0; i < nx; ++i)
          bad |= HUGE_STEP(dx[(size_t)s * nx + i]) | HUGE_STEP(dpi[(size_t)s * nx + i]);
        if (s < N)
          for (int i = 0; i < nu; ++i) bad |= HUGE_STEP(du[(size_t)s * nu + i]);
        for (int i = 0; i < st[s].nrow; ++i) {
          row_t* rw = &st[s].rows[i];
          if (rw->has_l) bad |= HUGE_STEP(rw->dt_l) | HUGE_STEP(rw->dlam_l);
          if (rw->has_u) bad |= HUGE_STEP(rw->dt_u) | HUGE_STEP(rw->dlam_u);
        }
      }
#undef HUGE_STEP
      if (bad) ap = ad = 0.0;
    }
    alpha_prim = ap; alpha_dual = ad;
    if (ap == 0.0 && ad == 0.0) { ++iter; continue; }
    /* update */
    for (int s = 1; s <= N; ++s)
      for (int i = 0; i < nx; ++i) x[(size_t)s * nx + i] += ap * dx[(size_t)s * nx + i];
    for (int s = 0; s < N; ++s)
      for (int i = 0; i < nu; ++i) u[(size_t)s * nu + i] += ap * du[(size_t)s * nu + i];
    for (int s = 1; s <= N; ++s)
      for (int i = 0; i < nx; ++i) pi[(size_t)s * nx + i] += ad * dpi[(size_t)s * nx + i];
    for (int s = 0; s <= N; ++s)
      for (int i = 0; i < st[s].nrow; ++i) {
        row_t* rw = &st[s].rows[i];
        if (rw->has_l) { rw->t_l += ap * rw->dt_l; rw->lam_l += ad * rw->dlam_l; }
        if (rw->has_u) { rw->t_u += ap * rw->dt_u; rw->lam_u += ad * rw->dlam_u; }
      }
    ++iter;
  }
  res->iter = iter;

  /* Riccati outputs (P, K) are those of the last factorization performed by
   * the IPM (the last step's barrier-augmented KKT system), as HPIPM's
   * d_ocp_qp_ipm_get_ric_* getters return (ocp_qp_ipm_solver.cpp:342-350);
   * vectors by consistency (write_outputs).  With no step taken (converged
   * at the initial point) the system is factorized at the returned iterate. */
  if (iter == 0 && res->status != 3) {
    for (int s = 0; s <= N; ++s) {
      int nu_k = st[s].nu_k;
      double* Ht = w.Ht + s * w.hstride;
      double* gt = w.gt + s * w.gstride;
      fill_stage_H(&d, s, Ht, gt);
      for (int i = 0; i < st[s].nrow; ++i) {
        row_t* rw = &st[s].rows[i];
        double G = 0.0;
        if (rw->has_l) G += rw->lam_l / rw->t_l;
        if (rw->has_u) G += rw->lam_u / rw->t_u;
        row_syr(&d, rw, nu_k, G, Ht);
      }
    }
    if (lqf == 2) {
      for (int s = 0; s <= N; ++s)
        for (int i = 0; i < st[s].nrow; ++i) {
          row_t* rw = &st[s].rows[i];
          rw->G = (rw->has_l ? rw->lam_l / rw->t_l : 0.0) + (rw->has_u ? rw->lam_u / rw->t_u : 0.0);
        }
      if (riccati_factor_lq(&d, &w, st, set->reg_prim) != 0) res->status = 3;
    } else if (factor(&d, &w, set->reg_prim, set->ric_alg) != 0) {
      res->status = 3;
    }
  }
  write_outputs(&d, &w, x, u, pi, P, p, K, k);
  goto done;

done_nan:
  res->iter = 0;
done:
  free_rows(&d, st);
  free(w.Ht); free(w.gt); free(w.bt); free(w.P); free(w.p); free(w.K); free(w.kk); free(w.Lg);
  free(w.Lf); free(w.yv);
  free(rg); free(rb); free(dx); free(du); free(dpi); free(zero);
  free(itg); free(itb); free(cdx); free(cdu); free(cdpi);
  return rc;
}

/* ------------------------------------------------------------------ */
/* threaded batch (cpu_baseline)                                        */
/* ------------------------------------------------------------------ */
typedef struct {
  int lo, hi;
  const oracle_ocp_qp* qp0;
  const oracle_settings* st;
  const double* x0;
  double *x, *u, *pi;
  int *status, *iters;
} job_t;

static const double* adv(const double* p, size_t per, int i) { return p ? p + per * (size_t)i : NULL; }

static void* batch_worker(void* arg) {
  job_t* j = (job_t*)arg;
  const oracle_ocp_qp* q = j->qp0;
  const int N = q->N, nx = q->nx, nu = q->nu, ng = q->ng;
  for (int i = j->lo; i < j->hi; ++i) {
    oracle_ocp_qp qi = *q;
    qi.A = adv(q->A, (size_t)N * nx * nx, i);
    qi.B = adv(q->B, (size_t)N * nx * nu, i);
    qi.b = adv(q->b, (size_t)N * nx, i);
    qi.Q = adv(q->Q, (size_t)(N + 1) * nx * nx, i);
    qi.S = adv(q->S, (size_t)N * nu * nx, i);
    qi.R = adv(q->R, (size_t)N * nu * nu, i);
    qi.q = adv(q->q, (size_t)(N + 1) * nx, i);
    qi.r = adv(q->r, (size_t)N * nu, i);
    qi.lbu = adv(q->lbu, (size_t)N * nu, i); qi.ubu = adv(q->ubu, (size_t)N * nu, i);
    qi.lbu_mask = adv(q->lbu_mask, (size_t)N * nu, i); qi.ubu_mask = adv(q->ubu_mask, (size_t)N * nu, i);
    qi.lbx = adv(q->lbx, (size_t)(N + 1) * nx, i); qi.ubx = adv(q->ubx, (size_t)(N + 1) * nx, i);
    qi.lbx_mask = adv(q->lbx_mask, (size_t)(N + 1) * nx, i); qi.ubx_mask = adv(q->ubx_mask, (size_t)(N + 1) * nx, i);
    qi.C = adv(q->C, (size_t)(N + 1) * ng * nx, i);
    qi.D = adv(q->D, (size_t)N * ng * nu, i);
    qi.lg = adv(q->lg, (size_t)(N + 1) * ng, i); qi.ug = adv(q->ug, (size_t)(N + 1) * ng, i);
    qi.lg_mask = adv(q->lg_mask, (size_t)(N + 1) * ng, i); qi.ug_mask = adv(q->ug_mask, (size_t)(N + 1) * ng, i);
    oracle_result r;
    oracle_solve(&qi, j->st, j->x0 + (size_t)i * nx, j->x + (size_t)i * (N + 1) * nx,
                 j->u + (size_t)i * N * nu, j->pi + (size_t)i * (N + 1) * nx, NULL, NULL, NULL,
                 NULL, &r);
    if (j->status) j->status[i] = r.status;
    if (j->iters) j->iters[i] = r.iter;
  }
  return NULL;
}

int oracle_solve_batch(int batch, const oracle_ocp_qp* qp0, const oracle_settings* st,
                       const double* x0, double* x, double* u, double* pi, int* status,
                       int* iters, int threads) {
  if (threads < 1) threads = 1;
  if (threads > batch) threads = batch > 0 ? batch : 1;
  pthread_t th[256];
  job_t jobs[256];
  if (threads > 256) threads = 256;
  for (int t = 0; t < threads; ++t) {
    jobs[t].lo = (int)((long)batch * t / threads);
    jobs[t].hi = (int)((long)batch * (t + 1) / threads);
    jobs[t].qp0 = qp0; jobs[t].st = st; jobs[t].x0 = x0;
    jobs[t].x = x; jobs[t].u = u; jobs[t].pi = pi; jobs[t].status = status; jobs[t].iters = iters;
    pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  return 0;
}
