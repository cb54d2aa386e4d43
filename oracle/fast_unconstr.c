/* fast_unconstr.c -- the CPU baseline of the unconstrained batched solve (bench.py
 * cpu_baseline, kind "port").
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY, like the rest of oracle/: bench.py's
 * cpu_baseline leg and tests/test_oracle.py load it; the product library never does.
 *
 * The same algorithm as the oracle's nc = 0 path (ocp_qp_oracle.c riccati_factor /
 * riccati_vectors / riccati_forward, classical Riccati = HPIPM's
 * d_ocp_qp_fact_solve_kkt_unconstr, hpipm_d_ocp_qp_kkt.h:54, pinned by
 * hpipm-cpp/test/ocp_qp_ipm_solver.cpp:60-90) specialised to the SRBD sizes nx = nu = 12:
 * fixed-size 12 x 12 blocks whose inner loops run over 12 contiguous doubles (three AVX2
 * vectors at -march=x86-64-v3), one QP per thread at a time, no allocation inside the
 * solve.  It computes what the GPU benchmark times -- x, u, pi -- and nothing else (no
 * residuals), so the two rates compare the same work.  It is the stronger of the two CPU
 * baselines (the generic oracle is ~5x slower); HPIPM + BLASFEO itself is not buildable in
 * this image.
 *
 * Layouts as the C-ABI's QP-major default (include/srbd_qp.h): per QP, stage-major,
 * column-major 12 x 12 blocks, M[i][j] = M[i + 12 j]. */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define D 12
#define DD 144

/* C = A B (all column-major 12 x 12): column j of C accumulates A's columns */
static inline void mm(const double* restrict A, const double* restrict B, double* restrict C) {
  for (int j = 0; j < D; ++j) {
    double c[D] = {0};
    for (int k = 0; k < D; ++k) {
      const double b = B[k + D * j];
      for (int i = 0; i < D; ++i) c[i] += A[i + D * k] * b;
    }
    memcpy(C + D * j, c, sizeof c);
  }
}

/* C += At B with At = A' given explicitly (column-major) */
static inline void mm_acc(const double* restrict At, const double* restrict B, double* restrict C) {
  for (int j = 0; j < D; ++j) {
    double c[D];
    memcpy(c, C + D * j, sizeof c);
    for (int k = 0; k < D; ++k) {
      const double b = B[k + D * j];
      for (int i = 0; i < D; ++i) c[i] += At[i + D * k] * b;
    }
    memcpy(C + D * j, c, sizeof c);
  }
}

static inline void transpose(const double* restrict A, double* restrict At) {
  for (int j = 0; j < D; ++j)
    for (int i = 0; i < D; ++i) At[j + D * i] = A[i + D * j];
}

/* y = M v (+ y0) */
static inline void mv(const double* restrict M, const double* restrict v, const double* y0,
                      double* restrict y) {
  double c[D];
  if (y0) memcpy(c, y0, sizeof c); else memset(c, 0, sizeof c);
  for (int k = 0; k < D; ++k) {
    const double b = v[k];
    for (int i = 0; i < D; ++i) c[i] += M[i + D * k] * b;
  }
  memcpy(y, c, sizeof c);
}

/* Cholesky of the column-major SPD G in place (lower); a non-positive pivot zeroes its
 * column, as BLASFEO's dpotrf_l and the oracle's chol do.  inv[j] = 1 / L[j][j] (0 there). */
static inline void chol(double* restrict G, double* restrict inv) {
  for (int j = 0; j < D; ++j) {
    double* cj = G + D * j;
    for (int k = 0; k < j; ++k) {
      const double l = G[j + D * k];
      const double* ck = G + D * k;
      for (int i = j; i < D; ++i) cj[i] -= ck[i] * l;
    }
    const double d = cj[j];
    const double s = d > 0.0 ? sqrt(d) : 0.0;
    const double r = d > 0.0 ? 1.0 / s : 0.0;
    inv[j] = r;
    for (int i = j; i < D; ++i) cj[i] *= r;
  }
}

/* X <- -G^-1 X for the 12 right-hand sides held as the rows of Xr (row-major: Xr[i][c] =
 * X[i][c], so each substitution step updates 12 contiguous values) */
static inline void chol_solve_neg_rows(const double* restrict L, const double* restrict inv,
                                       double* restrict Xr, int ncols) {
  for (int i = 0; i < D; ++i) { /* L y = x */
    double* xi = Xr + ncols * i;
    for (int k = 0; k < i; ++k) {
      const double l = L[i + D * k];
      const double* xk = Xr + ncols * k;
      for (int c = 0; c < ncols; ++c) xi[c] -= l * xk[c];
    }
    for (int c = 0; c < ncols; ++c) xi[c] *= inv[i];
  }
  for (int i = D - 1; i >= 0; --i) { /* L' z = y */
    double* xi = Xr + ncols * i;
    for (int k = i + 1; k < D; ++k) {
      const double l = L[k + D * i];
      const double* xk = Xr + ncols * k;
      for (int c = 0; c < ncols; ++c) xi[c] -= l * xk[c];
    }
    for (int c = 0; c < ncols; ++c) xi[c] *= inv[i];
  }
  for (int i = 0; i < D * ncols; ++i) Xr[i] = -Xr[i];
}

typedef struct {
  double K[DD], k[D], P[DD], p[D];
} stage_t;

/* one QP: N stages, pointers to its blocks (QP-major, stage-major) */
static void solve_one(int N, const double* A, const double* B, const double* b, const double* Q,
                      const double* S, const double* R, const double* q, const double* r,
                      const double* x0, double reg, stage_t* st, double* x, double* u, double* pi) {
  double P[DD], p[D];
  memcpy(P, Q + (size_t)N * DD, sizeof P);
  memcpy(p, q + (size_t)N * D, sizeof p);
  memcpy(st[N].P, P, sizeof P);
  memcpy(st[N].p, p, sizeof p);
  for (int kk = N - 1; kk >= 0; --kk) {
    const double *Ak = A + (size_t)kk * DD, *Bk = B + (size_t)kk * DD, *bk = b + (size_t)kk * D;
    double At[DD], Bt[DD], WA[DD], WB[DD], w[D], G[DD], H[DD], F[DD], g[D], f[D], inv[D];
    transpose(Ak, At);
    transpose(Bk, Bt);
    mm(P, Ak, WA);
    mm(P, Bk, WB);
    mv(P, bk, p, w); /* w = P b + p */
    memcpy(G, R + (size_t)kk * DD, sizeof G);
    memcpy(H, S + (size_t)kk * DD, sizeof H);
    memcpy(F, Q + (size_t)kk * DD, sizeof F);
    mm_acc(Bt, WB, G);
    mm_acc(Bt, WA, H);
    mm_acc(At, WA, F);
    mv(Bt, w, r + (size_t)kk * D, g);
    mv(At, w, q + (size_t)kk * D, f);
    for (int i = 0; i < D; ++i) G[i + D * i] += reg;
    chol(G, inv);
    /* [K | k] = -G^-1 [H | g], as rows: row i = (H[i][0..11], g[i]) */
    double Xr[D * (D + 1)];
    for (int i = 0; i < D; ++i) {
      for (int c = 0; c < D; ++c) Xr[(D + 1) * i + c] = H[i + D * c];
      Xr[(D + 1) * i + D] = g[i];
    }
    chol_solve_neg_rows(G, inv, Xr, D + 1);
    stage_t* s = st + kk;
    for (int i = 0; i < D; ++i) {
      for (int c = 0; c < D; ++c) s->K[i + D * c] = Xr[(D + 1) * i + c];
      s->k[i] = Xr[(D + 1) * i + D];
    }
    /* P = F + H' K, p = f + H' k */
    double Ht[DD];
    transpose(H, Ht);
    mm_acc(Ht, s->K, F);
    mv(Ht, s->k, f, p);
    memcpy(P, F, sizeof P);
    memcpy(s->P, P, sizeof P);
    memcpy(s->p, p, sizeof p);
  }
  double xk[D];
  memcpy(xk, x0, sizeof xk);
  for (int kk = 0; kk <= N; ++kk) {
    memcpy(x + (size_t)kk * D, xk, sizeof xk);
    mv(st[kk].P, xk, st[kk].p, pi + (size_t)kk * D);
    if (kk == N) break;
    double uk[D], xn[D], bu[D];
    mv(st[kk].K, xk, st[kk].k, uk);
    memcpy(u + (size_t)kk * D, uk, sizeof uk);
    mv(A + (size_t)kk * DD, xk, b + (size_t)kk * D, xn);
    mv(B + (size_t)kk * DD, uk, xn, bu);
    memcpy(xk, bu, sizeof xk);
  }
}

typedef struct {
  int N, lo, hi;
  const double *A, *B, *b, *Q, *S, *R, *q, *r, *x0;
  double reg;
  double *x, *u, *pi;
} job_t;

static void* worker(void* arg) {
  const job_t* j = (const job_t*)arg;
  const int N = j->N;
  stage_t* st = (stage_t*)malloc(sizeof(stage_t) * (size_t)(N + 1));
  if (!st) return NULL;
  for (int i = j->lo; i < j->hi; ++i) {
    const size_t s = (size_t)i * N, s1 = (size_t)i * (N + 1);
    solve_one(N, j->A + s * DD, j->B + s * DD, j->b + s * D, j->Q + s1 * DD, j->S + s * DD,
              j->R + s * DD, j->q + s1 * D, j->r + s * D, j->x0 + (size_t)i * D, j->reg, st,
              j->x + s1 * D, j->u + s * D, j->pi + s1 * D);
  }
  free(st);
  return NULL;
}

/* batch QPs (nx = nu = 12) over `threads` threads; returns 0 (or -1 on a thread error) */
int fast_unconstr_solve_batch(int batch, int N, const double* A, const double* B, const double* b,
                              const double* Q, const double* S, const double* R, const double* q,
                              const double* r, const double* x0, double reg, double* x, double* u,
                              double* pi, int threads) {
  if (threads < 1) threads = 1;
  if (threads > batch) threads = batch > 0 ? batch : 1;
  pthread_t tid[256];
  job_t job[256];
  if (threads > 256) threads = 256;
  int err = 0;
  for (int t = 0; t < threads; ++t) {
    job_t jb = {N, (int)((long long)batch * t / threads), (int)((long long)batch * (t + 1) / threads),
                A, B, b, Q, S, R, q, r, x0, reg, x, u, pi};
    job[t] = jb;
    if (pthread_create(&tid[t], NULL, worker, &job[t]) != 0) {
      worker(&job[t]);
      tid[t] = 0;
    }
  }
  for (int t = 0; t < threads; ++t)
    if (tid[t] && pthread_join(tid[t], NULL) != 0) err = -1;
  return err;
}
