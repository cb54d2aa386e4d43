// mfma_lat.h -- fp64 matrix-core pieces of the single-QP (latency) kernels: the unconstrained
// solve (riccati_latency_impl.h) and the IPM (ipm_latency.hip).
//
// A 12 x 12 block with its vector column (13 columns) is held in the C/D layout of
// v_mfma_f64_16x16x4_f64: lane l = (g = l >> 4, c = l & 15) register r holds M[g + 4 r][c]
// (rows >= 12, columns >= 13: zero or unused).  That layout is the B operand of the next
// product (k-block kb: lane (g, c) supplies M[4 kb + g][c] = register kb) and, for a symmetric
// M, its A operand, so P B, B'(P B), ... chain in registers.
#pragma once

#include "qp_group.h"
#include "riccati.h"

namespace srbd {

typedef double lat_d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ lat_d4 lat_mfma(double a, double b, lat_d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// An opaque copy of an index: the resident server (riccati_latency_impl.h) runs the solve in a
// loop, and the compiler would otherwise hoist the solve's address arithmetic out of it and
// keep it live across the whole solve (620 B/lane of scratch).
__device__ __forceinline__ int lat_opq(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// 1 / d by v_rcp_f64 and two Newton steps (3 dependent FMAs instead of the IEEE division's
// ~10 instructions on the stage's critical path)
__device__ __forceinline__ double lat_recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  return r;
}

// Column-owned Cholesky (riccati.h chol_cols; pivots by lat_recip, or IEEE division with IEEE
// set, as chol_cols divides -- the IPM's endgame is sensitive to the last bits):
// `reg` on each pivot, a
// non-positive pivot zeroes its column (BLASFEO dpotrf_l).  `hook(ic<K>)` runs at the top of
// pivot K: the caller issues its independent matrix-core work there, one MFMA per pivot, so the
// MFMA pipe runs beside the pivots' VALU chain instead of ahead of it (a wave cannot issue past
// an MFMA the pipe has not accepted).
template <bool IEEE = false, typename Hook>
__device__ __forceinline__ void lat_chol(double (&G)[12], const int lane, const double reg, double (&Lc)[12],
                                         double& rs, Hook&& hook) {
  double dmine = 1.0;
  sfor<0, 12>([&](auto kk) {
    constexpr int K = decltype(kk)::value;
    hook(kk);
    const double dk = bc<K>(G[K]) + reg;
    const double inv = dk > 0.0 ? (IEEE ? 1.0 / dk : lat_recip(dk)) : 0.0;
    const double s = lane > K ? G[K] * inv : 0.0;
    sfor<K + 1, 12>([&](auto i) {
      constexpr int I = decltype(i)::value;
      G[I] = fmadd(-bc<K>(G[I]), s, G[I]);
    });
    dmine = lane == K ? dk : dmine;
  });
  double inv_l;
  pivot_rs(dmine, rs, inv_l);
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    Lc[I] = G[I] * inv_l;
  });
}

}  // namespace srbd
