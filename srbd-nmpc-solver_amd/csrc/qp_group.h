// qp_group.h -- the 16-lane "QP group" execution model used by every kernel.
//
// One OCP-QP is owned by one DPP row (16 consecutive lanes of a 64-lane
// wavefront), so a wavefront advances four QPs in lockstep and a 256-thread
// workgroup sixteen.  Inside a group, lane j < 12 owns column j of every
// 12x12 stage block (the QP's matrices are stored column-major, so a lane's
// column is 96 contiguous bytes) and lane 15 (VL) owns the vector column
// (b / r / q / p ...).  Lanes 12..14 idle.
//
// Cross-lane traffic is a broadcast of one lane's register to its whole
// row: gfx950's DPP row_newbcast, which hipcc emits as v_mov_b64_dpp for
// __builtin_amdgcn_update_dpp(..., 0x150 + src, ...).  With the source lane
// and the register index both compile-time constants, every product the
// Riccati recursion needs becomes a chain of broadcast + FMA with no LDS and
// no bank conflicts:
//   C = X  Y   (X symmetric, Y column-owned):  C[:,j] += bc<k>(X[i]) * Y[k]
//   C = X' Y   (both column-owned):            C[i][j] += bc<i>(X[k]) * Y[k]
//   y = M  v   (M row-owned, v element-owned): y[i]   += M[j] * bc<j>(v)
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

namespace srbd {

constexpr int kMaxDim = 12;   // nx, nu handled in registers
constexpr int kGroup = 16;    // lanes per QP (one DPP row)
constexpr int kVecLane = 15;  // lane holding the vector column

template <int I>
using ic = std::integral_constant<int, I>;

// compile-time loop: f(ic<B>), f(ic<B+1>), ..., f(ic<E-1>)
template <int B, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(ic<B>{});
    sfor<B + 1, E>(static_cast<F&&>(f));
  }
}
// descending: f(ic<E-1>), ..., f(ic<B>)
template <int B, int E, typename F>
__device__ __forceinline__ void sfor_down(F&& f) {
  if constexpr (B < E) {
    f(ic<E - 1>{});
    sfor_down<B, E - 1>(static_cast<F&&>(f));
  }
}

// Broadcast lane SRC of this lane's 16-lane row (DPP row_newbcast:SRC).
template <int SRC>
__device__ __forceinline__ double bc(double v) {
  static_assert(SRC >= 0 && SRC < kGroup, "row_newbcast source lane");
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + SRC, 0xf, 0xf, true);
}

template <int SRC>
__device__ __forceinline__ float bc(float v) {
  static_assert(SRC >= 0 && SRC < kGroup, "row_newbcast source lane");
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150 + SRC, 0xf, 0xf, true));
}

// The group's lanes exchange data through LDS inside one wave: LDS executes a
// wave's instructions in order, so only the compiler must not move the reads
// above the writes (a compiler-only barrier: no wait on outstanding global loads).
__device__ __forceinline__ void lds_wave_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Opaque copy: the compiler can no longer prove the values equal to the
// originals, so broadcasts of the laundered array are not CSE'd with earlier
// broadcasts of the same registers (which would keep 144 broadcast values
// live across phases and spill).
template <typename T>
__device__ __forceinline__ void opaque(T& x) {
  asm volatile("" : "+v"(x));
}
template <typename T, int... Is>
__device__ __forceinline__ void launder_impl(T (&v)[12], std::integer_sequence<int, Is...>) {
  (opaque(v[Is]), ...);
}
template <typename T>
__device__ __forceinline__ void launder(T (&v)[12]) {
  launder_impl(v, std::make_integer_sequence<int, 12>{});
}

// ---------------------------------------------------------------------------
// Fused broadcast-FMA blocks: v_fmac_f64_dpp with row_newbcast, i.e. the
// broadcast rides on the FMA's src0 operand for free (hipcc does not combine
// v_mov_b64_dpp into v_fmac_f64 by itself).  Each block is one asm statement
// of 12 independent FMAs led by `s_nop 1`: the 2 wait states a DPP read needs
// after a VALU write of its source VGPR (the only hazard here -- inside a
// block no DPP source is written).
//
//   fma_bcast_src<S>(C, X, y):   C[i] += bc<S>(X[i]) * y     (i = 0..11)
//   fma_bcast_lane(C, x, Y):     C[i] += bc<i>(x)    * y_i   -> see below
// ---------------------------------------------------------------------------
#define SRBD_FMAC_DPP(D, S0, S1, LANE) "v_fmac_f64_dpp " D ", " S0 ", " S1 " row_newbcast:" #LANE " row_mask:0xf bank_mask:0xf\n\t"

// C[i] += bc<SRC>(X[i]) * y for i = 0..11
template <int SRC>
__device__ __forceinline__ void fma_bcast_src(double (&C)[12], const double (&X)[12], double y) {
  static_assert(SRC >= 0 && SRC < kGroup, "row_newbcast source lane");
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %12, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %13, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, %14, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, %15, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, %16, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, %17, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %6, %18, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %7, %19, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %8, %20, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %9, %21, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %10, %22, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %11, %23, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf"
      : "+v"(C[0]), "+v"(C[1]), "+v"(C[2]), "+v"(C[3]), "+v"(C[4]), "+v"(C[5]), "+v"(C[6]),
        "+v"(C[7]), "+v"(C[8]), "+v"(C[9]), "+v"(C[10]), "+v"(C[11])
      : "v"(X[0]), "v"(X[1]), "v"(X[2]), "v"(X[3]), "v"(X[4]), "v"(X[5]), "v"(X[6]), "v"(X[7]),
        "v"(X[8]), "v"(X[9]), "v"(X[10]), "v"(X[11]), "v"(y), "i"(SRC));
}

// C[i] += bc<i>(x) * y for i = 0..11 (x, y: one register each)
__device__ __forceinline__ void fma_bcast_lanes(double (&C)[12], double x, double y) {
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %12, %13 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %12, %13 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %2, %12, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %3, %12, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %4, %12, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %5, %12, %13 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %6, %12, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %7, %12, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %8, %12, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %9, %12, %13 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %10, %12, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %11, %12, %13 row_newbcast:11 row_mask:0xf bank_mask:0xf"
      : "+v"(C[0]), "+v"(C[1]), "+v"(C[2]), "+v"(C[3]), "+v"(C[4]), "+v"(C[5]), "+v"(C[6]),
        "+v"(C[7]), "+v"(C[8]), "+v"(C[9]), "+v"(C[10]), "+v"(C[11])
      : "v"(x), "v"(y));
}

// fp32 twins (v_fmac_f32_dpp): same shapes, same hazard rule
template <int SRC>
__device__ __forceinline__ void fma_bcast_src(float (&C)[12], const float (&X)[12], float y) {
  static_assert(SRC >= 0 && SRC < kGroup, "row_newbcast source lane");
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f32_dpp %0, %12, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %13, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %14, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %15, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %4, %16, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %5, %17, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %6, %18, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %7, %19, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %8, %20, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %9, %21, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %10, %22, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %11, %23, %24 row_newbcast:%25 row_mask:0xf bank_mask:0xf"
      : "+v"(C[0]), "+v"(C[1]), "+v"(C[2]), "+v"(C[3]), "+v"(C[4]), "+v"(C[5]), "+v"(C[6]),
        "+v"(C[7]), "+v"(C[8]), "+v"(C[9]), "+v"(C[10]), "+v"(C[11])
      : "v"(X[0]), "v"(X[1]), "v"(X[2]), "v"(X[3]), "v"(X[4]), "v"(X[5]), "v"(X[6]), "v"(X[7]),
        "v"(X[8]), "v"(X[9]), "v"(X[10]), "v"(X[11]), "v"(y), "i"(SRC));
}
__device__ __forceinline__ void fma_bcast_lanes(float (&C)[12], float x, float y) {
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f32_dpp %0, %12, %13 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %12, %13 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %2, %12, %13 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %3, %12, %13 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %4, %12, %13 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %5, %12, %13 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %6, %12, %13 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %7, %12, %13 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %8, %12, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %9, %12, %13 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %10, %12, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %11, %12, %13 row_newbcast:11 row_mask:0xf bank_mask:0xf"
      : "+v"(C[0]), "+v"(C[1]), "+v"(C[2]), "+v"(C[3]), "+v"(C[4]), "+v"(C[5]), "+v"(C[6]),
        "+v"(C[7]), "+v"(C[8]), "+v"(C[9]), "+v"(C[10]), "+v"(C[11])
      : "v"(x), "v"(y));
}

// acc + sum_j M[j] * bc<j>(x): a lane's dot product with the row's element-owned
// vector x (lane j holds x_j), the broadcast riding on src0 of each FMA -- no
// gathered 12-register copy of x.  Same rounding as fma(M[j], x_j, acc) in
// order j = 0..11.
__device__ __forceinline__ double dot_bcast(const double (&M)[12], double x, double acc) {
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %10 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %12 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %1, %13 row_newbcast:11 row_mask:0xf bank_mask:0xf"
      : "+&v"(acc)
      : "v"(x), "v"(M[0]), "v"(M[1]), "v"(M[2]), "v"(M[3]), "v"(M[4]), "v"(M[5]), "v"(M[6]), "v"(M[7]), "v"(M[8]), "v"(M[9]), "v"(M[10]), "v"(M[11]));
  return acc;
}
__device__ __forceinline__ float dot_bcast(const float (&M)[12], float x, float acc) {
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f32_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %6 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %10 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %11 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %12 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %1, %13 row_newbcast:11 row_mask:0xf bank_mask:0xf"
      : "+&v"(acc)
      : "v"(x), "v"(M[0]), "v"(M[1]), "v"(M[2]), "v"(M[3]), "v"(M[4]), "v"(M[5]), "v"(M[6]), "v"(M[7]), "v"(M[8]), "v"(M[9]), "v"(M[10]), "v"(M[11]));
  return acc;
}

// two such dots on the same x, interleaved (two independent FMA chains)
__device__ __forceinline__ void dot_bcast2(const double (&M1)[12], const double (&M2)[12], double x,
                                           double& acc1, double& acc2) {
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f64_dpp %0, %2, %3 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %15 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %4 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %16 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %17 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %6 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %18 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %19 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %20 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %21 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %10 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %22 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %11 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %23 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %24 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %25 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %0, %2, %14 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %1, %2, %26 row_newbcast:11 row_mask:0xf bank_mask:0xf"
      : "+&v"(acc1), "+&v"(acc2)
      : "v"(x), "v"(M1[0]), "v"(M1[1]), "v"(M1[2]), "v"(M1[3]), "v"(M1[4]), "v"(M1[5]), "v"(M1[6]), "v"(M1[7]), "v"(M1[8]), "v"(M1[9]), "v"(M1[10]), "v"(M1[11]),
        "v"(M2[0]), "v"(M2[1]), "v"(M2[2]), "v"(M2[3]), "v"(M2[4]), "v"(M2[5]), "v"(M2[6]), "v"(M2[7]), "v"(M2[8]), "v"(M2[9]), "v"(M2[10]), "v"(M2[11]));
}
__device__ __forceinline__ void dot_bcast2(const float (&M1)[12], const float (&M2)[12], float x,
                                           float& acc1, float& acc2) {
  asm volatile(
      "s_nop 1\n\t"
      "v_fmac_f32_dpp %0, %2, %3 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %15 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %4 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %16 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %17 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %6 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %18 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %19 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %20 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %21 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %10 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %22 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %11 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %23 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %12 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %24 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %13 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %25 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %0, %2, %14 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f32_dpp %1, %2, %26 row_newbcast:11 row_mask:0xf bank_mask:0xf"
      : "+&v"(acc1), "+&v"(acc2)
      : "v"(x), "v"(M1[0]), "v"(M1[1]), "v"(M1[2]), "v"(M1[3]), "v"(M1[4]), "v"(M1[5]), "v"(M1[6]), "v"(M1[7]), "v"(M1[8]), "v"(M1[9]), "v"(M1[10]), "v"(M1[11]),
        "v"(M2[0]), "v"(M2[1]), "v"(M2[2]), "v"(M2[3]), "v"(M2[4]), "v"(M2[5]), "v"(M2[6]), "v"(M2[7]), "v"(M2[8]), "v"(M2[9]), "v"(M2[10]), "v"(M2[11]));
}

template <typename T>
__device__ __forceinline__ T fmadd(T a, T b, T c) {
  return __builtin_fma(a, b, c);
}
template <>
__device__ __forceinline__ float fmadd<float>(float a, float b, float c) {
  return __builtin_fmaf(a, b, c);
}

// 12 contiguous values -> registers (16-byte vector loads for double).
__device__ __forceinline__ void load12(const double* __restrict__ p, double (&v)[12]) {
  const double2* p2 = reinterpret_cast<const double2*>(p);
  sfor<0, 6>([&](auto i) {
    constexpr int I = decltype(i)::value;
    double2 t = p2[I];
    v[2 * I] = t.x;
    v[2 * I + 1] = t.y;
  });
}
// same, non-temporal (streamed once: global_load_dwordx4 ... nt)
__device__ __forceinline__ void load12_nt(const double* __restrict__ p, double (&v)[12]) {
  typedef double dv2 __attribute__((ext_vector_type(2)));
  const dv2* p2 = reinterpret_cast<const dv2*>(p);
  sfor<0, 6>([&](auto i) {
    constexpr int I = decltype(i)::value;
    dv2 t = __builtin_nontemporal_load(p2 + I);
    v[2 * I] = t.x;
    v[2 * I + 1] = t.y;
  });
}
__device__ __forceinline__ void load12_nt(const float* __restrict__ p, float (&v)[12]) {
  typedef float fv2 __attribute__((ext_vector_type(2)));
  const fv2* p2 = reinterpret_cast<const fv2*>(p);
  sfor<0, 6>([&](auto i) {
    constexpr int I = decltype(i)::value;
    fv2 t = __builtin_nontemporal_load(p2 + I);
    v[2 * I] = t.x;
    v[2 * I + 1] = t.y;
  });
}
__device__ __forceinline__ void store12(double* __restrict__ p, const double (&v)[12]) {
  double2* p2 = reinterpret_cast<double2*>(p);
  sfor<0, 6>([&](auto i) {
    constexpr int I = decltype(i)::value;
    p2[I] = make_double2(v[2 * I], v[2 * I + 1]);
  });
}

// fp32: 12 contiguous floats as 8-byte pairs (record offsets are even)
__device__ __forceinline__ void load12(const float* __restrict__ p, float (&v)[12]) {
  const float2* p2 = reinterpret_cast<const float2*>(p);
  sfor<0, 6>([&](auto i) {
    constexpr int I = decltype(i)::value;
    float2 t = p2[I];
    v[2 * I] = t.x;
    v[2 * I + 1] = t.y;
  });
}
__device__ __forceinline__ void store12(float* __restrict__ p, const float (&v)[12]) {
  float2* p2 = reinterpret_cast<float2*>(p);
  sfor<0, 6>([&](auto i) {
    constexpr int I = decltype(i)::value;
    p2[I] = make_float2(v[2 * I], v[2 * I + 1]);
  });
}

// Generic predicated column load: v[i] = (col_ok && i < rows) ? p[i] : 0.
template <typename T>
__device__ __forceinline__ void load_col_pad(const T* __restrict__ p, int rows, bool col_ok,
                                             T (&v)[12]) {
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    v[I] = (col_ok && I < rows) ? p[I] : T(0);
  });
}

// ---------------------------------------------------------------------------
// Packed lower triangle of a 12x12 block, by columns (78 values): column j
// holds rows j..11 from packed_col(j).  Used for the symmetric P and the
// Cholesky factor L in the stage records.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int packed_col(int j) { return j * 12 - j * (j - 1) / 2; }

// lane j < 12 stores its column v[i] = M[i][j], rows i >= j only
template <typename T>
__device__ __forceinline__ void store_packed_col(T* pk, int lane, const T (&v)[12]) {
  const int cj = packed_col(lane) - lane;
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    if (I >= lane) pk[cj + I] = v[I];
  });
}
// (The loaders below read every element at an address inside the 78-value block, valid
// for every r, c in 0..11, and select: a load under a lane-dependent condition becomes a
// branch of its own that waits for its load, one memory round trip per element.)
// row r (= column r) of a symmetric matrix stored as its packed lower triangle
template <typename T>
__device__ __forceinline__ void load_packed_sym(const T* pk, int r, T (&v)[12]) {
  const int cr = packed_col(r) - r;
  sfor<0, 12>([&](auto j) {
    constexpr int J = decltype(j)::value;
    v[J] = pk[J <= r ? packed_col(J) + r - J : cr + J];
  });
}
// row r of a packed lower-triangular L, diagonal included: v[j] = L[r][j] (j <= r), else 0
template <typename T>
__device__ __forceinline__ void load_packed_lrow_d(const T* pk, int r, T (&v)[12]) {
  sfor<0, 12>([&](auto j) {
    constexpr int J = decltype(j)::value;
    const T x = pk[packed_col(J) + r - J];
    v[J] = J <= r ? x : T(0);
  });
}
// column c of a packed lower-triangular L, diagonal included: v[i] = L[i][c] (i >= c), else 0
template <typename T>
__device__ __forceinline__ void load_packed_lcol_d(const T* pk, int c, T (&v)[12]) {
  const int cc = packed_col(c) - c;
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    const T x = pk[cc + I];
    v[I] = I >= c ? x : T(0);
  });
}
// strictly-lower row r of a packed lower-triangular L: v[j] = L[r][j] (j < r), else 0
template <typename T>
__device__ __forceinline__ void load_packed_lrow(const T* pk, int r, T (&v)[12]) {
  sfor<0, 12>([&](auto j) {
    constexpr int J = decltype(j)::value;
    const T x = pk[packed_col(J) + r - J];
    v[J] = J < r ? x : T(0);
  });
}
// strictly-lower column c of a packed lower-triangular L: v[i] = L[i][c] (i > c), else 0
template <typename T>
__device__ __forceinline__ void load_packed_lcol(const T* pk, int c, T (&v)[12]) {
  const int cc = packed_col(c) - c;
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
    const T x = pk[cc + I];
    v[I] = I > c ? x : T(0);
  });
}

}  // namespace srbd
