// rescue.hip -- the data movement of the mixed-precision paths.
//
// srbd_qp_settings.f64_rescue: after an fp32
// solve, the QPs it left unsolved (status != Success) are listed in batch order,
// their fp32 data widened into a compact fp64 batch, solved by the fp64 kernels,
// and the fp64 solutions narrowed back into the caller's fp32 outputs.
//
// The reference has no such path (HPIPM's s_ocp_qp_ipm_solve,
// hpipm_s_ocp_qp_ipm.h:238, stops where fp32 stops); it exists because the
// fp32 factorization of R + D'Gamma D breaks down on the friction-cone QPs whose
// active rows reach Gamma ~ 1e8-1e10.  All of it is
// HBM-bound copy work over a few percent of the batch.
//
// srbd_qp_settings.f32_iters (fp64 solves): the fp64 data narrowed once to fp32 for
// the first IPM iterations, the fp32 iterate widened back for the fp64 ones.
#include "kernels.h"

#include <hip/hip_runtime.h>

namespace srbd {
namespace {

constexpr int kSelThreads = 1024;

// One workgroup walks the batch in 1024-QP tiles: per wave a ballot of the
// unsolved flags and its prefix popcount, per tile a 16-entry prefix over the
// waves, so idx[] lists the unsolved QPs in ascending order (deterministic).
__global__ __launch_bounds__(kSelThreads) void select_unsolved_kernel(const int* __restrict__ status,
                                                                      int batch, int min_status,
                                                                      int* __restrict__ idx,
                                                                      int* __restrict__ count) {
  __shared__ int wave_tot[kSelThreads / 64];
  __shared__ int wave_off[kSelThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int base_out = 0;
  for (int base = 0; base < batch; base += kSelThreads) {
    const int i = base + (int)threadIdx.x;
    const bool flag = i < batch && status[i] >= min_status;
    const unsigned long long m = __ballot(flag);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wave] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      int run = 0;
      for (int w = 0; w < kSelThreads / 64; ++w) {
        wave_off[w] = run;
        run += wave_tot[w];
      }
      wave_tot[0] = run;  // tile total (wave_tot is re-written next tile after the barrier)
    }
    __syncthreads();
    if (flag) idx[base_out + wave_off[wave] + before] = i;
    base_out += wave_tot[0];
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base_out;
}

__global__ void gather_widen_kernel(const float* __restrict__ src, double* __restrict__ dst,
                                    const int* __restrict__ idx, int rows, size_t elems) {
  const size_t total = (size_t)rows * elems;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t r = t / elems, j = t - r * elems;
    dst[t] = (double)src[(size_t)idx[r] * elems + j];
  }
}

__global__ void scatter_narrow_kernel(const double* __restrict__ src, float* __restrict__ dst,
                                      const int* __restrict__ idx, int rows, size_t elems) {
  const size_t total = (size_t)rows * elems;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t r = t / elems, j = t - r * elems;
    dst[(size_t)idx[r] * elems + j] = (float)src[t];
  }
}

__global__ void scatter_int_kernel(const int* __restrict__ src, int* __restrict__ dst,
                                   const int* __restrict__ idx, int rows) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < rows) dst[idx[t]] = src[t];
}

__global__ void gather_rows_kernel(const double* __restrict__ src, double* __restrict__ dst,
                                   const int* __restrict__ idx, int rows, size_t elems) {
  const size_t total = (size_t)rows * elems;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t r = t / elems, j = t - r * elems;
    dst[t] = src[(size_t)idx[r] * elems + j];
  }
}

__global__ void scatter_rows_kernel(const double* __restrict__ src, double* __restrict__ dst,
                                    const int* __restrict__ idx, int rows, size_t elems) {
  const size_t total = (size_t)rows * elems;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t r = t / elems, j = t - r * elems;
    dst[(size_t)idx[r] * elems + j] = src[t];
  }
}

__global__ void narrow_kernel(const double* __restrict__ src, float* __restrict__ dst, size_t n) {
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (size_t)gridDim.x * blockDim.x)
    dst[t] = (float)src[t];
}

__global__ void widen_kernel(const float* __restrict__ src, double* __restrict__ dst, size_t n) {
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (size_t)gridDim.x * blockDim.x)
    dst[t] = (double)src[t];
}

dim3 copy_grid(size_t total) {
  const size_t blocks = (total + 255) / 256;
  return dim3((unsigned)(blocks < 8192 ? (blocks ? blocks : 1) : 8192));
}

}  // namespace

hipError_t launch_select_unsolved(const int* status, int batch, int min_status, int* idx, int* count,
                                  hipStream_t s) {
  hipLaunchKernelGGL(select_unsolved_kernel, dim3(1), dim3(kSelThreads), 0, s, status, batch, min_status,
                     idx, count);
  return hipGetLastError();
}

hipError_t launch_gather_widen(const float* src, double* dst, const int* idx, int rows, size_t elems,
                               hipStream_t s) {
  if (!rows || !elems) return hipSuccess;
  hipLaunchKernelGGL(gather_widen_kernel, copy_grid((size_t)rows * elems), dim3(256), 0, s, src, dst,
                     idx, rows, elems);
  return hipGetLastError();
}

hipError_t launch_scatter_narrow(const double* src, float* dst, const int* idx, int rows, size_t elems,
                                 hipStream_t s) {
  if (!rows || !elems) return hipSuccess;
  hipLaunchKernelGGL(scatter_narrow_kernel, copy_grid((size_t)rows * elems), dim3(256), 0, s, src, dst,
                     idx, rows, elems);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const double* src, double* dst, const int* idx, int rows, size_t elems,
                              hipStream_t s) {
  if (!rows || !elems) return hipSuccess;
  hipLaunchKernelGGL(gather_rows_kernel, copy_grid((size_t)rows * elems), dim3(256), 0, s, src, dst, idx,
                     rows, elems);
  return hipGetLastError();
}

hipError_t launch_scatter_rows(const double* src, double* dst, const int* idx, int rows, size_t elems,
                               hipStream_t s) {
  if (!rows || !elems) return hipSuccess;
  hipLaunchKernelGGL(scatter_rows_kernel, copy_grid((size_t)rows * elems), dim3(256), 0, s, src, dst, idx,
                     rows, elems);
  return hipGetLastError();
}

hipError_t launch_narrow(const double* src, float* dst, size_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(narrow_kernel, copy_grid(n), dim3(256), 0, s, src, dst, n);
  return hipGetLastError();
}

hipError_t launch_widen(const float* src, double* dst, size_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(widen_kernel, copy_grid(n), dim3(256), 0, s, src, dst, n);
  return hipGetLastError();
}

hipError_t launch_scatter_int(const int* src, int* dst, const int* idx, int rows, hipStream_t s) {
  if (!rows) return hipSuccess;
  hipLaunchKernelGGL(scatter_int_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, src, dst,
                     idx, rows);
  return hipGetLastError();
}

}  // namespace srbd
