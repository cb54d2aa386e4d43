// Dev probe: does a streamed read with the non-temporal hint leave the Infinity Cache
// (MALL) contents alone?  (1) write a `rec` buffer, (2) stream a large `in` buffer with
// whole-line 16-byte loads, plain or non-temporal, (3) read `rec` back; time (3).
// If (3) runs at on-die rate after the nt stream and at HBM rate after the plain one,
// nt loads do not allocate in the MALL.
// hipcc -O3 --offload-arch=gfx950 scripts/dev/mall_probe.hip -o build/mall_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ void write_k(d2* p, size_t n, double v, int nt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (nt) __builtin_nontemporal_store(d2{v, v + 1.0}, p + i);
    else p[i] = d2{v, v + 1.0};
  }
}

// 8 independent 16-byte loads in flight per lane per step (whole 1 KiB per wave-instruction)
template <int NT>
__global__ void read_k(const d2* p, size_t n, double* sink) {
  d2 acc = {0.0, 0.0};
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 7 * stride < n; i += 8 * stride) {
    d2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (NT) v[u] = __builtin_nontemporal_load(p + i + u * stride);
      else v[u] = p[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  if (acc.x == -1.2345) sink[0] = acc.y;  // never: keeps the loads
}

int main(int argc, char** argv) {
  const size_t rec_mb = argc > 1 ? atoi(argv[1]) : 128, in_mb = argc > 2 ? atoi(argv[2]) : 2048;
  const int ntw = argc > 3 ? atoi(argv[3]) : 0;
  const size_t nr = rec_mb * (1 << 20) / 16, ni = in_mb * (1 << 20) / 16;
  d2 *rec, *in;
  double* sink;
  hipMalloc(&rec, nr * 16);
  hipMalloc(&in, ni * 16);
  hipMalloc(&sink, 8);
  const dim3 g(256 * 8), b(256);
  hipLaunchKernelGGL(write_k, g, b, 0, 0, in, ni, 1.0, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    for (int nt = 0; nt < 3; ++nt) {  // 0: plain stream, 1: nt stream, 2: no stream
      hipLaunchKernelGGL(write_k, g, b, 0, 0, rec, nr, 2.0, ntw);
      if (nt == 0) hipLaunchKernelGGL(read_k<0>, g, b, 0, 0, in, ni, sink);
      if (nt == 1) hipLaunchKernelGGL(read_k<1>, g, b, 0, 0, in, ni, sink);
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(read_k<0>, g, b, 0, 0, rec, nr, sink);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("rec %zu MB (%s writes) after %s stream of %zu MB: re-read %.3f ms = %.2f TB/s\n", rec_mb, ntw ? "nt" : "plain",
             nt == 0 ? "plain" : nt == 1 ? "nt" : "no", nt == 2 ? (size_t)0 : in_mb, ms,
             rec_mb * 1048576.0 / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
