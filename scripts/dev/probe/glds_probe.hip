// Probe: where global_load_lds_dwordx4 writes LDS (lane mapping, instruction offset, exec mask).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(const double* src, double* out) {
  __shared__ __attribute__((aligned(16))) double lds[512];
  for (int i = threadIdx.x; i < 512; i += 64) lds[i] = -1.0;
  __syncthreads();
  const int lane = threadIdx.x & 15, gw = threadIdx.x >> 4;
  const auto* g = (const __attribute__((address_space(1))) void*)(src + 2 * lane);
  if (gw == 1) {
    auto* l = (__attribute__((address_space(3))) void*)(lds + 64 - 32);
    __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(g, l, 16, 256, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}
int main() {
  double h[512], *d, *o;
  for (int i = 0; i < 512; ++i) h[i] = i;
  hipMalloc(&d, sizeof h); hipMalloc(&o, sizeof h);
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o);
  hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
  for (int i = 0; i < 512; ++i) if (h[i] != -1.0) printf("lds[%d] = %g\n", i, h[i]);
  return 0;
}
