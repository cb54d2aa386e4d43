// Probe: does a resident (spinning) kernel on one stream hold back kernels of other streams?
// A spinner runs on the "server" stream (plain non-blocking, high priority, or CU-masked) until
// the host releases it (or 300 ms of wall clock pass); meanwhile one tiny kernel is launched on
// each of 8 other non-blocking streams and on the null stream, and the time until each finishes
// is reported.  Build: hipcc --offload-arch=gfx950 -O2 server_queue_probe.hip -o probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

__global__ void spinner(volatile int* release, long long max_ticks) {
  const long long t0 = wall_clock64();
  if (threadIdx.x == 0)
    while (!__hip_atomic_load((int*)release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) &&
           wall_clock64() - t0 < max_ticks)
      __builtin_amdgcn_s_sleep(8);
  __syncthreads();
}
__global__ void tiny(int* p) { p[threadIdx.x] += 1; }

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                       \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

static int run(const char* mode) {
  int* rel = nullptr;
  CK(hipHostMalloc((void**)&rel, 64, hipHostMallocCoherent | hipHostMallocMapped));
  *(volatile int*)rel = 0;
  int* rel_dev = nullptr;
  CK(hipHostGetDevicePointer((void**)&rel_dev, rel, 0));
  int* buf = nullptr;
  CK(hipMalloc(&buf, 64 * sizeof(int) * 10));
  hipStream_t others[8];
  for (auto& s : others) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipStream_t srv = nullptr;
  if (!std::strcmp(mode, "plain")) {
    CK(hipStreamCreateWithFlags(&srv, hipStreamNonBlocking));
  } else if (!std::strcmp(mode, "prio")) {
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&srv, hipStreamNonBlocking, hi));
  } else {
    uint32_t mask[8];
    for (auto& m : mask) m = 0xffffffffu;
    CK(hipExtStreamCreateWithCUMask(&srv, 8, mask));
  }
  int khz = 100000;
  hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  // warm up every stream (queues are bound on first use)
  for (auto& s : others) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, buf);
  hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, srv, buf);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(spinner, dim3(1), dim3(64), 0, srv, rel_dev, (long long)khz * 300);
  std::this_thread::sleep_for(std::chrono::milliseconds(5));
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, others[i], buf + 64 * (i + 1));
  hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, (hipStream_t)0, buf + 64 * 9);
  double done_ms[9];
  for (auto& d : done_ms) d = -1;
  int left = 9;
  while (left && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(100)) {
    for (int i = 0; i < 9; ++i) {
      if (done_ms[i] >= 0) continue;
      hipStream_t s = i < 8 ? others[i] : (hipStream_t)0;
      if (hipStreamQuery(s) == hipSuccess) {
        done_ms[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        --left;
      }
    }
  }
  const bool spin_running = hipStreamQuery(srv) == hipErrorNotReady;
  *(volatile int*)rel = 1;  // release the spinner
  CK(hipDeviceSynchronize());
  std::printf("{\"mode\": \"%s\", \"spinner_running_at_100ms\": %s, \"done_ms\": [", mode,
              spin_running ? "true" : "false");
  for (int i = 0; i < 9; ++i) std::printf("%s%.3f", i ? ", " : "", done_ms[i]);
  std::printf("], \"note\": \"-1 = still blocked after 100 ms; last entry = null stream\"}\n");
  for (auto& s : others) hipStreamDestroy(s);
  hipStreamDestroy(srv);
  hipFree(buf);
  hipHostFree(rel);
  return 0;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "plain";
  return run(mode);
}
