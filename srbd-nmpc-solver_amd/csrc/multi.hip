// multi.hip -- one solver over several devices, from one host thread ("one
// process, 8 devices"; BASELINE config 4: 262144 QPs sharded over 8 MI355X with the solutions
// gathered to one device).  Built on the public C-ABI only: a handle per device, the
// asynchronous srbd_qp_solve_f64 on each (the IPM's stop decision is taken on the device, so
// the launches of every device are queued before any is waited for), and the gather of x, u,
// pi to the root device by peer copies over xGMI, each queued on its shard's stream behind
// its solve.  (Multi-process runs -- bench.py --gpus N -- gather over RCCL instead.)
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/srbd_qp.h"

struct srbd_qp_multi_s {
  srbd_qp_dims dims{};
  int capacity = 0;
  std::vector<int> dev;
  std::vector<srbd_qp_handle> h;
};

namespace srbd {
int set_error(int code, const std::string& msg);  // srbd_qp_capi.hip
}

extern "C" {

int srbd_qp_multi_create(const srbd_qp_dims* dims, int capacity_per_device, const int* devices, int ndev,
                         srbd_qp_multi* out) {
  if (!out || !dims || !devices) return srbd::set_error(SRBD_QP_EINVAL, "multi: NULL argument");
  *out = nullptr;
  if (ndev < 1) return srbd::set_error(SRBD_QP_EINVAL, "multi: ndev must be >= 1");
  auto* m = new srbd_qp_multi_s();
  m->dims = *dims;
  m->capacity = capacity_per_device;
  for (int i = 0; i < ndev; ++i) {
    srbd_qp_handle h = nullptr;
    const int rc = srbd_qp_create(dims, capacity_per_device, devices[i], &h);
    if (rc) {
      srbd_qp_multi_destroy(m);
      return rc;  // (message set by srbd_qp_create)
    }
    m->dev.push_back(devices[i]);
    m->h.push_back(h);
  }
  // peer access root <-> shard (xGMI); a device with itself, or a pair without peer access,
  // still copies (the runtime stages the copy)
  int prev = 0;
  hipGetDevice(&prev);
  for (int i = 1; i < ndev; ++i) {
    if (m->dev[i] == m->dev[0]) continue;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, m->dev[0], m->dev[i]) == hipSuccess && can) {
      hipSetDevice(m->dev[0]);
      (void)hipDeviceEnablePeerAccess(m->dev[i], 0);  // (already enabled: fine)
      hipSetDevice(m->dev[i]);
      (void)hipDeviceEnablePeerAccess(m->dev[0], 0);
    }
  }
  (void)hipGetLastError();
  hipSetDevice(prev);
  *out = m;
  return SRBD_QP_OK;
}

void srbd_qp_multi_destroy(srbd_qp_multi m) {
  if (!m) return;
  for (srbd_qp_handle h : m->h) srbd_qp_destroy(h);
  delete m;
}

srbd_qp_handle srbd_qp_multi_handle(srbd_qp_multi m, int i) {
  return m && i >= 0 && i < (int)m->h.size() ? m->h[i] : nullptr;
}

}  // extern "C"

namespace {
// srbd_qp_solve_f64 / _f32 by the precision's structs
int solve_one(srbd_qp_handle h, int b, const srbd_qp_settings* st, const srbd_qp_data_f64* d,
              const srbd_qp_solution_f64* s) {
  return srbd_qp_solve_f64(h, b, st, d, s, nullptr);
}
int solve_one(srbd_qp_handle h, int b, const srbd_qp_settings* st, const srbd_qp_data_f32* d,
              const srbd_qp_solution_f32* s) {
  return srbd_qp_solve_f32(h, b, st, d, s, nullptr);
}

template <typename T, typename Data, typename Sol>
int multi_solve(srbd_qp_multi m, const int* batch, const srbd_qp_settings* settings, const Data* data,
                const Sol* sol, T* root_x, T* root_u, T* root_pi) {
  if (!m || !batch || !data || !sol) return srbd::set_error(SRBD_QP_EINVAL, "multi: NULL argument");
  const int n = (int)m->h.size();
  const size_t N = (size_t)m->dims.N, nx = (size_t)m->dims.nx, nu = (size_t)m->dims.nu;
  // every shard's launch sequence first: the devices run concurrently
  for (int i = 0; i < n; ++i) {
    const int rc = solve_one(m->h[i], batch[i], settings, &data[i], &sol[i]);
    if (rc) {
      for (int j = 0; j < i; ++j) srbd_qp_synchronize(m->h[j]);
      return rc;
    }
  }
  // the gather: shard i's rows behind its solve, on its stream
  int prev = 0;
  hipGetDevice(&prev);
  hipError_t e = hipSuccess;
  size_t row = 0;
  for (int i = 0; i < n && e == hipSuccess; ++i) {
    const size_t b = (size_t)batch[i];
    hipSetDevice(m->dev[i]);
    hipStream_t s = reinterpret_cast<hipStream_t>(srbd_qp_stream(m->h[i]));
    auto copy = [&](T* dst, const T* src, size_t per_qp) {
      if (e != hipSuccess || !dst || !src || !b) return;
      e = hipMemcpyPeerAsync(dst + row * per_qp, m->dev[0], src, m->dev[i], b * per_qp * sizeof(T), s);
    };
    copy(root_x, sol[i].x, (N + 1) * nx);
    copy(root_u, sol[i].u, N * nu);
    copy(root_pi, sol[i].pi, (N + 1) * nx);
    row += b;
  }
  hipSetDevice(prev);
  int rc = SRBD_QP_OK;
  for (int i = 0; i < n; ++i) {
    const int r = srbd_qp_synchronize(m->h[i]);
    if (r && !rc) rc = r;
  }
  if (e != hipSuccess) return srbd::set_error(SRBD_QP_EDEVICE, std::string("multi gather: ") + hipGetErrorString(e));
  return rc;
}
}  // namespace

extern "C" {

int srbd_qp_multi_solve_f64(srbd_qp_multi m, const int* batch, const srbd_qp_settings* settings,
                            const srbd_qp_data_f64* data, const srbd_qp_solution_f64* sol, double* root_x,
                            double* root_u, double* root_pi) {
  return multi_solve<double>(m, batch, settings, data, sol, root_x, root_u, root_pi);
}

int srbd_qp_multi_solve_f32(srbd_qp_multi m, const int* batch, const srbd_qp_settings* settings,
                            const srbd_qp_data_f32* data, const srbd_qp_solution_f32* sol, float* root_x,
                            float* root_u, float* root_pi) {
  return multi_solve<float>(m, batch, settings, data, sol, root_x, root_u, root_pi);
}

}  // extern "C"
