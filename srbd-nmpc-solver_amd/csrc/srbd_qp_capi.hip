// srbd_qp_capi.hip -- implementation of the C-ABI in include/srbd_qp.h.
//
// Host-side orchestration only: argument checks (the batched analogue of
// OcpQpDim::checkSize, hpipm-cpp/src/ocp_qp_dim.cpp:59-246, and
// OcpQpIpmSolverSettings::checkSettings, ocp_qp_ipm_solver_settings.cpp:7-38),
// workspace ownership (what d_ocp_qp_ipm_ws_wrapper did,
// src/detail/d_ocp_qp_ipm_ws_wrapper.cpp:141-155 -- sized once here instead of
// on every solve() as the reference does at ocp_qp_ipm_solver.cpp:185), and
// dispatch to the HIP kernels.  No CPU fallback exists: without a GPU every
// solve returns SRBD_QP_EDEVICE.
#include "../../include/srbd_qp.h"
#include "kernels.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <type_traits>
#include <vector>

namespace {

thread_local std::string g_last_error = "";

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

}  // namespace

namespace srbd {
// the thread's last-error message, for the other translation units of the ABI (multi.hip)
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace srbd

struct srbd_qp_handle_s {
  srbd_qp_dims dims{};
  int capacity = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  double* ws = nullptr;
  size_t ws_qp = 0;  // doubles per QP
  size_t ws_bytes = 0;
  // host-solve staging (device)
  double* stage = nullptr;
  size_t stage_bytes = 0;
  // small host solves (batch 1: the reference's call pattern): pinned mirror of the
  // staging buffer, so inputs go over in one copy and the outputs come back in one
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  // nx < 12 or nu < 12: the 12 x 12 embedding (pad.hip), allocated on first use
  void* pad = nullptr;
  size_t pad_bytes = 0;
  // srbd_qp_srbd_nmpc_f64: QP data, solution and loop state, allocated on first use
  void* nmpc = nullptr;
  size_t nmpc_bytes = 0;
  int* nmpc_active_host = nullptr;  // pinned
  // settings.f64_rescue: unsolved-QP list + status (capacity ints each, then the count),
  // and the compact fp64 batch, allocated on first use
  int* resc_idx = nullptr;
  int* resc_count_host = nullptr;  // pinned
  void* resc = nullptr;
  size_t resc_bytes = 0;
  // the cold fp64 re-solve of rescued QPs the continuation left unsolved (first use)
  void* resc2 = nullptr;
  size_t resc2_bytes = 0;
  // settings.f32_iters: fp32 copy of the data, fp32 iterate, barrier state (first use)
  void* mixed = nullptr;
  size_t mixed_bytes = 0;
  // the latency IPM's lq_fact 1 switch: its flag (device) and read-back (pinned), the list,
  // status and count of the QPs that raised it (capacity ints each, then the count) and their
  // compact batch for the batched kernels (first use); force_batched while those are solved
  int* lat_flag = nullptr;
  int* lat_flag_host = nullptr;
  int* lqsw_idx = nullptr;
  void* lqsw = nullptr;
  size_t lqsw_bytes = 0;
  bool force_batched = false;
  // live-QP control of the IPM launch sequence (ProblemArgsT::ctl): device counters and
  // control words, decided on the device (the host never waits on them)
  int* ctl = nullptr;
  int* qp_buf = nullptr;  // active-QP list of the IPM sweeps: capacity + 1 ints
  // srbd_qp_solve_host_cb_f64: per-QP "factors written" flags (pinned, coherent, first use)
  // and, for the one launch that arms them, their device address (ProblemArgsT::factors_ready)
  int* fac_flags = nullptr;
  int* fac_arm = nullptr;
  // the one-QP host call's resident server (riccati_latency_server_kernel; first use): its
  // mailbox in mapped coherent host memory, its own stream, the arguments it was launched
  // with, launches so far (epoch), requests posted so far
  srbd::LatMailbox* srv_mb = nullptr;
  srbd::LatMailbox* srv_mb_dev = nullptr;
  hipStream_t srv_stream = nullptr;
  srbd::ProblemArgsT<double> srv_args{};
  int srv_epoch = 0;
  int srv_seq = 0;
  bool srv_live = false;
};

extern "C" {

int srbd_qp_abi_version(void) { return SRBD_QP_ABI_VERSION; }

const char* srbd_qp_last_error(void) { return g_last_error.c_str(); }

const char* srbd_qp_status_string(int s) {
  switch (s) {
    case SRBD_QP_SUCCESS: return "HpipmStatus::Success";
    case SRBD_QP_MAX_ITER: return "HpipmStatus::MaxIterReached";
    case SRBD_QP_MIN_STEP: return "HpipmStatus::MinStepLengthReached";
    case SRBD_QP_NAN_SOL: return "HpipmStatus::NaNDetected";
    default: return "HpipmStatus::UnknownFailure";
  }
}

const char* srbd_qp_error_string(int e) {
  switch (e) {
    case SRBD_QP_OK: return "ok";
    case SRBD_QP_EINVAL: return "invalid argument";
    case SRBD_QP_EDIM: return "unsupported dimensions";
    case SRBD_QP_ENOMEM: return "device out of memory";
    case SRBD_QP_EDEVICE: return "HIP device error";
    case SRBD_QP_ECAPACITY: return "batch exceeds handle capacity";
    case SRBD_QP_ESETTINGS: return "invalid settings";
    default: return "unknown error";
  }
}

void srbd_qp_default_settings(srbd_qp_settings* s) {
  if (!s) return;
  // hpipm-cpp/include/hpipm-cpp/ocp_qp_ipm_solver_settings.hpp:26-86
  s->mode = SRBD_QP_MODE_SPEED;
  s->iter_max = 15;
  s->alpha_min = 1.0e-08;
  s->mu0 = 1.0e+02;
  s->tol_stat = 1.0e-08;
  s->tol_eq = 1.0e-08;
  s->tol_ineq = 1.0e-08;
  s->tol_comp = 1.0e-08;
  s->reg_prim = 1.0e-12;
  s->warm_start = 0;
  s->pred_corr = 1;
  s->ric_alg = 1;
  s->split_step = 0;
  s->compute_residuals = 1;  // HPIPM's comp_res_exit
  s->f64_rescue = 0;
  s->f32_iters = 0;
  s->lq_fact = -1;
}

int srbd_qp_check_settings(const srbd_qp_settings* s) {
  if (!s) return fail(SRBD_QP_EINVAL, "settings is NULL");
  // messages of OcpQpIpmSolverSettings::checkSettings (settings.cpp:7-38)
  if (s->iter_max < 0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.iter_max must be non-negative");
  if (s->alpha_min <= 0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.alpha_min must be positive");
  if (s->alpha_min > 1.0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.alpha_min must be less than 1.0");
  if (s->mu0 <= 0.0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.mu0 must be positive");
  if (s->tol_stat <= 0.0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.tol_stat must be positive");
  if (s->tol_eq <= 0.0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.tol_eq must be positive");
  if (s->tol_ineq <= 0.0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.tol_ineq must be positive");
  if (s->tol_comp <= 0.0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.tol_comp must be positive");
  if (s->reg_prim < 0.0) return fail(SRBD_QP_ESETTINGS, "OcpQpIpmSolverSettings.reg_prim must be non-negative");
  // extensions (srbd_qp.h)
  if (s->f64_rescue < 0) return fail(SRBD_QP_ESETTINGS, "srbd_qp_settings.f64_rescue must be non-negative");
  if (s->f32_iters < 0) return fail(SRBD_QP_ESETTINGS, "srbd_qp_settings.f32_iters must be non-negative");
  if (s->lq_fact < -1 || s->lq_fact > 2)
    return fail(SRBD_QP_ESETTINGS, "srbd_qp_settings.lq_fact must be -1 (the mode's), 0, 1 or 2");
  return SRBD_QP_OK;
}

static int check_dims(const srbd_qp_dims* d) {
  if (!d) return fail(SRBD_QP_EINVAL, "dims is NULL");
  if (d->layout != SRBD_QP_LAYOUT_QP_MAJOR && d->layout != SRBD_QP_LAYOUT_STAGE_MAJOR)
    return fail(SRBD_QP_EINVAL, "unknown layout " + std::to_string(d->layout));
  if (d->layout == SRBD_QP_LAYOUT_STAGE_MAJOR &&
      (d->has_box_u || d->has_box_x || d->ng > 0 || d->nx != 12 || d->nu != 12))
    return fail(SRBD_QP_EINVAL, "stage-major inputs are supported by the unconstrained 12 x 12 solve only");
  if (d->N < 1 || d->N > 1024)
    return fail(SRBD_QP_EDIM, "N must be in [1, 1024], got " + std::to_string(d->N));
  if (d->nx < 1 || d->nx > SRBD_QP_MAX_NX)
    return fail(SRBD_QP_EDIM, "nx must be in [1, 12], got " + std::to_string(d->nx));
  if (d->nu < 1 || d->nu > SRBD_QP_MAX_NU)
    return fail(SRBD_QP_EDIM, "nu must be in [1, 12], got " + std::to_string(d->nu));
  if (d->ng < 0 || d->ng > SRBD_QP_MAX_NG)
    return fail(SRBD_QP_EDIM, "ng must be in [0, 64], got " + std::to_string(d->ng));
  return SRBD_QP_OK;
}

static bool constrained(const srbd_qp_dims& d) { return d.has_box_u || d.has_box_x || d.ng > 0; }

static size_t ws_doubles_per_qp(const srbd_qp_dims& d) {
  return constrained(d) ? srbd::ws_doubles_ipm(d.N, d.ng) : srbd::ws_doubles_unconstr(d.N);
}

int srbd_qp_create(const srbd_qp_dims* dims, int batch_capacity, int device, srbd_qp_handle* out) {
  if (!out) return fail(SRBD_QP_EINVAL, "out handle pointer is NULL");
  *out = nullptr;
  int rc = check_dims(dims);
  if (rc) return rc;
  if (batch_capacity < 1) return fail(SRBD_QP_EINVAL, "batch_capacity must be >= 1");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(SRBD_QP_EDEVICE, "no HIP device available (libsrbd_qp has no CPU fallback)");
  if (device < 0 || device >= ndev)
    return fail(SRBD_QP_EDEVICE, "device index " + std::to_string(device) + " out of range");
  int prev = 0;
  hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return fail(SRBD_QP_EDEVICE, "hipSetDevice failed");
  auto* h = new srbd_qp_handle_s();
  h->dims = *dims;
  h->capacity = batch_capacity;
  h->device = device;
  h->ws_qp = ws_doubles_per_qp(*dims);
  h->ws_bytes = h->ws_qp * sizeof(double) * (size_t)batch_capacity;
  hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = srbd::prepare_riccati_device();  // per-device kernel attributes
  if (e == hipSuccess) e = srbd::prepare_ipm_latency_device();
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->ws), h->ws_bytes);
  if (e == hipSuccess && constrained(*dims)) {
    e = hipMalloc(reinterpret_cast<void**>(&h->ctl), sizeof(int) * srbd::kCtlInts);
    if (e == hipSuccess) e = hipMemset(h->ctl, 0, sizeof(int) * srbd::kCtlInts);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&h->qp_buf), sizeof(int) * ((size_t)batch_capacity + 1));
  }
  hipSetDevice(prev);
  if (e != hipSuccess) {
    srbd_qp_destroy(h);
    return fail(e == hipErrorOutOfMemory ? SRBD_QP_ENOMEM : SRBD_QP_EDEVICE,
                std::string("workspace allocation failed: ") + hipGetErrorString(e));
  }
  *out = h;
  return SRBD_QP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// The resident server of the one-QP host call (riccati_latency_server_kernel)
// ---------------------------------------------------------------------------
namespace {
// wall-clock idle time after which a server leaves its CU (the next call relaunches it)
constexpr int kServerIdleMs = 5;
// and leaves after its first answer once this long has passed since its launch: whatever
// shares its hardware queue (other high-priority streams) waits at most about this long
constexpr int kServerLifeMs = 20;
// SRBD_LAT_SERVER_IDLE_MS overrides it (0: the server leaves as soon as it finds no request,
// so a call's post usually lands after the server left -- the test of the relaunch path)
int server_idle_ms() {
  const char* v = std::getenv("SRBD_LAT_SERVER_IDLE_MS");  // (read per launch: tests set it)
  return v && *v ? std::max(0, std::atoi(v)) : kServerIdleMs;
}
// test hook: SRBD_LAT_SERVER_POST_DELAY_US holds the post back this long after the host found
// the server live, so that with a zero idle time the server leaves in between -- every call
// then takes the wait loop's relaunch-after-post branch
int server_post_delay_us() {
  const char* v = std::getenv("SRBD_LAT_SERVER_POST_DELAY_US");
  return v && *v ? std::max(0, std::atoi(v)) : 0;
}
// a request not answered in this long is a device failure (generous: a server launch can
// queue behind long kernels of other streams before it reaches a CU)
constexpr auto kServerTimeout = std::chrono::seconds(30);
std::mutex g_srv_mu;
std::vector<srbd_qp_handle> g_srv_live;  // handles whose server may be running
// at exit: ask every live server to leave and give it a moment to drain (no HIP calls: the
// runtime may already be going down)
void server_atexit() {
  std::lock_guard<std::mutex> lk(g_srv_mu);
  for (srbd_qp_handle h : g_srv_live) {
    volatile srbd::LatMailbox* mb = h->srv_mb;
    mb->flags = srbd::kLatQuit;
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(200);
    while (mb->exited != h->srv_epoch && std::chrono::steady_clock::now() < t_end) std::this_thread::yield();
  }
  g_srv_live.clear();
}
bool server_enabled() {
  const char* v = std::getenv("SRBD_LAT_SERVER");  // 0: every call launches its kernel
  return !(v && v[0] == '0');
}
}  // namespace

// on the handle's device
static void server_stop(srbd_qp_handle h) {
  if (h->srv_live) {
    reinterpret_cast<volatile srbd::LatMailbox*>(h->srv_mb)->flags = srbd::kLatQuit;
    hipStreamSynchronize(h->srv_stream);
    reinterpret_cast<volatile srbd::LatMailbox*>(h->srv_mb)->flags = 0;
    h->srv_live = false;
  }
  // always off the exit hook's list: a handle whose relaunch failed (srv_live false) may
  // still be listed, and srbd_qp_destroy frees it and its mailbox right after this
  std::lock_guard<std::mutex> lk(g_srv_mu);
  g_srv_live.erase(std::remove(g_srv_live.begin(), g_srv_live.end(), h), g_srv_live.end());
}

// (re)launch the server with `a` on the handle's device.  `last_done` is the last request
// number that was answered (or abandoned): the server serves the first mailbox seq that
// differs from it.  Before a post that is h->srv_seq; after the post (the wait loop's
// relaunch of a server that idled out just before it) it is h->srv_seq - 1, or the pending
// request would count as done and never be served.
static hipError_t server_launch(srbd_qp_handle h, const srbd::ProblemArgsT<double>& a, int last_done) {
  hipError_t e = hipSuccess;
  if (!h->srv_mb) {
    e = hipHostMalloc(reinterpret_cast<void**>(&h->srv_mb), sizeof(srbd::LatMailbox),
                      hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) return e;
    std::memset(h->srv_mb, 0, sizeof(srbd::LatMailbox));
    void* dev = nullptr;
    e = hipHostGetDevicePointer(&dev, h->srv_mb, 0);
    if (e == hipSuccess) h->srv_mb_dev = reinterpret_cast<srbd::LatMailbox*>(dev);
    // The server's stream at the greatest priority: HIP maps a process's streams onto a few
    // hardware queues (GPU_MAX_HW_QUEUES, 4 here) per priority, each processing its packets in
    // order, so a kernel of another stream that shares the server's queue would wait until the
    // server leaves.  High-priority streams come from their own queue pool, which only other
    // high-priority streams share (scripts/dev/server_queue_probe.hip: with a plain stream 2 of
    // 8 other streams were held back by a resident kernel, with a high-priority one none).
    int prio_lo = 0, prio_hi = 0;
    if (e == hipSuccess && hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_hi = 0;
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&h->srv_stream, hipStreamNonBlocking, prio_hi);
    if (e != hipSuccess) return e;
    static std::once_flag once;
    std::call_once(once, [] { std::atexit(server_atexit); });
  }
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device) != hipSuccess || khz <= 0)
    khz = 100000;
  std::memcpy(&h->srv_args, &a, sizeof a);
  e = srbd::launch_latency_server(a, h->srv_mb_dev, ++h->srv_epoch, last_done, (long long)khz * server_idle_ms(),
                                  (long long)khz * kServerLifeMs, h->srv_stream);
  h->srv_live = e == hipSuccess;
  if (h->srv_live) {
    std::lock_guard<std::mutex> lk(g_srv_mu);
    if (std::find(g_srv_live.begin(), g_srv_live.end(), h) == g_srv_live.end()) g_srv_live.push_back(h);
  }
  return e;
}

extern "C" {

void srbd_qp_destroy(srbd_qp_handle h) {
  if (!h) return;
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  server_stop(h);
  if (h->srv_stream) hipStreamDestroy(h->srv_stream);
  if (h->srv_mb) hipHostFree(h->srv_mb);
  if (h->ws) hipFree(h->ws);
  if (h->stage) hipFree(h->stage);
  if (h->pinned) hipHostFree(h->pinned);
  if (h->pad) hipFree(h->pad);
  if (h->nmpc) hipFree(h->nmpc);
  if (h->nmpc_active_host) hipHostFree(h->nmpc_active_host);
  if (h->resc_idx) hipFree(h->resc_idx);
  if (h->resc) hipFree(h->resc);
  if (h->resc2) hipFree(h->resc2);
  if (h->mixed) hipFree(h->mixed);
  if (h->resc_count_host) hipHostFree(h->resc_count_host);
  if (h->fac_flags) hipHostFree(h->fac_flags);
  if (h->lat_flag) hipFree(h->lat_flag);
  if (h->lat_flag_host) hipHostFree(h->lat_flag_host);
  if (h->lqsw_idx) hipFree(h->lqsw_idx);
  if (h->lqsw) hipFree(h->lqsw);
  if (h->ctl) hipFree(h->ctl);
  if (h->qp_buf) hipFree(h->qp_buf);
  if (h->stream) hipStreamDestroy(h->stream);
  hipSetDevice(prev);
  delete h;
}

void* srbd_qp_stream(srbd_qp_handle h) { return h ? reinterpret_cast<void*>(h->stream) : nullptr; }

size_t srbd_qp_workspace_bytes(srbd_qp_handle h) { return h ? h->ws_bytes : 0; }

size_t srbd_qp_memory_bytes(srbd_qp_handle h) {
  if (!h) return 0;
  return h->ws_bytes + h->stage_bytes + h->pinned_bytes + h->pad_bytes + h->nmpc_bytes +
         (h->ctl ? sizeof(int) * srbd::kCtlInts : 0) +
         (h->qp_buf ? sizeof(int) * ((size_t)h->capacity + 1) : 0) +
         h->resc_bytes + h->resc2_bytes + h->mixed_bytes + h->lqsw_bytes +
         (h->resc_idx ? sizeof(int) * (2 * (size_t)h->capacity + 1) : 0) +
         (h->lqsw_idx ? sizeof(int) * (2 * (size_t)h->capacity + 1) : 0);
}

int srbd_qp_synchronize(srbd_qp_handle h) {
  if (!h) return fail(SRBD_QP_EINVAL, "handle is NULL");
  hipError_t e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("stream sync: ") + hipGetErrorString(e));
  return SRBD_QP_OK;
}

}  // extern "C"

template <typename DataT, typename SolT>
static int validate_call(srbd_qp_handle h, int batch, const srbd_qp_settings* st, const DataT* d,
                         const SolT* s) {
  if (!h) return fail(SRBD_QP_EINVAL, "handle is NULL");
  if (!d || !s) return fail(SRBD_QP_EINVAL, "data/solution is NULL");
  if (batch < 0) return fail(SRBD_QP_EINVAL, "batch must be >= 0");
  if (batch > h->capacity)
    return fail(SRBD_QP_ECAPACITY, "batch " + std::to_string(batch) + " exceeds capacity " +
                                       std::to_string(h->capacity));
  int rc = srbd_qp_check_settings(st);
  if (rc) return rc;
  if (!d->A || !d->B || !d->b || !d->Q || !d->S || !d->R || !d->q || !d->r || !d->x0)
    return fail(SRBD_QP_EINVAL, "A, B, b, Q, S, R, q, r and x0 are required");
  if (!s->x || !s->u || !s->pi) return fail(SRBD_QP_EINVAL, "x, u and pi outputs are required");
  const srbd_qp_dims& dm = h->dims;
  if ((d->lbu != nullptr) != (dm.has_box_u != 0) || (d->lbx != nullptr) != (dm.has_box_x != 0))
    return fail(SRBD_QP_EINVAL, "box-constraint pointers do not match the handle's dims");
  if (dm.ng > 0 && (!d->lg || !d->ug))
    return fail(SRBD_QP_EINVAL, "ng > 0 needs lg and ug (C, D and the masks are optional)");
  return SRBD_QP_OK;
}

static hipError_t rescue_f32(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                             const srbd_qp_data_f32* d, const srbd_qp_solution_f32* s,
                             const int* status, hipStream_t strm, int* rc);
static int mixed_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                     const srbd_qp_data_f64* d, const srbd_qp_solution_f64* s, hipStream_t strm);
static int fallback_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                        const srbd_qp_data_f64* d, const srbd_qp_solution_f64* sc,
                        const srbd_qp_solution_f64* s, hipStream_t strm, int min_status, int* idx,
                        int* count, void** buf, size_t* buf_bytes, const double* warm_x = nullptr,
                        const double* warm_u = nullptr);

// The launch arguments of a solve (solve_impl; the resident server's request).
template <typename T, typename DataT, typename SolT>
static srbd::ProblemArgsT<T> build_args(srbd_qp_handle h, int batch, const srbd_qp_settings* st, const DataT* d,
                                        const SolT* s, int* status, const T* warm_bars, int skip_last_rb) {
  srbd::ProblemArgsT<T> a;
  std::memset(&a, 0, sizeof a);  // (padding too: the resident server compares launches bytewise)
  a.batch = batch;
  a.N = h->dims.N;
  a.nx = h->dims.nx;
  a.nu = h->dims.nu;
  a.ng = h->dims.ng;
  a.layout = h->dims.layout;
  a.A = d->A; a.B = d->B; a.b = d->b; a.Q = d->Q; a.S = d->S; a.R = d->R; a.q = d->q; a.r = d->r;
  a.x0 = d->x0;
  a.lbu = d->lbu; a.ubu = d->ubu; a.lbu_mask = d->lbu_mask; a.ubu_mask = d->ubu_mask;
  a.lbx = d->lbx; a.ubx = d->ubx; a.lbx_mask = d->lbx_mask; a.ubx_mask = d->ubx_mask;
  a.C = d->C; a.D = d->D; a.lg = d->lg; a.ug = d->ug; a.lg_mask = d->lg_mask; a.ug_mask = d->ug_mask;
  a.x = s->x; a.u = s->u; a.pi = s->pi;
  a.P = s->P; a.p = s->p; a.K = s->K; a.k = s->k;
  a.status = status; a.iter = s->iter; a.res = s->res; a.obj = s->obj;
  a.stat = s->stat;
  a.ws = reinterpret_cast<T*>(h->ws);
  a.ws_qp = h->ws_qp;
  a.reg = st->reg_prim;
  a.iter_max = st->iter_max;
  a.stat_rows = st->iter_max + 2;
  a.warm_bars = warm_bars;
  a.skip_last_rb = skip_last_rb;
  a.pred_corr = st->pred_corr;
  a.split_step = st->split_step;
  a.ric_alg = st->ric_alg != 0;  // HPIPM: any nonzero square_root_alg
  // HPIPM's mode-dependent iterative refinement of the corrector (d_ocp_qp_ipm_arg_set_default:
  // itref_corr_max 2 in Balance, 4 in Robust, 0 in Speed / SpeedAbs)
  a.itref_corr_max = st->mode == 2 ? 2 : st->mode == 3 ? 4 : 0;
  // and its lq_fact: 1 in Balance, 2 in Robust, with the square-root Riccati only
  // ("for square_root_alg==1", hpipm_d_ocp_qp_ipm.h:78)
  a.lq_fact = !st->ric_alg ? 0 : st->lq_fact >= 0 ? st->lq_fact : st->mode == 2 ? 1 : st->mode == 3 ? 2 : 0;
  a.lq_redo = 0;
  a.warm_start = st->warm_start;
  a.alpha_min = st->alpha_min;
  a.mu0 = st->mu0;
  a.tol_stat = st->tol_stat;
  a.tol_eq = st->tol_eq;
  a.tol_ineq = st->tol_ineq;
  a.tol_comp = st->tol_comp;
  if constexpr (std::is_same_v<T, double>) a.factors_ready = h->fac_arm;
  if (h->ctl) {
    a.ctl = h->ctl;
    a.ctl_cap = srbd::kCtlCap;
    a.qp_buf = h->qp_buf;
  }
  return a;
}

// warm_bars: warm_start 2 only (the fp64 continuation of rescue_f32), see ProblemArgsT;
// iter_cap >= 0 (the f32_iters continuation): at most that many iterations, while the stat
// table keeps the caller's st->iter_max + 2 rows
template <typename T, typename DataT, typename SolT>
static int solve_impl(srbd_qp_handle h, int batch, const srbd_qp_settings* st, const DataT* d,
                      const SolT* s, void* stream, const T* warm_bars = nullptr,
                      int skip_last_rb = 0, int iter_cap = -1) {
  int rc = validate_call(h, batch, st, d, s);
  if (rc) return rc;
  if (batch == 0) return SRBD_QP_OK;
  hipStream_t strm = stream ? reinterpret_cast<hipStream_t>(stream) : h->stream;
  if constexpr (std::is_same_v<T, double>) {
    if (st->f32_iters > 0 && st->iter_max > 1 && constrained(h->dims) && h->dims.nx == 12 &&
        h->dims.nu == 12)
      return mixed_f64(h, batch, st, d, s, strm);
  }
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(h->device);
  // fp32 with f64_rescue: the status the fp32 pass leaves decides what is solved again
  const bool rescue = std::is_same_v<T, float> && st->f64_rescue && constrained(h->dims);
  if (rescue && !h->resc_idx) {
    hipError_t ea = hipMalloc(reinterpret_cast<void**>(&h->resc_idx),
                              sizeof(int) * (2 * (size_t)h->capacity + 1));
    if (ea == hipSuccess) ea = hipHostMalloc(reinterpret_cast<void**>(&h->resc_count_host), sizeof(int));
    if (ea != hipSuccess) {
      hipSetDevice(prev);
      return fail(SRBD_QP_ENOMEM, std::string("rescue buffers: ") + hipGetErrorString(ea));
    }
  }
  int* status = s->status;
  if (rescue && !status) status = h->resc_idx + h->capacity;
  srbd::ProblemArgsT<T> a = build_args<T>(h, batch, st, d, s, status, warm_bars, skip_last_rb);
  // f64_rescue = n: the fp32 pass stops after n iterations at most, the rest is fp64's
  if (rescue && st->f64_rescue < a.iter_max) a.iter_max = st->f64_rescue;
  if (iter_cap >= 0 && iter_cap < a.iter_max) a.iter_max = iter_cap;
  hipError_t e = hipSuccess;
  // (unconstrained with residuals: unconstr_residuals_kernel clears and fills the table)
  if (s->stat && (constrained(h->dims) || !st->compute_residuals))
    e = hipMemsetAsync(s->stat, 0,
                       sizeof(T) * srbd::kStatCols * (size_t)(st->iter_max + 2) * (size_t)batch, strm);
  // nx < 12 or nu < 12: solve the problem embedded in 12 x 12 stages
  const bool padded = a.nx != 12 || a.nu != 12;
  srbd::ProblemArgsT<T> run = a;
  if (e == hipSuccess && padded) {
    const size_t need = srbd::pad_elems(h->capacity, a.N, a.ng) * sizeof(T);
    if (need > h->pad_bytes) {
      if (h->pad) hipFree(h->pad);
      h->pad = nullptr;
      h->pad_bytes = 0;
      e = hipMalloc(&h->pad, need);
      if (e == hipSuccess) h->pad_bytes = need;
    }
    if (e == hipSuccess) e = srbd::pad_problem<T>(a, reinterpret_cast<T*>(h->pad), run, strm);
  }
  if (e != hipSuccess) {
  } else if (constrained(h->dims)) {
    // ric_alg 1 with lq_fact 1 (Balance's default) on the latency IPM: its predictor check may
    // ask for HPIPM's switch to the LQ factorization, which only the batched kernels have.  Such
    // a QP ends with status kLatNeedsLq and raises the flag; the call then waits once for the
    // flag and, if it is up, solves those QPs (and only those) again on the batched kernels, so
    // each QP ends as it does in any batch
    bool lq_watch = false;
    if constexpr (std::is_same_v<T, double>) {
      if (run.ric_alg && run.lq_fact == 1 && iter_cap < 0 && !h->force_batched) {
        if (!h->lat_flag) {
          e = hipMalloc(reinterpret_cast<void**>(&h->lat_flag), sizeof(int));
          if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&h->lat_flag_host), sizeof(int));
          if (e == hipSuccess)
            e = hipMalloc(reinterpret_cast<void**>(&h->lqsw_idx), sizeof(int) * (2 * (size_t)h->capacity + 1));
          if (e == hipSuccess && !h->resc_count_host)
            e = hipHostMalloc(reinterpret_cast<void**>(&h->resc_count_host), sizeof(int));
        }
        run.lat_lq_flag = e == hipSuccess ? h->lat_flag : nullptr;
        lq_watch = e == hipSuccess && srbd::ipm_latency_ok(run, srbd::ipm_latency_max_batch());
        if (!lq_watch) {
          run.lat_lq_flag = nullptr;
        } else {
          if (!a.status) a.status = run.status = h->lqsw_idx + h->capacity;
          e = hipMemsetAsync(h->lat_flag, 0, sizeof(int), strm);
        }
      }
      if (e == hipSuccess)
        e = h->force_batched ? srbd::launch_ipm_box_batched(run, strm) : srbd::launch_ipm_box(run, strm);
    } else {
      if (e == hipSuccess) e = srbd::launch_ipm_box(run, strm);
    }
    if (e == hipSuccess && padded) e = srbd::unpad_solution<T>(a, run, strm);
    if constexpr (std::is_same_v<T, double>) {
      if (e == hipSuccess && lq_watch) {
        e = hipMemcpyAsync(h->lat_flag_host, h->lat_flag, sizeof(int), hipMemcpyDeviceToHost, strm);
        if (e == hipSuccess) e = hipStreamSynchronize(strm);
        if (e == hipSuccess && *h->lat_flag_host) {
          SolT sc = *s;
          sc.status = a.status;
          hipSetDevice(prev);
          h->force_batched = true;
          rc = fallback_f64(h, batch, st, d, &sc, s, strm, srbd::kLatNeedsLq, h->lqsw_idx,
                            h->lqsw_idx + 2 * (size_t)h->capacity, &h->lqsw, &h->lqsw_bytes);
          h->force_batched = false;
          return rc;
        }
      }
    }
    if constexpr (std::is_same_v<T, float>) {
      if (e == hipSuccess && rescue) {
        hipSetDevice(prev);
        e = rescue_f32(h, batch, st, d, s, status, strm, &rc);
        if (rc) return rc;
        hipSetDevice(h->device);
      }
    }
  } else {
    // (the single-QP kernel computes the residuals itself when the problem is not embedded)
    run.fuse_res = st->compute_residuals && !padded;
    e = srbd::launch_riccati_unconstr(run, strm);
    if (e == hipSuccess && padded) e = srbd::unpad_solution<T>(a, run, strm);
    // residual norms / objective of the solution when asked for (HPIPM computes them
    // for nc = 0 too; an extra pass over the QP data, so only on request); the stat
    // table's row 0 gets them as well
    if (e == hipSuccess && (s->res || s->obj || s->stat) && !srbd::unconstr_fused_residuals(run)) {
      if (st->compute_residuals) {
        e = srbd::launch_unconstr_residuals<T>(a, strm);
      } else {
        if (s->res) e = hipMemsetAsync(s->res, 0, sizeof(T) * 4 * (size_t)batch, strm);
        if (e == hipSuccess && s->obj) e = hipMemsetAsync(s->obj, 0, sizeof(T) * (size_t)batch, strm);
      }
    }
  }
  hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("kernel launch: ") + hipGetErrorString(e));
  return SRBD_QP_OK;
}

// ---------------------------------------------------------------------------
// settings.f64_rescue: the QPs an fp32 pass left unsolved, solved again in fp64
// ---------------------------------------------------------------------------
static hipError_t rescue_f32(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                             const srbd_qp_data_f32* d, const srbd_qp_solution_f32* s,
                             const int* status, hipStream_t strm, int* rc) {
  *rc = SRBD_QP_OK;
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(h->device);
  int* idx = h->resc_idx;
  int* count = h->resc_idx + 2 * (size_t)h->capacity;
  hipError_t e = srbd::launch_select_unsolved(status, batch, 1, idx, count, strm);
  if (e == hipSuccess) e = hipMemcpyAsync(h->resc_count_host, count, sizeof(int), hipMemcpyDeviceToHost, strm);
  if (e == hipSuccess) e = hipStreamSynchronize(strm);
  const int R = e == hipSuccess ? *h->resc_count_host : 0;
  if (e != hipSuccess || R == 0) {
    hipSetDevice(prev);
    return e;
  }
  const srbd_qp_dims& m = h->dims;
  const size_t N = (size_t)m.N, nx = (size_t)m.nx, nu = (size_t)m.nu, ng = (size_t)m.ng;
  const size_t stat_e = srbd::kStatCols * (size_t)(st->iter_max + 2);
  // (fp32 source, values per QP) of every input the caller passed, then every output
  struct In { const float* src; size_t e; const double** dst; };
  struct Out { float* dst; size_t e; double** src; };
  srbd_qp_data_f64 d64{};
  srbd_qp_solution_f64 s64{};
  const In ins[] = {
      {d->A, N * nx * nx, &d64.A}, {d->B, N * nx * nu, &d64.B}, {d->b, N * nx, &d64.b},
      {d->Q, (N + 1) * nx * nx, &d64.Q}, {d->S, N * nu * nx, &d64.S}, {d->R, N * nu * nu, &d64.R},
      {d->q, (N + 1) * nx, &d64.q}, {d->r, N * nu, &d64.r}, {d->x0, nx, &d64.x0},
      {d->lbu, N * nu, &d64.lbu}, {d->ubu, N * nu, &d64.ubu}, {d->lbu_mask, N * nu, &d64.lbu_mask},
      {d->ubu_mask, N * nu, &d64.ubu_mask}, {d->lbx, (N + 1) * nx, &d64.lbx},
      {d->ubx, (N + 1) * nx, &d64.ubx}, {d->lbx_mask, (N + 1) * nx, &d64.lbx_mask},
      {d->ubx_mask, (N + 1) * nx, &d64.ubx_mask}, {d->C, (N + 1) * ng * nx, &d64.C},
      {d->D, N * ng * nu, &d64.D}, {d->lg, (N + 1) * ng, &d64.lg}, {d->ug, (N + 1) * ng, &d64.ug},
      {d->lg_mask, (N + 1) * ng, &d64.lg_mask}, {d->ug_mask, (N + 1) * ng, &d64.ug_mask}};
  const Out outs[] = {
      {s->x, (N + 1) * nx, &s64.x}, {s->u, N * nu, &s64.u}, {s->pi, (N + 1) * nx, &s64.pi},
      {s->P, (N + 1) * nx * nx, &s64.P}, {s->p, (N + 1) * nx, &s64.p}, {s->K, N * nu * nx, &s64.K},
      {s->k, N * nu, &s64.k}, {s->res, 4, &s64.res}, {s->obj, 1, &s64.obj}, {s->stat, stat_e, &s64.stat}};
  // fp64 continuation from the fp32 iterate (x, u, pi and the barrier state: HPIPM's
  // warm_start = 2) on 12 x 12 stages; a padded problem is re-solved cold
  const bool cont = m.nx == 12 && m.nu == 12;
  const size_t warm_e = cont ? (N + 1) * (96 + (size_t)((m.ng + 11) / 12) * 48) : 0;
  size_t per_qp = warm_e;  // doubles
  for (const In& f : ins) per_qp += f.src ? f.e : 0;
  for (const Out& f : outs) per_qp += f.dst ? f.e : 0;
  const size_t need = sizeof(double) * per_qp * (size_t)R + 2 * sizeof(int) * (size_t)R + 256;
  if (need > h->resc_bytes) {
    if (h->resc) hipFree(h->resc);
    h->resc = nullptr;
    h->resc_bytes = 0;
    e = hipMalloc(&h->resc, need);
    if (e != hipSuccess) {
      hipSetDevice(prev);
      *rc = fail(SRBD_QP_ENOMEM, std::string("rescue batch: ") + hipGetErrorString(e));
      return e;
    }
    h->resc_bytes = need;
  }
  double* cur = reinterpret_cast<double*>(h->resc);
  for (const In& f : ins) {
    if (!f.src || e != hipSuccess) continue;
    e = srbd::launch_gather_widen(f.src, cur, idx, R, f.e, strm);
    *f.dst = cur;
    cur += f.e * (size_t)R;
  }
  for (const Out& f : outs) {
    if (!f.dst) continue;
    *f.src = cur;
    cur += f.e * (size_t)R;
  }
  double* warm = cur;
  cur += warm_e * (size_t)R;
  s64.status = reinterpret_cast<int*>(cur);
  s64.iter = s64.status + R;
  if (cont && e == hipSuccess) {
    // the iterate the fp32 pass ended on: x, u, pi (caller's buffers), barrier state (its
    // workspace, read before the fp64 solve reuses that memory)
    e = srbd::launch_gather_widen(s->x, s64.x, idx, R, (N + 1) * nx, strm);
    if (e == hipSuccess) e = srbd::launch_gather_widen(s->u, s64.u, idx, R, N * nu, strm);
    if (e == hipSuccess) e = srbd::launch_gather_widen(s->pi, s64.pi, idx, R, (N + 1) * nx, strm);
    if (e == hipSuccess)
      e = srbd::launch_gather_warm_bars(reinterpret_cast<const float*>(h->ws), h->ws_qp, m.N, m.ng, idx,
                                        R, warm, strm);
  }
  hipSetDevice(prev);
  if (e != hipSuccess) return e;
  srbd_qp_settings st64 = *st;
  st64.warm_start = cont ? 2 : 0;
  st64.f64_rescue = 0;
  st64.f32_iters = 0;
  *rc = solve_impl<double>(h, R, &st64, &d64, &s64, strm, cont ? warm : nullptr);
  if (*rc) return hipSuccess;
  // A QP the continuation leaves unsolved (an fp32 pass can end far off, with the barrier
  // collapsed: t, lam -> 0 at a large stationarity residual, from where a warm-started IPM
  // does not recover) is solved again cold in fp64 (its own list, buffer and idx slots:
  // [capacity, 2 capacity) of resc_idx)
  if (cont) {
    *rc = fallback_f64(h, R, &st64, &d64, &s64, &s64, strm, 1, h->resc_idx + h->capacity,
                       h->resc_idx + 2 * (size_t)h->capacity, &h->resc2, &h->resc2_bytes);
    if (*rc) return hipSuccess;
  }
  hipSetDevice(h->device);
  for (const Out& f : outs)
    if (f.dst && e == hipSuccess) e = srbd::launch_scatter_narrow(*f.src, f.dst, idx, R, f.e, strm);
  if (e == hipSuccess && s->status) e = srbd::launch_scatter_int(s64.status, s->status, idx, R, strm);
  if (e == hipSuccess && s->iter) e = srbd::launch_scatter_int(s64.iter, s->iter, idx, R, strm);
  hipSetDevice(prev);
  return e;
}

// ---------------------------------------------------------------------------
// settings.f32_iters: mixed-precision IPM (fp32 iterations, then fp64 to the end)
// ---------------------------------------------------------------------------
// A QP a warm-started fp64 continuation ends with status >= min_status is solved again in
// fp64 (compact batch in *buf, list in idx) exactly as the plain fp64 call solves it: the
// caller's iter_max, and its x / u warm start when warm_x / warm_u are given (the caller's
// buffers as they were on entry), cold otherwise.  Both users pass min_status 1, so neither
// the mixed path (f32_iters) nor the rescue (f64_rescue) ends a QP worse than fp64 does.
static int fallback_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                        const srbd_qp_data_f64* d, const srbd_qp_solution_f64* sc,
                        const srbd_qp_solution_f64* s, hipStream_t strm, int min_status, int* idx,
                        int* count, void** buf, size_t* buf_bytes, const double* warm_x, const double* warm_u) {
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(h->device);
  hipError_t e = srbd::launch_select_unsolved(sc->status, batch, min_status, idx, count, strm);
  if (e == hipSuccess) e = hipMemcpyAsync(h->resc_count_host, count, sizeof(int), hipMemcpyDeviceToHost, strm);
  if (e == hipSuccess) e = hipStreamSynchronize(strm);
  const int R = e == hipSuccess ? *h->resc_count_host : 0;
  if (e != hipSuccess || R == 0) {
    hipSetDevice(prev);
    return e == hipSuccess ? SRBD_QP_OK : fail(SRBD_QP_EDEVICE, std::string("fallback: ") + hipGetErrorString(e));
  }
  const srbd_qp_dims& m = h->dims;
  const size_t N = (size_t)m.N, nx = (size_t)m.nx, nu = (size_t)m.nu, ng = (size_t)m.ng;
  struct In { const double* src; size_t e; const double** dst; };
  struct Out { double* dst; size_t e; double** src; };
  srbd_qp_data_f64 d2{};
  srbd_qp_solution_f64 s2{};
  const In ins[] = {
      {d->A, N * nx * nx, &d2.A}, {d->B, N * nx * nu, &d2.B}, {d->b, N * nx, &d2.b},
      {d->Q, (N + 1) * nx * nx, &d2.Q}, {d->S, N * nu * nx, &d2.S}, {d->R, N * nu * nu, &d2.R},
      {d->q, (N + 1) * nx, &d2.q}, {d->r, N * nu, &d2.r}, {d->x0, nx, &d2.x0},
      {d->lbu, N * nu, &d2.lbu}, {d->ubu, N * nu, &d2.ubu}, {d->lbu_mask, N * nu, &d2.lbu_mask},
      {d->ubu_mask, N * nu, &d2.ubu_mask}, {d->lbx, (N + 1) * nx, &d2.lbx},
      {d->ubx, (N + 1) * nx, &d2.ubx}, {d->lbx_mask, (N + 1) * nx, &d2.lbx_mask},
      {d->ubx_mask, (N + 1) * nx, &d2.ubx_mask}, {d->C, (N + 1) * ng * nx, &d2.C},
      {d->D, N * ng * nu, &d2.D}, {d->lg, (N + 1) * ng, &d2.lg}, {d->ug, (N + 1) * ng, &d2.ug},
      {d->lg_mask, (N + 1) * ng, &d2.lg_mask}, {d->ug_mask, (N + 1) * ng, &d2.ug_mask}};
  const Out outs[] = {
      {s->x, (N + 1) * nx, &s2.x}, {s->u, N * nu, &s2.u}, {s->pi, (N + 1) * nx, &s2.pi},
      {s->P, (N + 1) * nx * nx, &s2.P}, {s->p, (N + 1) * nx, &s2.p}, {s->K, N * nu * nx, &s2.K},
      {s->k, N * nu, &s2.k}, {s->res, 4, &s2.res}, {s->obj, 1, &s2.obj},
      {s->stat, srbd::kStatCols * (size_t)(st->iter_max + 2), &s2.stat}};
  size_t per_qp = 0;
  for (const In& f : ins) per_qp += f.src ? f.e : 0;
  for (const Out& f : outs) per_qp += f.dst ? f.e : 0;
  const size_t need = sizeof(double) * per_qp * (size_t)R + 2 * sizeof(int) * (size_t)R + 256;
  if (need > *buf_bytes) {
    if (*buf) hipFree(*buf);
    *buf = nullptr;
    *buf_bytes = 0;
    e = hipMalloc(buf, need);
    if (e != hipSuccess) {
      hipSetDevice(prev);
      return fail(SRBD_QP_ENOMEM, std::string("fallback batch: ") + hipGetErrorString(e));
    }
    *buf_bytes = need;
  }
  double* cur = reinterpret_cast<double*>(*buf);
  for (const In& f : ins) {
    if (!f.src || e != hipSuccess) continue;
    e = srbd::launch_gather_rows(f.src, cur, idx, R, f.e, strm);
    *f.dst = cur;
    cur += f.e * (size_t)R;
  }
  for (const Out& f : outs) {
    if (!f.dst) continue;
    *f.src = cur;
    cur += f.e * (size_t)R;
  }
  s2.status = reinterpret_cast<int*>(cur);
  s2.iter = s2.status + R;
  const bool warm = warm_x && warm_u && st->warm_start;
  if (warm && e == hipSuccess) e = srbd::launch_gather_rows(warm_x, s2.x, idx, R, (N + 1) * nx, strm);
  if (warm && e == hipSuccess) e = srbd::launch_gather_rows(warm_u, s2.u, idx, R, N * nu, strm);
  hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("fallback: ") + hipGetErrorString(e));
  srbd_qp_settings st2 = *st;
  st2.warm_start = warm ? st->warm_start : 0;
  st2.f32_iters = 0;
  int rc = solve_impl<double>(h, R, &st2, &d2, &s2, strm);
  if (rc) return rc;
  hipSetDevice(h->device);
  for (const Out& f : outs)
    if (f.dst && e == hipSuccess) e = srbd::launch_scatter_rows(*f.src, f.dst, idx, R, f.e, strm);
  if (e == hipSuccess) e = srbd::launch_scatter_int(s2.status, sc->status, idx, R, strm);
  if (e == hipSuccess && s->iter) e = srbd::launch_scatter_int(s2.iter, s->iter, idx, R, strm);
  hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("fallback: ") + hipGetErrorString(e));
  return SRBD_QP_OK;
}

static int mixed_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                     const srbd_qp_data_f64* d, const srbd_qp_solution_f64* s, hipStream_t strm) {
  const srbd_qp_dims& m = h->dims;
  const size_t B = (size_t)batch, N = (size_t)m.N, nx = (size_t)m.nx, nu = (size_t)m.nu,
               ng = (size_t)m.ng;
  srbd_qp_data_f32 d32{};
  struct F { const double* src; size_t e; const float** dst; };
  const F ins[] = {
      {d->A, N * nx * nx, &d32.A}, {d->B, N * nx * nu, &d32.B}, {d->b, N * nx, &d32.b},
      {d->Q, (N + 1) * nx * nx, &d32.Q}, {d->S, N * nu * nx, &d32.S}, {d->R, N * nu * nu, &d32.R},
      {d->q, (N + 1) * nx, &d32.q}, {d->r, N * nu, &d32.r}, {d->x0, nx, &d32.x0},
      {d->lbu, N * nu, &d32.lbu}, {d->ubu, N * nu, &d32.ubu}, {d->lbu_mask, N * nu, &d32.lbu_mask},
      {d->ubu_mask, N * nu, &d32.ubu_mask}, {d->lbx, (N + 1) * nx, &d32.lbx},
      {d->ubx, (N + 1) * nx, &d32.ubx}, {d->lbx_mask, (N + 1) * nx, &d32.lbx_mask},
      {d->ubx_mask, (N + 1) * nx, &d32.ubx_mask}, {d->C, (N + 1) * ng * nx, &d32.C},
      {d->D, N * ng * nu, &d32.D}, {d->lg, (N + 1) * ng, &d32.lg}, {d->ug, (N + 1) * ng, &d32.ug},
      {d->lg_mask, (N + 1) * ng, &d32.lg_mask}, {d->ug_mask, (N + 1) * ng, &d32.ug_mask}};
  const size_t ex = (N + 1) * nx, eu = N * nu;
  const size_t warm_e = (N + 1) * (96 + (size_t)((m.ng + 11) / 12) * 48);
  size_t floats = 2 * ex + eu;  // per QP: x, u, pi
  for (const F& f : ins) floats += f.src ? f.e : 0;
  // warm_start: the caller's x / u as they are on entry (the fp64 fallback starts from them)
  const size_t keep_e = st->warm_start ? ex + eu : 0;
  const size_t need = B * (floats * sizeof(float) + (warm_e + keep_e) * sizeof(double)) + 512;
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(h->device);
  hipError_t e = hipSuccess;
  if (need > h->mixed_bytes) {
    if (h->mixed) hipFree(h->mixed);
    h->mixed = nullptr;
    h->mixed_bytes = 0;
    e = hipMalloc(&h->mixed, need);
    if (e != hipSuccess) {
      hipSetDevice(prev);
      return fail(SRBD_QP_ENOMEM, std::string("mixed-precision buffers: ") + hipGetErrorString(e));
    }
    h->mixed_bytes = need;
  }
  double* warm = reinterpret_cast<double*>(h->mixed);
  double* keep_x = keep_e ? warm + B * warm_e : nullptr;
  double* keep_u = keep_e ? keep_x + B * ex : nullptr;
  float* cur = reinterpret_cast<float*>(warm + B * (warm_e + keep_e));
  if (keep_e) {
    e = hipMemcpyAsync(keep_x, s->x, sizeof(double) * B * ex, hipMemcpyDeviceToDevice, strm);
    if (e == hipSuccess) e = hipMemcpyAsync(keep_u, s->u, sizeof(double) * B * eu, hipMemcpyDeviceToDevice, strm);
  }
  for (const F& f : ins) {
    if (!f.src || e != hipSuccess) continue;
    e = srbd::launch_narrow(f.src, cur, f.e * B, strm);
    *f.dst = cur;
    cur += f.e * B;
  }
  srbd_qp_solution_f32 s32{};
  s32.x = cur;
  s32.u = cur + ex * B;
  s32.pi = cur + (ex + eu) * B;
  if (e == hipSuccess && st->warm_start) {
    e = srbd::launch_narrow(s->x, s32.x, ex * B, strm);
    if (e == hipSuccess) e = srbd::launch_narrow(s->u, s32.u, eu * B, strm);
  }
  hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("mixed precision: ") + hipGetErrorString(e));
  // fp32 iterations: tolerances out of reach, so every QP runs them all (a QP that stops
  // early on NaN / min step continues cold in fp64: its iterate fails the finiteness test
  // or is simply where it stopped).  They count against iter_max: n = min(f32_iters,
  // iter_max - 1) fp32 iterations, then at most iter_max - n fp64 ones.
  const int n32 = st->f32_iters < st->iter_max - 1 ? st->f32_iters : st->iter_max - 1;
  srbd_qp_settings st32 = *st;
  st32.iter_max = n32;
  st32.tol_stat = st32.tol_eq = st32.tol_ineq = st32.tol_comp = 1e-30;
  st32.f64_rescue = 0;
  st32.f32_iters = 0;
  // (the loop ends after the last corrector step; its application rides on the widening)
  int rc = solve_impl<float>(h, batch, &st32, &d32, &s32, strm, nullptr, 1);
  if (rc) return rc;
  hipSetDevice(h->device);
  e = srbd::launch_gather_warm_apply(reinterpret_cast<const float*>(h->ws), h->ws_qp, m.N, m.ng, batch,
                                     s32.x, s32.u, s32.pi, s->x, s->u, s->pi, warm, strm);
  hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("mixed precision: ") + hipGetErrorString(e));
  srbd_qp_settings st64 = *st;
  st64.warm_start = 2;
  st64.f32_iters = 0;
  if (!h->resc_idx) {
    hipSetDevice(h->device);
    e = hipMalloc(reinterpret_cast<void**>(&h->resc_idx), sizeof(int) * (2 * (size_t)h->capacity + 1));
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&h->resc_count_host), sizeof(int));
    hipSetDevice(prev);
    if (e != hipSuccess) return fail(SRBD_QP_ENOMEM, std::string("fallback buffers: ") + hipGetErrorString(e));
  }
  srbd_qp_solution_f64 sc = *s;
  if (!sc.status) sc.status = h->resc_idx + h->capacity;
  rc = solve_impl<double>(h, batch, &st64, d, &sc, strm, warm, 0, st->iter_max - n32);
  if (rc) return rc;
  return fallback_f64(h, batch, st, d, &sc, s, strm, 1, h->resc_idx, h->resc_idx + 2 * (size_t)h->capacity,
                      &h->resc, &h->resc_bytes, keep_x, keep_u);
}

// ---------------------------------------------------------------------------
// host-buffer convenience path
// ---------------------------------------------------------------------------
namespace {
// one polling step of the zero-copy wait: a pause hint where the host has one
inline void spin_pause() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}
// The single-QP launch is a few tens of microseconds: the zero-copy host solve polls for it
// (the blocking wait's wake-up costs about as much as the kernel), for at most this long; a
// longer solve (or a hung one) falls back to the blocking wait, so no host core spins for more.
constexpr auto kSpinBudget = std::chrono::milliseconds(2);
// flags of srbd_qp_solve_host_cb_f64's early factors: the single-QP kernels' batch limit
constexpr int kFacFlagsMax = 256;
// host solves whose staged bytes fit this go through the handle's pinned buffer
constexpr size_t kPinnedMaxBytes = size_t(8) << 20;
struct Field {
  const void* host;
  size_t bytes;
  size_t off;
};
}  // namespace

// stage_d / stage_s set (srbd_qp_host_staging_*): only lay out the pinned staging buffer for
// the fields d / s mark and return pointers into it, so a caller can pack its QPs in place.
// A host pointer that already is its field's place in the staging buffer is not copied.
// on_factors (srbd_qp_solve_host_cb_f64): called once, on success, as soon as P, p, K, k are
// in the caller's buffers -- mid-kernel on the zero-copy single-QP path, else at the end.
template <typename T, typename DataT, typename SolT>
static int solve_host_impl(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                           const DataT* d, const SolT* s, DataT* stage_d = nullptr,
                           SolT* stage_s = nullptr, void (*on_factors)(void*) = nullptr,
                           void* ctx = nullptr) {
  int rc = validate_call(h, batch, st, d, s);
  if (rc) return rc;
  if (batch == 0) return SRBD_QP_OK;
  const srbd_qp_dims& m = h->dims;
  const size_t B = (size_t)batch, N = (size_t)m.N, nx = (size_t)m.nx, nu = (size_t)m.nu,
               ng = (size_t)m.ng;
  const size_t D = sizeof(T);
  // input fields
  std::vector<Field> in;
  size_t off = 0;
  auto add = [&](const T* p, size_t n) -> size_t {
    if (!p) return (size_t)-1;
    size_t o = off;
    in.push_back({p, n * D, o});
    off += ((n * D + 255) / 256) * 256;
    return o;
  };
  size_t oA = add(d->A, B * N * nx * nx), oB = add(d->B, B * N * nx * nu), ob = add(d->b, B * N * nx);
  size_t oQ = add(d->Q, B * (N + 1) * nx * nx), oS = add(d->S, B * N * nu * nx),
         oR = add(d->R, B * N * nu * nu);
  size_t oq = add(d->q, B * (N + 1) * nx), orr = add(d->r, B * N * nu), ox0 = add(d->x0, B * nx);
  size_t olbu = add(d->lbu, B * N * nu), oubu = add(d->ubu, B * N * nu),
         olbum = add(d->lbu_mask, B * N * nu), oubum = add(d->ubu_mask, B * N * nu);
  size_t olbx = add(d->lbx, B * (N + 1) * nx), oubx = add(d->ubx, B * (N + 1) * nx),
         olbxm = add(d->lbx_mask, B * (N + 1) * nx), oubxm = add(d->ubx_mask, B * (N + 1) * nx);
  size_t oC = add(d->C, B * (N + 1) * ng * nx), oD = add(d->D, B * N * ng * nu),
         olg = add(d->lg, B * (N + 1) * ng), oug = add(d->ug, B * (N + 1) * ng),
         olgm = add(d->lg_mask, B * (N + 1) * ng), ougm = add(d->ug_mask, B * (N + 1) * ng);
  // outputs
  struct OutF {
    void* host;
    size_t bytes;
    size_t off;
  };
  std::vector<OutF> outs;
  auto addo = [&](void* p, size_t bytes) -> size_t {
    if (!p) return (size_t)-1;
    size_t o = off;
    outs.push_back({p, bytes, o});
    off += ((bytes + 255) / 256) * 256;
    return o;
  };
  size_t ox = addo(s->x, B * (N + 1) * nx * D), ou = addo(s->u, B * N * nu * D),
         opi = addo(s->pi, B * (N + 1) * nx * D);
  size_t oP = addo(s->P, B * (N + 1) * nx * nx * D), op = addo(s->p, B * (N + 1) * nx * D),
         oK = addo(s->K, B * N * nu * nx * D), ok = addo(s->k, B * N * nu * D);
  size_t ost = addo(s->status, B * sizeof(int)), oit = addo(s->iter, B * sizeof(int));
  size_t ores = addo(s->res, B * 4 * D), oobj = addo(s->obj, B * D);
  size_t ostat = addo(s->stat, B * srbd::kStatCols * (size_t)(st->iter_max + 2) * D);

  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(h->device);
  hipError_t e = hipSuccess;
  if (off > h->stage_bytes) {
    if (h->stage) hipFree(h->stage);
    h->stage = nullptr;
    h->stage_bytes = 0;
    e = hipMalloc(reinterpret_cast<void**>(&h->stage), off);
    if (e == hipSuccess) h->stage_bytes = off;
  }
  char* base = reinterpret_cast<char*>(h->stage);
  // Small problems go through a pinned mirror of the staging buffer: the fields are
  // packed with memcpy and cross PCIe in one DMA each way (per-field pageable copies
  // cost ~10 us of driver latency apiece).  Large ones copy field by field: the
  // pageable path streams at PCIe rate with no extra host pass over the data.
  const size_t in_end = outs.empty() ? off : outs.front().off;
  const bool small = off <= kPinnedMaxBytes;
  char* pin = nullptr;
  if (e == hipSuccess && small) {
    if (off > h->pinned_bytes) {
      server_stop(h);  // (it holds pointers into the old buffer)
      if (h->pinned) hipHostFree(h->pinned);
      h->pinned = nullptr;
      h->pinned_bytes = 0;
      e = hipHostMalloc(&h->pinned, off);
      if (e == hipSuccess) h->pinned_bytes = off;
    }
    pin = reinterpret_cast<char*>(h->pinned);
  }
  if (stage_d) {
    hipSetDevice(prev);
    if (e != hipSuccess)
      return fail(SRBD_QP_ENOMEM, std::string("host staging: ") + hipGetErrorString(e));
    if (!small) return fail(SRBD_QP_ECAPACITY, "host staging: the batch's buffers exceed the pinned staging size");
    auto hp = [&](size_t o) -> T* { return o == (size_t)-1 ? nullptr : reinterpret_cast<T*>(pin + o); };
    auto hi = [&](size_t o) -> int* { return o == (size_t)-1 ? nullptr : reinterpret_cast<int*>(pin + o); };
    DataT& dd = *stage_d;
    dd = DataT{};
    dd.A = hp(oA); dd.B = hp(oB); dd.b = hp(ob); dd.Q = hp(oQ); dd.S = hp(oS); dd.R = hp(oR);
    dd.q = hp(oq); dd.r = hp(orr); dd.x0 = hp(ox0);
    dd.lbu = hp(olbu); dd.ubu = hp(oubu); dd.lbu_mask = hp(olbum); dd.ubu_mask = hp(oubum);
    dd.lbx = hp(olbx); dd.ubx = hp(oubx); dd.lbx_mask = hp(olbxm); dd.ubx_mask = hp(oubxm);
    dd.C = hp(oC); dd.D = hp(oD); dd.lg = hp(olg); dd.ug = hp(oug); dd.lg_mask = hp(olgm);
    dd.ug_mask = hp(ougm);
    SolT& ss = *stage_s;
    ss = SolT{};
    ss.x = hp(ox); ss.u = hp(ou); ss.pi = hp(opi); ss.P = hp(oP); ss.p = hp(op); ss.K = hp(oK);
    ss.k = hp(ok); ss.status = hi(ost); ss.iter = hi(oit); ss.res = hp(ores); ss.obj = hp(oobj);
    ss.stat = hp(ostat);
    return SRBD_QP_OK;
  }
  // Zero copy: when the launch reads each QP's data exactly once (the single-QP kernel's
  // copy into LDS) and writes each output once, the kernel reads the pinned staging buffer
  // over PCIe and writes its outputs straight into it -- no DMA either way, one launch, one
  // wait (the reference's one-QP-per-solve() call pattern, NMPC_solver.cpp:316-330).
  bool zero_copy = false;
  if (e == hipSuccess && small && !constrained(m)) {
    srbd::ProblemArgsT<T> probe{};
    probe.batch = batch;
    probe.N = m.N;
    probe.nx = m.nx;
    probe.nu = m.nu;
    probe.layout = m.layout;
    probe.fuse_res = st->compute_residuals;
    T dummy = T(0);
    probe.res = s->res ? &dummy : nullptr;
    probe.obj = s->obj ? &dummy : nullptr;
    probe.stat = s->stat ? &dummy : nullptr;
    zero_copy = srbd::unconstr_reads_once(probe);
  }
  if (zero_copy) {
    void* dev = nullptr;
    e = hipHostGetDevicePointer(&dev, pin, 0);
    if (e == hipSuccess) base = reinterpret_cast<char*>(dev);
  }
  // early factors: the latency kernel sets fac_flags[qp] once the QP's P, p, K, k are written
  // (system scope), and the caller's callback runs on them while the kernel finishes
  bool arm = false;
  if constexpr (std::is_same_v<T, double>) {
    if (e == hipSuccess && zero_copy && on_factors && (s->P || s->p || s->K || s->k)) {
      if (!h->fac_flags)
        e = hipHostMalloc(reinterpret_cast<void**>(&h->fac_flags), sizeof(int) * kFacFlagsMax,
                          hipHostMallocCoherent | hipHostMallocMapped);
      void* dev = nullptr;
      if (e == hipSuccess) e = hipHostGetDevicePointer(&dev, h->fac_flags, 0);
      if (e == hipSuccess && batch <= kFacFlagsMax) {
        for (int i = 0; i < batch; ++i) reinterpret_cast<volatile int*>(h->fac_flags)[i] = 0;
        h->fac_arm = reinterpret_cast<int*>(dev);
        arm = true;
      }
    }
  }
  if (e == hipSuccess && small) {
    for (const Field& f : in)
      if (f.host != pin + f.off) std::memmove(pin + f.off, f.host, f.bytes);  // (staged in place: no copy)
    if (!zero_copy) e = hipMemcpyAsync(base, pin, in_end, hipMemcpyHostToDevice, h->stream);
  }
  for (size_t i = 0; !small && e == hipSuccess && i < in.size(); ++i)
    e = hipMemcpyAsync(base + in[i].off, in[i].host, in[i].bytes, hipMemcpyHostToDevice, h->stream);
  // warm start: x/u outputs are inputs too
  if (e == hipSuccess && st->warm_start) {
    const size_t bx = B * (N + 1) * nx * D, bu = B * N * nu * D;
    if (small) {
      if ((const void*)s->x != pin + ox) std::memmove(pin + ox, s->x, bx);
      if ((const void*)s->u != pin + ou) std::memmove(pin + ou, s->u, bu);
      // x and u are adjacent in the staging layout (addo order, 256-byte aligned)
      if (!zero_copy) e = hipMemcpyAsync(base + ox, pin + ox, ou + bu - ox, hipMemcpyHostToDevice, h->stream);
    } else {
      e = hipMemcpyAsync(base + ox, s->x, bx, hipMemcpyHostToDevice, h->stream);
      if (e == hipSuccess) e = hipMemcpyAsync(base + ou, s->u, bu, hipMemcpyHostToDevice, h->stream);
    }
  }
  if (e != hipSuccess) {
    // an earlier copy from the pinned buffer may still be queued: drain the stream before
    // the next call may overwrite (or free) that buffer
    hipStreamSynchronize(h->stream);
    hipSetDevice(prev);
    return fail(SRBD_QP_EDEVICE, std::string("host->device copy: ") + hipGetErrorString(e));
  }
  auto dp = [&](size_t o) -> T* {
    return o == (size_t)-1 ? nullptr : reinterpret_cast<T*>(base + o);
  };
  auto ip = [&](size_t o) -> int* { return o == (size_t)-1 ? nullptr : reinterpret_cast<int*>(base + o); };
  DataT dd{};
  dd.A = dp(oA); dd.B = dp(oB); dd.b = dp(ob); dd.Q = dp(oQ); dd.S = dp(oS); dd.R = dp(oR);
  dd.q = dp(oq); dd.r = dp(orr); dd.x0 = dp(ox0);
  dd.lbu = dp(olbu); dd.ubu = dp(oubu); dd.lbu_mask = dp(olbum); dd.ubu_mask = dp(oubum);
  dd.lbx = dp(olbx); dd.ubx = dp(oubx); dd.lbx_mask = dp(olbxm); dd.ubx_mask = dp(oubxm);
  dd.C = dp(oC); dd.D = dp(oD); dd.lg = dp(olg); dd.ug = dp(oug); dd.lg_mask = dp(olgm);
  dd.ug_mask = dp(ougm);
  SolT ss{};
  ss.x = dp(ox); ss.u = dp(ou); ss.pi = dp(opi); ss.P = dp(oP); ss.p = dp(op); ss.K = dp(oK);
  ss.k = dp(ok); ss.status = ip(ost); ss.iter = ip(oit); ss.res = dp(ores); ss.obj = dp(oobj);
  ss.stat = dp(ostat);
  // One QP that the latency kernel would solve in place: post it to the resident server
  // instead of launching (no launch, dispatch or completion-signal latency).
  bool served = false;
  if constexpr (std::is_same_v<T, double>) {
    if (zero_copy && batch == 1 && server_enabled()) {
      const srbd::ProblemArgsT<double> a = build_args<double>(h, batch, st, &dd, &ss, ss.status, nullptr, 0);
      srbd::ProblemArgsT<double> ar = a;
      ar.fuse_res = st->compute_residuals;  // (not embedded: nx = nu = 12)
      served = srbd::latency_server_ok(ar);
      // the early-factor flags: a fixed pointer for the server's life, switched per request
      // through the mailbox (LatMailbox::arm), so callback and plain calls share one server
      if (served && !h->fac_flags) {
        if (hipHostMalloc(reinterpret_cast<void**>(&h->fac_flags), sizeof(int) * kFacFlagsMax,
                          hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
          h->fac_flags = nullptr;
      }
      void* fdev = nullptr;
      if (served && (!h->fac_flags || hipHostGetDevicePointer(&fdev, h->fac_flags, 0) != hipSuccess)) fdev = nullptr;
      ar.factors_ready = reinterpret_cast<int*>(fdev);
      if (served && arm && !fdev) served = false;  // (cannot happen: arm allocated the flags)
      if (served) {
        // the handle's workspace: earlier work queued on its stream finishes first
        if (hipStreamQuery(h->stream) != hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e == hipSuccess && h->srv_live && std::memcmp(&ar, &h->srv_args, sizeof ar) != 0) server_stop(h);
        if (e == hipSuccess &&
            (!h->srv_live || reinterpret_cast<volatile srbd::LatMailbox*>(h->srv_mb)->exited == h->srv_epoch))
          e = server_launch(h, ar, h->srv_seq);  // (before the post: nothing pending)
        volatile srbd::LatMailbox* mb = h->srv_mb;
        if (e == hipSuccess) {
          if (const int us = server_post_delay_us()) std::this_thread::sleep_for(std::chrono::microseconds(us));
          std::atomic_thread_fence(std::memory_order_release);  // the staged QP before the post
          // seq and the request's flags in one 8-byte store (the server reads them as one word)
          const unsigned long long post =
              ((unsigned long long)(unsigned)(arm ? srbd::kLatArm : 0) << 32) | (unsigned)++h->srv_seq;
          *reinterpret_cast<volatile unsigned long long*>(mb) = post;
        }
      }
    }
  }
  if (!served) {
    hipSetDevice(prev);
    rc = solve_impl<T>(h, batch, st, &dd, &ss, nullptr);
    if (rc) {
      h->fac_arm = nullptr;
      // copies from the pinned buffer may still be queued: the next call must not
      // overwrite (or free) it under a pending DMA
      hipStreamSynchronize(h->stream);
      return rc;
    }
    hipSetDevice(h->device);
  }
  h->fac_arm = nullptr;
  if (small) {
    if (e == hipSuccess && in_end < off && !zero_copy)
      e = hipMemcpyAsync(pin + in_end, base + in_end, off - in_end, hipMemcpyDeviceToHost, h->stream);
    // poll for the single-QP launch for at most kSpinBudget, then block (spin_pause above)
    auto is_fac = [&](size_t o) { return o == oP || o == op || o == oK || o == ok; };
    bool fired = false;
    int seen = 0;  // QPs whose early-factor flag is up
    auto factors_check = [&]() {
      if (!arm || fired) return false;
      const volatile int* f = h->fac_flags;
      while (seen < batch && f[seen]) ++seen;
      if (seen < batch) return false;
      std::atomic_thread_fence(std::memory_order_acquire);
      for (const OutF& o : outs)
        if (is_fac(o.off) && o.host != pin + o.off) std::memmove(o.host, pin + o.off, o.bytes);
      on_factors(ctx);
      fired = true;
      return true;
    };
    if (e == hipSuccess && served) {
      // wait for the server's answer; it may have left (idle) just before the post: relaunch
      volatile srbd::LatMailbox* mb = h->srv_mb;
      const auto t_end = std::chrono::steady_clock::now() + kServerTimeout;
      for (unsigned n = 1; e == hipSuccess && mb->done != h->srv_seq; ++n) {
        if (factors_check()) continue;
        if (mb->exited == h->srv_epoch) {
          // the server left: it writes `done` before `exited`, so read `done` again -- it may
          // have answered this request before leaving (then a relaunch would solve it twice,
          // the second time under the next call's packing)
          std::atomic_thread_fence(std::memory_order_acquire);
          if (mb->done == h->srv_seq) break;
          // it left before seeing the post: the request is still pending
          e = server_launch(h, h->srv_args, h->srv_seq - 1);
          continue;
        }
        if ((n & 1023) == 0) {
          const hipError_t q = hipStreamQuery(h->srv_stream);
          if (q != hipSuccess && q != hipErrorNotReady) e = q;
          if (e == hipSuccess && std::chrono::steady_clock::now() > t_end) e = hipErrorLaunchTimeOut;
        }
        spin_pause();
      }
      std::atomic_thread_fence(std::memory_order_acquire);
      if (e != hipSuccess) server_stop(h);  // leave no server behind a failed request
    }
    if (e == hipSuccess && zero_copy && !served) {
      const auto t_end = std::chrono::steady_clock::now() + kSpinBudget;
      hipError_t q;
      while ((q = hipStreamQuery(h->stream)) == hipErrorNotReady && std::chrono::steady_clock::now() < t_end) {
        if (factors_check()) continue;
        spin_pause();
      }
      if (q != hipSuccess && q != hipErrorNotReady) e = q;
    }
    if (e == hipSuccess && !served) e = hipStreamSynchronize(h->stream);
    for (size_t i = 0; e == hipSuccess && i < outs.size(); ++i)
      if (outs[i].host != pin + outs[i].off && !(fired && is_fac(outs[i].off)))
        std::memmove(outs[i].host, pin + outs[i].off, outs[i].bytes);
    if (e == hipSuccess && on_factors && !fired) on_factors(ctx);
  } else {
    for (size_t i = 0; e == hipSuccess && i < outs.size(); ++i)
      e = hipMemcpyAsync(outs[i].host, base + outs[i].off, outs[i].bytes, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess && on_factors) on_factors(ctx);
  }
  hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("device->host copy: ") + hipGetErrorString(e));
  return SRBD_QP_OK;
}

extern "C" {

int srbd_qp_solve_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                      const srbd_qp_data_f64* d, const srbd_qp_solution_f64* s, void* stream) {
  return solve_impl<double>(h, batch, st, d, s, stream);
}
int srbd_qp_solve_host_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                           const srbd_qp_data_f64* d, const srbd_qp_solution_f64* s) {
  return solve_host_impl<double>(h, batch, st, d, s);
}
int srbd_qp_solve_host_cb_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                              const srbd_qp_data_f64* d, const srbd_qp_solution_f64* s,
                              void (*on_factors)(void* ctx), void* ctx) {
  return solve_host_impl<double, srbd_qp_data_f64, srbd_qp_solution_f64>(h, batch, st, d, s, nullptr, nullptr,
                                                                       on_factors, ctx);
}
int srbd_qp_host_staging_f64(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                             srbd_qp_data_f64* d, srbd_qp_solution_f64* s) {
  if (!d || !s) return fail(SRBD_QP_EINVAL, "host staging: data / solution struct is NULL");
  const srbd_qp_data_f64 want = *d;
  const srbd_qp_solution_f64 want_s = *s;
  return solve_host_impl<double>(h, batch, st, &want, &want_s, d, s);
}
void srbd_qp_srbd_default_params(srbd_model_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  const double Q[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 10};
  const double Qf[12] = {0.5, 0.5, 0.5, 0.01, 0.01, 0.01, 100, 100, 100, 0.0, 0.0, 100.0};
  const double xr[12] = {0, 0, 0.2, 0, 0, 0, 0.5, 0, 1.0, 0, 0, 0};
  const double lo[6] = {-50.0, -50.0, 0.0, -5.0, -5.0, -5.0}, hi[6] = {50.0, 50.0, 300.0, 5.0, 5.0, 5.0};
  for (int i = 0; i < 12; ++i) {
    p->Q[i] = Q[i];
    p->Qf[i] = Qf[i];
    p->x_ref[i] = xr[i];
    p->u_lo[i] = lo[i % 6];
    p->u_hi[i] = hi[i % 6];
  }
  p->R = 0.0001;
  p->dt = 0.015;
  p->Lbody[0] = 0.541667;
  p->Lbody[1] = 0.516667;
  p->Lbody[2] = 1.0416667;
  p->mu_b = 0.1;
  p->theta_b = 5.0;
  p->mass = 15.0;
  p->foot_r[1] = -0.1;
  p->foot_l[1] = 0.1;
  p->mu = 0.5;
  p->Lfx = 0.05;
  p->Lfz = 0.05;
  p->fmax = 1000.0;
  p->fmin = 0.0;
  p->qf_scale = 0.0;  // N
}

int srbd_qp_srbd_linearize_f64(srbd_qp_handle h, int batch, const srbd_model_params* params,
                               int constraints, const double* xs, const double* us,
                               const srbd_qp_data_f64* out, void* stream) {
  if (!h || !params || !xs || !us || !out) return fail(SRBD_QP_EINVAL, "NULL argument");
  const srbd_qp_dims& d = h->dims;
  if (d.nx != 12 || d.nu != 12) return fail(SRBD_QP_EDIM, "SRBD linearisation needs nx = nu = 12");
  if (batch < 0 || batch > h->capacity) return fail(SRBD_QP_ECAPACITY, "batch exceeds capacity");
  if (constraints < SRBD_QP_SRBD_NONE || constraints > SRBD_QP_SRBD_CONE)
    return fail(SRBD_QP_EINVAL, "unknown constraints mode");
  if (!out->A || !out->B || !out->b || !out->Q || !out->S || !out->R || !out->q || !out->r)
    return fail(SRBD_QP_EINVAL, "A, B, b, Q, S, R, q, r outputs are required");
  if (constraints == SRBD_QP_SRBD_BOX_U && (!out->lbu || !out->ubu))
    return fail(SRBD_QP_EINVAL, "BOX_U needs lbu / ubu outputs");
  if (constraints == SRBD_QP_SRBD_CONE &&
      (d.ng != 24 || !out->D || !out->lg || !out->ug || !out->lg_mask || !out->ug_mask))
    return fail(SRBD_QP_EINVAL, "CONE needs ng = 24 and D, lg, ug, lg_mask, ug_mask outputs (C optional)");
  srbd_model_params p = *params;
  if (p.qf_scale <= 0.0) p.qf_scale = (double)d.N;
  hipStream_t strm = stream ? reinterpret_cast<hipStream_t>(stream) : h->stream;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(h->device);
  const hipError_t e = srbd::launch_srbd_linearize(p, batch, d.N, constraints, xs, us, *out, strm);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("kernel launch: ") + hipGetErrorString(e));
  return SRBD_QP_OK;
}

void srbd_qp_srbd_default_linesearch(srbd_linesearch_params* p) {
  if (!p) return;
  p->theta_max = 1e-6;
  p->theta_min = 5e-10;
  p->eta = 1e-4;
  p->beta_phi = 1e-6;
  p->beta_theta = 1e-6;
  p->beta_alpha = 0.5;
  p->alpha_min = 1e-4;
}

int srbd_qp_srbd_linesearch_f64(srbd_qp_handle h, int batch, const srbd_model_params* params,
                                const srbd_linesearch_params* ls, double* xs, double* us,
                                const double* dx, const double* du, double* alpha, double* merit,
                                int* converged, void* stream) {
  if (!h || !params || !ls || !xs || !us || !dx || !du || !alpha)
    return fail(SRBD_QP_EINVAL, "NULL argument");
  const srbd_qp_dims& d = h->dims;
  if (d.nx != 12 || d.nu != 12) return fail(SRBD_QP_EDIM, "SRBD line search needs nx = nu = 12");
  if (batch < 0 || batch > h->capacity) return fail(SRBD_QP_ECAPACITY, "batch exceeds capacity");
  if (!(ls->beta_alpha > 0.0 && ls->beta_alpha < 1.0) || !(ls->alpha_min > 0.0))
    return fail(SRBD_QP_EINVAL, "line search needs 0 < beta_alpha < 1 and alpha_min > 0");
  srbd_model_params p = *params;
  if (p.qf_scale <= 0.0) p.qf_scale = (double)d.N;
  hipStream_t strm = stream ? reinterpret_cast<hipStream_t>(stream) : h->stream;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(h->device);
  const hipError_t e = srbd::launch_srbd_linesearch(p, *ls, batch, d.N, xs, us, dx, du, alpha,
                                                    merit, converged, strm);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("kernel launch: ") + hipGetErrorString(e));
  return SRBD_QP_OK;
}

int srbd_qp_srbd_nmpc_f64(srbd_qp_handle h, int batch, const srbd_model_params* params,
                          const srbd_linesearch_params* ls, const srbd_qp_settings* settings,
                          int constraints, int sqp_max_loop, double* xs, double* us,
                          const double* x0, double* alpha, int* sqp_iter, int* converged) {
  if (!h || !params || !ls || !settings || !xs || !us || !x0 || !alpha || !sqp_iter || !converged)
    return fail(SRBD_QP_EINVAL, "NULL argument");
  const srbd_qp_dims& d = h->dims;
  if (d.nx != 12 || d.nu != 12) return fail(SRBD_QP_EDIM, "the SRBD NMPC loop needs nx = nu = 12");
  if (batch < 0 || batch > h->capacity) return fail(SRBD_QP_ECAPACITY, "batch exceeds capacity");
  if (sqp_max_loop < 0) return fail(SRBD_QP_EINVAL, "sqp_max_loop must be non-negative");
  if (constraints < SRBD_QP_SRBD_NONE || constraints > SRBD_QP_SRBD_CONE)
    return fail(SRBD_QP_EINVAL, "unknown constraints mode");
  const bool box = constraints == SRBD_QP_SRBD_BOX_U, cone = constraints == SRBD_QP_SRBD_CONE;
  if ((d.has_box_u != 0) != box || (d.ng > 0) != cone || d.has_box_x || (cone && d.ng != 24))
    return fail(SRBD_QP_EINVAL, "the handle's dims do not match the constraints mode");
  int rc = srbd_qp_check_settings(settings);
  if (rc) return rc;
  if (batch == 0 || sqp_max_loop == 0) return SRBD_QP_OK;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(h->device);
  hipStream_t strm = h->stream;
  // scratch: QP data (linearisation), x0 - x_nmpc(:,0), QP solution, loop state
  const size_t B = (size_t)h->capacity, N = (size_t)d.N;
  struct Buf { size_t off, n; };
  size_t top = 0;
  auto take = [&](size_t n) { Buf b{top, n}; top += (n + 31) / 32 * 32; return b; };
  const Buf bA = take(B * N * 144), bB = take(B * N * 144), bb = take(B * N * 12),
            bQ = take(B * (N + 1) * 144), bS = take(B * N * 144), bR = take(B * N * 144),
            bq = take(B * (N + 1) * 12), br = take(B * N * 12);
  const Buf blbu = take(box ? B * N * 12 : 0), bubu = take(box ? B * N * 12 : 0);
  const Buf bD = take(cone ? B * N * 288 : 0), blg = take(cone ? B * (N + 1) * 24 : 0),
            bug = take(cone ? B * (N + 1) * 24 : 0), blgm = take(cone ? B * (N + 1) * 24 : 0),
            bugm = take(cone ? B * (N + 1) * 24 : 0);
  const Buf bx0 = take(B * 12), bx = take(B * (N + 1) * 12), bu = take(B * N * 12),
            bpi = take(B * (N + 1) * 12);
  const Buf bint = take(B * 4 + 8);  // conv, done, status, iter (ints) + active
  const size_t need = top * sizeof(double);
  hipError_t e = hipSuccess;
  if (need > h->nmpc_bytes) {
    if (h->nmpc) (void)hipFree(h->nmpc);
    h->nmpc = nullptr;
    h->nmpc_bytes = 0;
    e = hipMalloc(&h->nmpc, need);
    if (e == hipSuccess) h->nmpc_bytes = need;
  }
  if (e == hipSuccess && !h->nmpc_active_host)
    e = hipHostMalloc(reinterpret_cast<void**>(&h->nmpc_active_host), sizeof(int));
  if (e != hipSuccess) {
    (void)hipSetDevice(prev);
    return fail(e == hipErrorOutOfMemory ? SRBD_QP_ENOMEM : SRBD_QP_EDEVICE,
                std::string("NMPC scratch allocation failed: ") + hipGetErrorString(e));
  }
  double* base = reinterpret_cast<double*>(h->nmpc);
  auto at = [&](const Buf& b) -> double* { return b.n ? base + b.off : nullptr; };
  srbd_qp_data_f64 qd{};
  qd.A = at(bA); qd.B = at(bB); qd.b = at(bb); qd.Q = at(bQ); qd.S = at(bS); qd.R = at(bR);
  qd.q = at(bq); qd.r = at(br); qd.lbu = at(blbu); qd.ubu = at(bubu);
  qd.D = at(bD); qd.lg = at(blg); qd.ug = at(bug); qd.lg_mask = at(blgm); qd.ug_mask = at(bugm);
  qd.x0 = at(bx0);
  int* ints = reinterpret_cast<int*>(at(bint));
  int *conv = ints, *done = ints + B, *status = ints + 2 * B, *iters = ints + 3 * B,
      *active = ints + 4 * B;
  srbd_qp_solution_f64 sol{};
  sol.x = at(bx); sol.u = at(bu); sol.pi = at(bpi); sol.status = status; sol.iter = iters;
  srbd_model_params p = *params;
  if (p.qf_scale <= 0.0) p.qf_scale = (double)d.N;
  // NMPC_solver.cpp:362-372: prepareQpStructures; solveQpProblems; if (checkConvergence()) break;
  for (int it = 0; it < sqp_max_loop && e == hipSuccess; ++it) {
    e = srbd::launch_srbd_linearize(p, batch, d.N, constraints, xs, us, qd, strm);
    if (e == hipSuccess)
      e = srbd::launch_nmpc_prep(batch, d.N, it, xs, x0, at(bx0), done, sqp_iter, converged, strm);
    if (e != hipSuccess) break;
    (void)hipSetDevice(prev);
    rc = solve_impl<double>(h, batch, settings, &qd, &sol, strm);
    if (rc) return rc;  // the caller's device is current again
    (void)hipSetDevice(h->device);
    e = srbd::launch_srbd_linesearch(p, *ls, batch, d.N, xs, us, at(bx), at(bu), alpha, nullptr,
                                     conv, strm, done);
    if (e == hipSuccess)
      e = srbd::launch_nmpc_after(batch, it, conv, done, sqp_iter, converged, active, strm);
    if (e == hipSuccess)
      e = hipMemcpyAsync(h->nmpc_active_host, active, sizeof(int), hipMemcpyDeviceToHost, strm);
    if (e == hipSuccess) e = hipStreamSynchronize(strm);
    if (e == hipSuccess && *h->nmpc_active_host == 0) break;  // every robot has converged
  }
  if (e == hipSuccess) e = hipStreamSynchronize(strm);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return fail(SRBD_QP_EDEVICE, std::string("NMPC loop: ") + hipGetErrorString(e));
  return SRBD_QP_OK;
}

int srbd_qp_solve_f32(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                      const srbd_qp_data_f32* d, const srbd_qp_solution_f32* s, void* stream) {
  return solve_impl<float>(h, batch, st, d, s, stream);
}
int srbd_qp_solve_host_f32(srbd_qp_handle h, int batch, const srbd_qp_settings* st,
                           const srbd_qp_data_f32* d, const srbd_qp_solution_f32* s) {
  return solve_host_impl<float>(h, batch, st, d, s);
}

}  // extern "C"
