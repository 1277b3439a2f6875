// C-ABI plumbing: version, thread-local error message, layout conversion.
#include <stdarg.h>

#include "common.h"

namespace eunet {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return EUNET_ERR_HIP;
  }
  return EUNET_OK;
}
}  // namespace eunet

EUNET_DEBUG_UNIT(capi)

namespace eunet {
#ifdef EUNET_DEBUG
int debug_read_conv3x3(unsigned*, unsigned*, bool);
int debug_read_bnpool(unsigned*, unsigned*, bool);
int debug_read_head(unsigned*, unsigned*, bool);
#endif
}  // namespace eunet

namespace {
// a deliberately failing check (eunet_debug_selftest): proves the debug build's reporting path
__global__ void debug_selftest_kernel(int n) { EUNET_DASSERT(threadIdx.x >= (unsigned)n); }

template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* x, int N, int C, int H, int W, T* out, int ct, int co) {
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * C * H * W;
  if (id >= total) return;
  // id enumerates the NHWC destination
  const int c = (int)(id % C);
  const long long p = id / C;  // n*H*W + y*W + x
  const long long hw = (long long)H * W;
  const long long n = p / hw, s = p - n * hw;
  Elem<T>::st(out + p * ct + co + c, x[(n * C + c) * hw + s]);
}
}  // namespace

extern "C" {

const char* eunet_version(void) { return "eunet-mi355x 0.1 (gfx950)"; }

const char* eunet_last_error(void) { return eunet::g_err; }

int eunet_debug_enabled(void) {
#ifdef EUNET_DEBUG
  return 1;
#else
  return 0;
#endif
}

int eunet_debug_status(unsigned* unit_line, unsigned* count, int reset) {
  EUNET_REQUIRE(unit_line && count, "debug_status: null outputs");
  *unit_line = 0;
  *count = 0;
#ifdef EUNET_DEBUG
  if (hipDeviceSynchronize() != hipSuccess) {
    eunet::set_error("debug_status: device synchronisation failed");
    return EUNET_ERR_HIP;
  }
  int (*readers[4])(unsigned*, unsigned*, bool) = {eunet::debug_read_capi, eunet::debug_read_conv3x3,
                                                   eunet::debug_read_bnpool, eunet::debug_read_head};
  for (int u = 0; u < 4; ++u) {
    unsigned line = 0, cnt = 0;
    const int rc = readers[u](&line, &cnt, reset != 0);
    if (rc != EUNET_OK) {
      eunet::set_error("debug_status: reading unit %d failed", u);
      return rc;
    }
    if (cnt && !*unit_line) *unit_line = (unsigned)(u + 1) * 100000u + line;
    *count += cnt;
  }
#endif
  return EUNET_OK;
}

int eunet_debug_selftest(void* stream) {
  debug_selftest_kernel<<<1, 64, 0, (hipStream_t)stream>>>(1);
  EUNET_LAUNCH_CHECK("debug_selftest");
  return EUNET_OK;
}

int eunet_nchw_to_nhwc(const float* x, const eunet_act* out, void* stream) {
  EUNET_REQUIRE(x && out && out->ptr && out->c > 0 && out->coff + out->c <= out->ctot, "nchw_to_nhwc: bad args");
  const long long total = (long long)out->n * out->c * out->h * out->w;
  const unsigned g = (unsigned)((total + 255) / 256);
  if (out->dtype == EUNET_BF16)
    nchw_to_nhwc_kernel<bf16_t><<<g, 256, 0, (hipStream_t)stream>>>(x, out->n, out->c, out->h, out->w,
                                                                     (bf16_t*)out->ptr, out->ctot, out->coff);
  else
    nchw_to_nhwc_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>(x, out->n, out->c, out->h, out->w,
                                                                    (float*)out->ptr, out->ctot, out->coff);
  EUNET_LAUNCH_CHECK("nchw_to_nhwc");
  return EUNET_OK;
}

int eunet_set_update_guard(int device, const double* guard) {
  EUNET_REQUIRE(device >= 0 && device < eunet::GUARD_NDEV, "set_update_guard: device index %d out of range", device);
  eunet::update_guard_slot(device) = guard;
  return EUNET_OK;
}

// Stream-to-stream ordering on the streams' device: `to` waits for the work enqueued on `from` so far.  The
// events have a device-scope release and no timing (torch's Stream.wait_stream records an event with the
// default system-scope release, whose cache writeback / invalidate sits between the producing kernel and
// the recording stream's next kernel).  A ring of events per device; re-recording one whose wait is
// already enqueued is allowed (the wait captured the earlier record).
int eunet_stream_wait(void* from, void* to) {
  constexpr int NDEV = 64, RING = 64;
  static std::mutex mu;
  static hipEvent_t ring[NDEV][RING];
  static unsigned next[NDEV];
  // the device of the streams, not the calling thread's current device (a DataParallel replica or an
  // autograd thread need not have entered it); both streams must be on it
  int dev = 0, dev_to = 0;
  if (hipStreamGetDevice((hipStream_t)from, &dev) != hipSuccess ||
      hipStreamGetDevice((hipStream_t)to, &dev_to) != hipSuccess || dev < 0 || dev >= NDEV) {
    eunet::set_error("stream_wait: cannot query the streams' device (or device index >= %d)", NDEV);
    return EUNET_ERR_HIP;
  }
  EUNET_REQUIRE(dev == dev_to, "stream_wait: streams on devices %d and %d", dev, dev_to);
  std::lock_guard<std::mutex> lock(mu);
  hipEvent_t& e = ring[dev][next[dev]++ % RING];
  if (e == nullptr) {
    int cur = 0;
    const bool sw = hipGetDevice(&cur) == hipSuccess && cur != dev;
    if (sw) (void)hipSetDevice(dev);  // the event belongs to the device current at its creation
    const hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice);
    if (sw) (void)hipSetDevice(cur);
    if (rc != hipSuccess) {
      e = nullptr;
      eunet::set_error("stream_wait: hipEventCreateWithFlags failed");
      return EUNET_ERR_HIP;
    }
  }
  if (hipEventRecord(e, (hipStream_t)from) != hipSuccess || hipStreamWaitEvent((hipStream_t)to, e, 0) != hipSuccess) {
    eunet::set_error("stream_wait: record / wait failed");
    return EUNET_ERR_HIP;
  }
  return EUNET_OK;
}

}  // extern "C"
