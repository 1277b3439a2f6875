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

namespace {
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

}  // extern "C"
