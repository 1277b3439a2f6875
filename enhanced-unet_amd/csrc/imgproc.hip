// cv2 image operations of the reference's data path, as HIP kernels.
//
// Reference call sites:
//   dataset.py:58-131   CellDataset._apply_cell_specific_preprocessing (every split, :204):
//                       RGB->LAB, CLAHE(2.5, 8x8) on L, LAB->RGB; Sobel / Laplacian edge features of
//                       the gray image; live-cell brightening; CLAHE(3.0) of the gray image on dead
//                       cells; edge blend; 0.85 / 0.15 mix with the input; GaussianBlur(3x3, 1.0)
//                       unsharp mask (addWeighted 1.3 / -0.3)
//   dataset.py:255-294  augmentations: HSV saturation, CLAHE(U(1.5, 3)), filter2D sharpen, HSV jitter
//   train_eval.py:365-395  Evaluator._prepare_image_tensor: CLAHE(2.0) on L + filter2D sharpen 0.15
//
// cv2 is not importable in this image, so these follow OpenCV's documented algorithms and are
// pinned to the numpy restatement in oracle/imgproc_ref.py, not to cv2 (parity unpinned):
//   RGB2GRAY 8U    Y = (4899 R + 9617 G + 1868 B + 2^13) >> 14
//   RGB<->Lab 8U   cv2's bit-exact fixed-point conversion (color_lab.cpp, OpenCV >= 3.4): sRGB gamma /
//                  cube-root / L->(y, fy) / inverse-gamma tables built once on the host from the same
//                  integer-presented constants (LabTabs), RGB2Lab_b / Lab2RGBinteger integer arithmetic
//   RGB<->HSV 8U   H in [0, 180): cv2's hsv_shift = 12 integer division tables; HSV2RGB in fp32
//   CLAHE          OpenCV CLAHE_Impl: tiles of the image padded to a multiple of the grid by
//                  BORDER_REFLECT_101, clip = max(int(clipLimit * tileArea / 256), 1), excess
//                  redistributed (batch + residual stepping), LUT = round(cdf * 255 / tileArea),
//                  bilinear blend of the four neighbouring tile LUTs (txf = x / tileW - 0.5)
//   filter2D 8U    fp32 sum over the 3x3 taps in row-major order, BORDER_REFLECT_101, round + saturate
//   GaussianBlur   3x3, sigma 1, 8U: separable fixed-point weights (70, 116, 70) / 256
//   Sobel / Laplacian (CV_64F, ksize 3 / 1), BORDER_REFLECT_101
// One thread per pixel except the CLAHE histograms (one block per tile, integer LDS counts) and
// the edge-feature maximum (per-block maxima, reduced in a second pass).
#include <cmath>
#include <cstring>
#include <mutex>

#include "common.h"

// every fp32 / fp64 expression below rounds per operation, as the reference's numpy arrays do
#pragma clang fp contract(off)

namespace {

constexpr int NT = 256;

unsigned grid1(long long n) {
  long long b = (n + NT - 1) / NT;
  return (unsigned)(b > 65535 ? 65535 : (b < 1 ? 1 : b));
}

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * (n - 1) - i;
  return i;
}

__device__ __forceinline__ uint8_t sat_u8(float v) {  // saturate_cast<uchar>(v): round half to even, clamp
  const float r = rintf(v);
  return (uint8_t)(r < 0.f ? 0.f : (r > 255.f ? 255.f : r));
}

__device__ __forceinline__ uint8_t gray_u8(int r, int g, int b) { return (uint8_t)((4899 * r + 9617 * g + 1868 * b + (1 << 13)) >> 14); }

// ---- Lab 8U (cv2 RGB2Lab_b / Lab2RGBinteger; tables: lab_tables_build below) ----
constexpr int LAB_SHIFT = 12, GAMMA_SHIFT = 3, LAB_SHIFT2 = LAB_SHIFT + GAMMA_SHIFT;
constexpr int CBRT_TAB_B = 256 * 3 / 2 * (1 << GAMMA_SHIFT);  // 3072
constexpr int INV_GAMMA_TAB = 1 << 12, LAB_BASE = 1 << 14, MIN_AB = -8145;
struct LabTabs {
  uint16_t gamma[256];            // sRGBGammaTab_b
  uint16_t cbrt[CBRT_TAB_B];      // LabCbrtTab_b
  uint16_t yf[512];               // LabToYF_b: (y, ify) per L
  uint16_t invgamma[INV_GAMMA_TAB];  // sRGBInvGammaTab_b
  int c_fwd[9], c_inv[9];         // RGB2Lab_b / Lab2RGBinteger coefficients, RGB order
};
__device__ LabTabs g_lab;

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }
__device__ __forceinline__ uint8_t clamp_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

__device__ __forceinline__ void rgb2lab(int R8, int G8, int B8, uint8_t& L8, uint8_t& a8, uint8_t& b8) {
  const LabTabs& T = g_lab;
  const int R = T.gamma[R8], G = T.gamma[G8], B = T.gamma[B8];
  const int* C = T.c_fwd;
  const int fX = T.cbrt[descale(R * C[0] + G * C[1] + B * C[2], LAB_SHIFT)];
  const int fY = T.cbrt[descale(R * C[3] + G * C[4] + B * C[5], LAB_SHIFT)];
  const int fZ = T.cbrt[descale(R * C[6] + G * C[7] + B * C[8], LAB_SHIFT)];
  constexpr int Lscale = (116 * 255 + 50) / 100, Lshift = -((16 * 255 * (1 << LAB_SHIFT2) + 50) / 100);
  L8 = clamp_u8(descale(Lscale * fY + Lshift, LAB_SHIFT2));
  a8 = clamp_u8(descale(500 * (fX - fY) + 128 * (1 << LAB_SHIFT2), LAB_SHIFT2));
  b8 = clamp_u8(descale(200 * (fY - fZ) + 128 * (1 << LAB_SHIFT2), LAB_SHIFT2));
}

// abToXZ_b[v - minABvalue], evaluated instead of tabulated (integer only)
__device__ __forceinline__ int ab_to_xz(int v) {
  return v <= 3390 ? v * 108 / 841 - LAB_BASE * 16 / 116 * 108 / 841 : v * v / LAB_BASE * v / LAB_BASE;
}

__device__ __forceinline__ void lab2rgb(int L8, int a8, int b8, uint8_t& R, uint8_t& G, uint8_t& B) {
  const LabTabs& T = g_lab;
  const int y = T.yf[2 * L8], ify = T.yf[2 * L8 + 1];
  const int adiv = ((5 * a8 * 53687 + (1 << 7)) >> 13) - 128 * LAB_BASE / 500;
  const int bdiv = ((b8 * 41943 + (1 << 4)) >> 9) - 128 * LAB_BASE / 200 + 1;
  const int x = ab_to_xz(ify + adiv), z = ab_to_xz(ify - bdiv);
  const int* C = T.c_inv;
  constexpr int SH = LAB_SHIFT + (14 - 12);  // lab_shift + (base_shift - inv_gamma_shift)
  int o[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int v = descale(C[3 * r] * x + C[3 * r + 1] * y + C[3 * r + 2] * z, SH);
    o[r] = T.invgamma[v < 0 ? 0 : (v > INV_GAMMA_TAB - 1 ? INV_GAMMA_TAB - 1 : v)];
  }
  R = (uint8_t)o[0];
  G = (uint8_t)o[1];
  B = (uint8_t)o[2];
}

// ---- HSV (8U: H in [0, 180)) ----
__device__ __forceinline__ void rgb2hsv(int r, int g, int b, int& h, int& s, int& v) {
  constexpr int SH = 12;
  int vmin = min(r, min(g, b));
  v = max(r, max(g, b));
  const int diff = v - vmin;
  const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
  // sdiv_table[i] = round((255 << 12) / i), hdiv_table[i] = round((180 << 12) / (6 i))
  const int sdiv = v == 0 ? 0 : (int)rint((double)(255 << SH) / v);
  const int hdiv = diff == 0 ? 0 : (int)rint((double)(180 << SH) / (6.0 * diff));
  s = (diff * sdiv + (1 << (SH - 1))) >> SH;
  int hh = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
  hh = (hh * hdiv + (1 << (SH - 1))) >> SH;
  h = hh + (hh < 0 ? 180 : 0);
}

__device__ __forceinline__ void hsv2rgb(int h8, int s8, int v8, uint8_t& R, uint8_t& G, uint8_t& B) {
  float h = h8 * (6.f / 180.f), s = s8 * (1.f / 255.f), v = v8 * (1.f / 255.f);
  float r, g, b;
  if (s == 0.f) {
    r = g = b = v;
  } else {
    if (h < 0.f) h += 6.f;
    if (h >= 6.f) h -= 6.f;
    const int sector = (int)floorf(h);
    h -= (float)sector;
    const float t0 = v, t1 = v * (1.f - s), t2 = v * (1.f - s * h), t3 = v * (1.f - s * (1.f - h));
    switch (sector) {
      case 0: r = t0; g = t3; b = t1; break;
      case 1: r = t2; g = t0; b = t1; break;
      case 2: r = t1; g = t0; b = t3; break;
      case 3: r = t1; g = t2; b = t0; break;
      case 4: r = t3; g = t1; b = t0; break;
      default: r = t0; g = t1; b = t2; break;
    }
  }
  R = sat_u8(r * 255.f);
  G = sat_u8(g * 255.f);
  B = sat_u8(b * 255.f);
}

// ---- kernels ----
__global__ __launch_bounds__(NT) void rgb2lab_kernel(const uint8_t* rgb, uint8_t* lab, long long n) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    uint8_t L, a, b;
    rgb2lab(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], L, a, b);
    lab[3 * i] = L;
    lab[3 * i + 1] = a;
    lab[3 * i + 2] = b;
  }
}

__global__ __launch_bounds__(NT) void lab2rgb_kernel(const uint8_t* lab, uint8_t* rgb, long long n) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    uint8_t R, G, B;
    lab2rgb(lab[3 * i], lab[3 * i + 1], lab[3 * i + 2], R, G, B);
    rgb[3 * i] = R;
    rgb[3 * i + 1] = G;
    rgb[3 * i + 2] = B;
  }
}

__global__ __launch_bounds__(NT) void rgb2gray_kernel(const uint8_t* rgb, uint8_t* gray, long long n) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT)
    gray[i] = gray_u8(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]);
}

// mode bit 0: S = trunc(clip(S * sat_mul, 0, 255))      (dataset.py:257-261)
// mode bit 1: H = trunc((H + hue_add) mod 180), V = trunc(clip(V * val_mul, 0, 255))  (:288-292)
// all in fp32 as the reference's float32 HSV arrays
__global__ __launch_bounds__(NT) void hsv_adjust_kernel(uint8_t* rgb, long long n, float sat_mul, float hue_add,
                                                        float val_mul, int mode) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    int h, s, v;
    rgb2hsv(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2], h, s, v);
    if (mode & 1) s = (int)fminf(fmaxf((float)s * sat_mul, 0.f), 255.f);
    if (mode & 2) {
      float hf = fmodf((float)h + hue_add, 180.f);  // numpy %: result takes the divisor's sign
      if (hf < 0.f) hf += 180.f;
      h = (int)hf;
      v = (int)fminf(fmaxf((float)v * val_mul, 0.f), 255.f);
    }
    uint8_t R, G, B;
    hsv2rgb(h, s, v, R, G, B);
    rgb[3 * i] = R;
    rgb[3 * i + 1] = G;
    rgb[3 * i + 2] = B;
  }
}

// CLAHE tile LUTs: one block per tile of the REFLECT_101-padded image; src channel ch of a
// pixel-stride-ps image
__global__ __launch_bounds__(NT) void clahe_lut_kernel(const uint8_t* src, int ps, int h, int w, int tw, int th,
                                                       int tiles_x, int clip, float lut_scale, uint8_t* luts) {
  __shared__ unsigned hist[256];
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
  for (int i = threadIdx.x; i < 256; i += NT) hist[i] = 0u;
  __syncthreads();
  for (int p = threadIdx.x; p < tw * th; p += NT) {
    const int y = reflect101(ty * th + p / tw, h), x = reflect101(tx * tw + p % tw, w);
    atomicAdd(&hist[src[((long long)y * w + x) * ps]], 1u);  // LDS integer counts: order-free
  }
  __syncthreads();
  // clip + redistribute + cumulate as OpenCV's serial loops do, one bin per thread (the serial form
  // in one thread was 3 x 256 dependent steps with byte stores, most of the kernel's 44 us):
  // excess = block sum, the residual's +1 lands on bins 0, step, 2 step, ... (residual of them),
  // the LUT is the inclusive prefix sum (wave scans + the waves' totals through LDS), integer-exact
  static_assert(NT == 256, "one histogram bin per thread");
  __shared__ int wsum[NT / 64];
  const int i = threadIdx.x, lane = i & 63, wv = i >> 6;
  int c = (int)hist[i];
  int ex = c > clip ? c - clip : 0;
  c = min(c, clip);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ex += __shfl_xor(ex, o, 64);
  if (lane == 0) wsum[wv] = ex;
  __syncthreads();
  const int excess = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  const int batch = excess / 256, residual = excess - batch * 256;
  c += batch;
  if (residual != 0) {
    const int step = max(256 / residual, 1);
    if (i % step == 0 && i / step < residual) c += 1;
  }
  unsigned sum = (unsigned)c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned v = __shfl_up(sum, o, 64);
    if (lane >= o) sum += v;
  }
  __syncthreads();  // every thread has read wsum (excess)
  if (lane == 63) wsum[wv] = (int)sum;
  __syncthreads();
  for (int w = 0; w < wv; ++w) sum += (unsigned)wsum[w];
  luts[(long long)blockIdx.x * 256 + i] = sat_u8((float)sum * lut_scale);
}

// bilinear blend of the four neighbouring tile LUTs (OpenCV CLAHE_Interpolation_Body)
__device__ __forceinline__ uint8_t clahe_px(const uint8_t* luts, int tiles_x, int tiles_y, float inv_tw, float inv_th,
                                            int x, int y, int v) {
  const float txf = x * inv_tw - 0.5f, tyf = y * inv_th - 0.5f;
  int tx1 = (int)floorf(txf), ty1 = (int)floorf(tyf);
  const float xa = txf - tx1, ya = tyf - ty1;
  int tx2 = tx1 + 1, ty2 = ty1 + 1;
  tx1 = max(tx1, 0);
  ty1 = max(ty1, 0);
  tx2 = min(tx2, tiles_x - 1);
  ty2 = min(ty2, tiles_y - 1);
  const uint8_t* l11 = luts + ((long long)ty1 * tiles_x + tx1) * 256;
  const uint8_t* l12 = luts + ((long long)ty1 * tiles_x + tx2) * 256;
  const uint8_t* l21 = luts + ((long long)ty2 * tiles_x + tx1) * 256;
  const uint8_t* l22 = luts + ((long long)ty2 * tiles_x + tx2) * 256;
  const float res = (l11[v] * (1.f - xa) + l12[v] * xa) * (1.f - ya) + (l21[v] * (1.f - xa) + l22[v] * xa) * ya;
  return sat_u8(res);
}

// mode 0: gray -> gray; mode 1: Lab image, L replaced, converted back to RGB (dst 3 channels)
__global__ __launch_bounds__(NT) void clahe_apply_kernel(const uint8_t* src, int ps, int h, int w, const uint8_t* luts,
                                                         int tiles_x, int tiles_y, float inv_tw, float inv_th,
                                                         uint8_t* dst, int mode) {
  const long long n = (long long)h * w;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int y = (int)(i / w), x = (int)(i - (long long)y * w);
    const uint8_t L = clahe_px(luts, tiles_x, tiles_y, inv_tw, inv_th, x, y, src[i * ps]);
    if (mode == 0) {
      dst[i] = L;
    } else {
      uint8_t R, G, B;
      lab2rgb(L, src[i * ps + 1], src[i * ps + 2], R, G, B);
      dst[3 * i] = R;
      dst[3 * i + 1] = G;
      dst[3 * i + 2] = B;
    }
  }
}

// cv2.filter2D(src, -1, k) 8U, 3x3, anchor centre, BORDER_REFLECT_101: fp32 taps in row-major order
struct K9 { float k[9]; };
__global__ __launch_bounds__(NT) void filter3x3_kernel(const uint8_t* src, uint8_t* dst, int h, int w, int c, K9 k) {
  const long long n = (long long)h * w * c;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const long long p = i / c;
    const int ch = (int)(i - p * c), y = (int)(p / w), x = (int)(p - (long long)y * w);
    float s = 0.f;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int yy = reflect101(y + dy, h), xx = reflect101(x + dx, w);
        s += k.k[(dy + 1) * 3 + dx + 1] * (float)src[((long long)yy * w + xx) * c + ch];
      }
    dst[i] = sat_u8(s);
  }
}

// GaussianBlur(3x3, sigma 1) 8U fixed point (70, 116, 70) / 256 rows then columns, then
// addWeighted(src, 1.3, blur, -0.3, 0) (dataset.py:126-128)
__global__ __launch_bounds__(NT) void unsharp_kernel(const uint8_t* src, uint8_t* dst, int h, int w, int c) {
  const long long n = (long long)h * w * c;
  const int wk[3] = {70, 116, 70};
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const long long p = i / c;
    const int ch = (int)(i - p * c), y = (int)(p / w), x = (int)(p - (long long)y * w);
    unsigned col = 0;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int yy = reflect101(y + dy, h);
      unsigned row = 0;
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) row += wk[dx + 1] * src[((long long)yy * w + reflect101(x + dx, w)) * c + ch];
      col += wk[dy + 1] * row;
    }
    const int g = (int)((col + (1u << 15)) >> 16);
    dst[i] = sat_u8((float)src[i] * 1.3f + (float)g * -0.3f);
  }
}

// Sobel magnitude and |Laplacian| of a gray image in fp64 (CV_64F), per-block maxima
__global__ __launch_bounds__(NT) void edge_raw_kernel(const uint8_t* gray, int h, int w, double* mag, double* lap,
                                                      double* bmax) {
  __shared__ double sm[2][NT];
  const long long n = (long long)h * w;
  double m1 = 0.0, m2 = 0.0;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int y = (int)(i / w), x = (int)(i - (long long)y * w);
    int v[3][3];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) v[dy][dx] = gray[(long long)reflect101(y + dy - 1, h) * w + reflect101(x + dx - 1, w)];
    const double sx = (double)((v[0][2] - v[0][0]) + 2 * (v[1][2] - v[1][0]) + (v[2][2] - v[2][0]));
    const double sy = (double)((v[2][0] - v[0][0]) + 2 * (v[2][1] - v[0][1]) + (v[2][2] - v[0][2]));
    const double mg = sqrt(sx * sx + sy * sy);
    const double lp = fabs((double)(v[0][1] + v[1][0] - 4 * v[1][1] + v[1][2] + v[2][1]));
    mag[i] = mg;
    lap[i] = lp;
    m1 = fmax(m1, mg);
    m2 = fmax(m2, lp);
  }
  sm[0][threadIdx.x] = m1;
  sm[1][threadIdx.x] = m2;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sm[0][threadIdx.x] = fmax(sm[0][threadIdx.x], sm[0][threadIdx.x + s]);
      sm[1][threadIdx.x] = fmax(sm[1][threadIdx.x], sm[1][threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    bmax[2 * blockIdx.x] = sm[0][0];
    bmax[2 * blockIdx.x + 1] = sm[1][0];
  }
}

// edges = trunc(trunc(clip(mag / (max + 1e-6) * 255)) * 0.7 + trunc(clip(|lap| / (max + 1e-6) * 255)) * 0.3)
// (dataset.py:81-91: fp64 normalisation, fp32 blend, astype(uint8) truncations)
__global__ __launch_bounds__(NT) void edge_combine_kernel(const double* mag, const double* lap, const double* bmax,
                                                          int nb, long long n, uint8_t* edges) {
  // the maxima over edge_raw's per-block rows: every block reduces them with all its threads (a
  // serial loop over ~1200 rows in two threads was a 1200-deep chain of dependent loads, 120 us)
  __shared__ double sm[2][NT];
  __shared__ double mx[2];
  double m1 = 0.0, m2 = 0.0;
  for (int b = threadIdx.x; b < nb; b += NT) {
    m1 = fmax(m1, bmax[2 * b]);
    m2 = fmax(m2, bmax[2 * b + 1]);
  }
  sm[0][threadIdx.x] = m1;
  sm[1][threadIdx.x] = m2;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sm[0][threadIdx.x] = fmax(sm[0][threadIdx.x], sm[0][threadIdx.x + s]);
      sm[1][threadIdx.x] = fmax(sm[1][threadIdx.x], sm[1][threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 2) mx[threadIdx.x] = sm[threadIdx.x][0];
  __syncthreads();
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const double e = fmin(fmax(mag[i] / (mx[0] + 1e-6) * 255.0, 0.0), 255.0);
    const double l = fmin(fmax(lap[i] / (mx[1] + 1e-6) * 255.0, 0.0), 255.0);
    const float c = (float)(uint8_t)e * 0.7f + (float)(uint8_t)l * 0.3f;
    edges[i] = (uint8_t)c;
  }
}

// live-cell brightening (dataset.py:103-107): img = trunc(clip(img * 1.1)) where live
__global__ __launch_bounds__(NT) void live_boost_kernel(uint8_t* img, const int64_t* live, long long n) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT)
    if (live[i] > 0)
#pragma unroll
      for (int c = 0; c < 3; ++c) img[3 * i + c] = (uint8_t)fminf((float)img[3 * i + c] * 1.1f, 255.f);
}

// dataset.py:109-124: dead-cell CLAHE gray where dead (dead_gray may be null: no dead pixels), edge
// blend trunc(clip(img * 0.9 + edges * 0.1)), then trunc(that * 0.85 + original * 0.15)
__global__ __launch_bounds__(NT) void cell_mix_kernel(const uint8_t* orig, const uint8_t* clahe_img,
                                                      const uint8_t* edges, const int64_t* dead,
                                                      const uint8_t* dead_gray, long long n, uint8_t* out) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const bool dd = dead_gray != nullptr && dead[i] > 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = dd ? (float)dead_gray[i] : (float)clahe_img[3 * i + c];
      const float we = fminf(fmaxf(v * 0.9f + (float)edges[i] * 0.1f, 0.f), 255.f);
      const float fin = (float)(uint8_t)we * 0.85f + (float)orig[3 * i + c] * 0.15f;
      out[3 * i + c] = (uint8_t)fin;
    }
  }
}

// Evaluator input (train_eval.py:367-377): per-block maxima of the CHW float image ...
__global__ __launch_bounds__(NT) void max_partial_kernel(const float* x, long long n, float* bmax) {
  __shared__ float sm[NT];
  float m = -INFINITY;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) m = fmaxf(m, x[i]);
  sm[threadIdx.x] = m;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sm[threadIdx.x] = fmaxf(sm[threadIdx.x], sm[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) bmax[blockIdx.x] = sm[0];
}

// ... then HWC uint8 = astype(uint8) of (max <= 1 ? x * 255 : x): fp32, truncation (C cast through int)
__global__ __launch_bounds__(NT) void chw_to_u8_kernel(const float* x, int c, int h, int w, const float* bmax, int nb,
                                                       uint8_t* out) {
  __shared__ float mx;
  if (threadIdx.x == 0) {
    float m = -INFINITY;
    for (int b = 0; b < nb; ++b) m = fmaxf(m, bmax[b]);
    mx = m;
  }
  __syncthreads();
  const bool unit = mx <= 1.f;
  const long long hw = (long long)h * w, n = hw * c;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const long long p = i / c;
    const int ch = (int)(i - p * c);
    const float v = x[(long long)ch * hw + p];
    out[i] = (uint8_t)(int)(unit ? v * 255.f : v);
  }
}

// ---- host: initLabTabs (color_lab.cpp) from the same integer-presented constants.  softfloat
// operations are IEEE float32 operations (this file has FP contraction off), softdouble ones float64;
// mulAdd is a fused multiply-add; cvRound rounds half to even (nearbyint).  oracle/imgproc_ref.py
// lab_tables is the same construction in numpy. ----
double apply_gamma(float x) {
  const double xd = x;
  return xd <= 809.0 / 20000.0 ? xd / (323.0 / 25.0) : std::pow((xd + 11.0 / 200.0) / (1.0 + 11.0 / 200.0), 12.0 / 5.0);
}
double apply_inv_gamma(float x) {
  const double xd = x;
  return xd <= 7827.0 / 2500000.0 ? xd * (323.0 / 25.0)
                                  : std::pow(xd, 1.0 / (12.0 / 5.0)) * (1.0 + 11.0 / 200.0) - 11.0 / 200.0;
}
int rne(double v) { return (int)std::nearbyint(v); }

LabTabs build_lab_tabs() {
  LabTabs t{};
  for (int i = 0; i < 256; ++i) {
    const float g = (float)apply_gamma((float)i / 255.f);
    t.gamma[i] = (uint16_t)rne((float)(255 * (1 << GAMMA_SHIFT)) * g);
  }
  const float lthresh = 216.f / 24389.f, lscale = 841.f / 108.f, lbias = 16.f / 116.f;
  const float cbs = 1.f / (255.f * (float)(1 << GAMMA_SHIFT));
  for (int i = 0; i < CBRT_TAB_B; ++i) {
    const float x = cbs * (float)i;
    const float f = x < lthresh ? (float)std::fma((double)x, (double)lscale, (double)lbias) : (float)std::cbrt((double)x);
    t.cbrt[i] = (uint16_t)rne((float)(1 << LAB_SHIFT2) * f);
  }
  for (int L = 0; L < 256; ++L) {
    int y, ify;
    if (L <= 20) {
      y = rne((float)(L * LAB_BASE * 20 * 9) / (float)(17 * 29 * 29 * 29));
      ify = rne((float)LAB_BASE * (16.f / 116.f + (float)(L * 5) / (float)(3 * 17 * 29)));
    } else {
      const float fy = (float)(L * 100 * LAB_BASE) / (float)(255 * 116) + (float)(16 * LAB_BASE) / 116.f;
      ify = rne(fy);
      y = rne(fy * fy * fy / (float)(LAB_BASE * LAB_BASE));
    }
    t.yf[2 * L] = (uint16_t)y;
    t.yf[2 * L + 1] = (uint16_t)ify;
  }
  for (int i = 0; i < INV_GAMMA_TAB; ++i) {
    const float x = 1.f / (float)INV_GAMMA_TAB * (float)i;
    t.invgamma[i] = (uint16_t)rne(255.f * (float)apply_inv_gamma(x));
  }
  const double d65[3] = {0.950456, 1.0, 1.088754};
  const double m_fwd[9] = {0.412453, 0.357580, 0.180423, 0.212671, 0.715160, 0.072169, 0.019334, 0.119193, 0.950227};
  const double m_inv[9] = {3.240479, -1.53715, -0.498535, -0.969256, 1.875991, 0.041556, 0.055648, -0.204043, 1.057311};
  const double lshift = (double)(1 << LAB_SHIFT);
  for (int r = 0; r < 3; ++r)
    for (int j = 0; j < 3; ++j) {
      t.c_fwd[3 * r + j] = rne(lshift * m_fwd[3 * r + j] / d65[r]);
      t.c_inv[3 * r + j] = rne(lshift * m_inv[3 * r + j] * d65[j]);
    }
  return t;
}

// the tables reach each device once (a synchronous copy into the g_lab symbol, ordered before every
// later launch from this host thread); the C-ABI still allocates nothing
std::mutex g_lab_mu;
bool g_lab_ready[64];
int lab_tables_ready() {
  int dev = 0;
  EUNET_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64, "Lab tables: no current device");
  std::lock_guard<std::mutex> lk(g_lab_mu);
  if (!g_lab_ready[dev]) {
    static const LabTabs host = build_lab_tabs();
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lab), &host, sizeof(LabTabs)) != hipSuccess) {
      eunet::set_error("Lab tables: copy to the device failed");
      return EUNET_ERR_HIP;
    }
    g_lab_ready[dev] = true;
  }
  return EUNET_OK;
}

}  // namespace

extern "C" {

int eunet_chw_to_u8_workspace_bytes(int c, int h, int w, size_t* bytes) {
  EUNET_REQUIRE(c > 0 && h > 0 && w > 0 && bytes, "chw_to_u8_workspace_bytes: bad args");
  *bytes = (size_t)grid1((long long)c * h * w) * sizeof(float);
  return EUNET_OK;
}

int eunet_chw_to_u8(const float* x, int c, int h, int w, void* ws, uint8_t* out, void* stream) {
  EUNET_REQUIRE(x && ws && out && c > 0 && h > 0 && w > 0, "chw_to_u8: bad args");
  const long long n = (long long)c * h * w;
  const unsigned nb = grid1(n);
  max_partial_kernel<<<nb, NT, 0, (hipStream_t)stream>>>(x, n, (float*)ws);
  EUNET_LAUNCH_CHECK("max_partial");
  chw_to_u8_kernel<<<nb, NT, 0, (hipStream_t)stream>>>(x, c, h, w, (const float*)ws, (int)nb, out);
  EUNET_LAUNCH_CHECK("chw_to_u8");
  return EUNET_OK;
}

int eunet_lab_tables(void* out, size_t bytes) {
  static_assert(sizeof(LabTabs) == 2 * (256 + CBRT_TAB_B + 512 + INV_GAMMA_TAB) + 4 * 18, "LabTabs layout");
  EUNET_REQUIRE(out && bytes >= sizeof(LabTabs), "lab_tables: need %zu bytes", sizeof(LabTabs));
  static const LabTabs t = build_lab_tabs();
  std::memcpy(out, &t, sizeof(LabTabs));
  return EUNET_OK;
}

int eunet_rgb2lab_u8(const uint8_t* rgb, uint8_t* lab, long long npix, void* stream) {
  EUNET_REQUIRE(rgb && lab && npix > 0, "rgb2lab_u8: bad args");
  if (int rc = lab_tables_ready()) return rc;
  rgb2lab_kernel<<<grid1(npix), NT, 0, (hipStream_t)stream>>>(rgb, lab, npix);
  EUNET_LAUNCH_CHECK("rgb2lab_u8");
  return EUNET_OK;
}

int eunet_lab2rgb_u8(const uint8_t* lab, uint8_t* rgb, long long npix, void* stream) {
  EUNET_REQUIRE(rgb && lab && npix > 0, "lab2rgb_u8: bad args");
  if (int rc = lab_tables_ready()) return rc;
  lab2rgb_kernel<<<grid1(npix), NT, 0, (hipStream_t)stream>>>(lab, rgb, npix);
  EUNET_LAUNCH_CHECK("lab2rgb_u8");
  return EUNET_OK;
}

int eunet_rgb2gray_u8(const uint8_t* rgb, uint8_t* gray, long long npix, void* stream) {
  EUNET_REQUIRE(rgb && gray && npix > 0, "rgb2gray_u8: bad args");
  rgb2gray_kernel<<<grid1(npix), NT, 0, (hipStream_t)stream>>>(rgb, gray, npix);
  EUNET_LAUNCH_CHECK("rgb2gray_u8");
  return EUNET_OK;
}

int eunet_hsv_adjust_u8(uint8_t* rgb, long long npix, float sat_mul, float hue_add, float val_mul, int mode,
                        void* stream) {
  EUNET_REQUIRE(rgb && npix > 0 && (mode & ~3) == 0, "hsv_adjust_u8: bad args");
  hsv_adjust_kernel<<<grid1(npix), NT, 0, (hipStream_t)stream>>>(rgb, npix, sat_mul, hue_add, val_mul, mode);
  EUNET_LAUNCH_CHECK("hsv_adjust_u8");
  return EUNET_OK;
}

int eunet_clahe_u8(const uint8_t* src, int mode, int h, int w, double clip_limit, int tiles_x, int tiles_y,
                   uint8_t* luts, uint8_t* dst, void* stream) {
  EUNET_REQUIRE(src && dst && luts && h > 0 && w > 0 && tiles_x > 0 && tiles_y > 0 && (mode == 0 || mode == 1),
                "clahe_u8: bad args");
  const int ps = mode == 0 ? 1 : 3;
  // OpenCV CLAHE_Impl::apply: when the image is a multiple of the grid on both axes the tile is
  // size / grid; otherwise BOTH axes are padded (BORDER_REFLECT_101, bottom / right) by
  // tiles - size % tiles, so the tile is size / tiles + 1 on each axis -- also on an axis that
  // divides evenly
  const bool even = w % tiles_x == 0 && h % tiles_y == 0;
  const int tw = w / tiles_x + (even ? 0 : 1), th = h / tiles_y + (even ? 0 : 1);
  const int area = tw * th;
  const int clip = clip_limit > 0.0 ? std::max((int)(clip_limit * area / 256), 1) : (1 << 30);
  clahe_lut_kernel<<<tiles_x * tiles_y, NT, 0, (hipStream_t)stream>>>(src, ps, h, w, tw, th, tiles_x, clip,
                                                                     255.f / (float)area, luts);
  EUNET_LAUNCH_CHECK("clahe_lut");
  if (mode == 1)
    if (int rc = lab_tables_ready()) return rc;
  clahe_apply_kernel<<<grid1((long long)h * w), NT, 0, (hipStream_t)stream>>>(src, ps, h, w, luts, tiles_x, tiles_y,
                                                                              1.f / tw, 1.f / th, dst, mode);
  EUNET_LAUNCH_CHECK("clahe_apply");
  return EUNET_OK;
}

int eunet_filter3x3_u8(const uint8_t* src, uint8_t* dst, int h, int w, int c, const float* k9, void* stream) {
  EUNET_REQUIRE(src && dst && k9 && h > 0 && w > 0 && c > 0 && src != dst, "filter3x3_u8: bad args");
  K9 k;
  for (int i = 0; i < 9; ++i) k.k[i] = k9[i];
  filter3x3_kernel<<<grid1((long long)h * w * c), NT, 0, (hipStream_t)stream>>>(src, dst, h, w, c, k);
  EUNET_LAUNCH_CHECK("filter3x3_u8");
  return EUNET_OK;
}

int eunet_unsharp_u8(const uint8_t* src, uint8_t* dst, int h, int w, int c, void* stream) {
  EUNET_REQUIRE(src && dst && h > 0 && w > 0 && c > 0 && src != dst, "unsharp_u8: bad args");
  unsharp_kernel<<<grid1((long long)h * w * c), NT, 0, (hipStream_t)stream>>>(src, dst, h, w, c);
  EUNET_LAUNCH_CHECK("unsharp_u8");
  return EUNET_OK;
}

int eunet_edge_features_workspace_bytes(int h, int w, size_t* bytes) {
  EUNET_REQUIRE(h > 0 && w > 0 && bytes, "edge_features_workspace_bytes: bad args");
  *bytes = (size_t)h * w * 2 * sizeof(double) + (size_t)grid1((long long)h * w) * 2 * sizeof(double);
  return EUNET_OK;
}

int eunet_edge_features_u8(const uint8_t* gray, int h, int w, void* ws, uint8_t* edges, void* stream) {
  EUNET_REQUIRE(gray && ws && edges && h > 0 && w > 0, "edge_features_u8: bad args");
  const long long n = (long long)h * w;
  double* mag = (double*)ws;
  double* lap = mag + n;
  double* bmax = lap + n;
  const unsigned nb = grid1(n);
  edge_raw_kernel<<<nb, NT, 0, (hipStream_t)stream>>>(gray, h, w, mag, lap, bmax);
  EUNET_LAUNCH_CHECK("edge_raw");
  edge_combine_kernel<<<nb, NT, 0, (hipStream_t)stream>>>(mag, lap, bmax, (int)nb, n, edges);
  EUNET_LAUNCH_CHECK("edge_combine");
  return EUNET_OK;
}

int eunet_live_boost_u8(uint8_t* img, const int64_t* live_mask, long long npix, void* stream) {
  EUNET_REQUIRE(img && live_mask && npix > 0, "live_boost_u8: bad args");
  live_boost_kernel<<<grid1(npix), NT, 0, (hipStream_t)stream>>>(img, live_mask, npix);
  EUNET_LAUNCH_CHECK("live_boost_u8");
  return EUNET_OK;
}

int eunet_cell_mix_u8(const uint8_t* orig, const uint8_t* clahe_img, const uint8_t* edges, const int64_t* dead_mask,
                      const uint8_t* dead_gray, long long npix, uint8_t* out, void* stream) {
  EUNET_REQUIRE(orig && clahe_img && edges && out && npix > 0 && (dead_gray == nullptr || dead_mask != nullptr),
                "cell_mix_u8: bad args");
  cell_mix_kernel<<<grid1(npix), NT, 0, (hipStream_t)stream>>>(orig, clahe_img, edges, dead_mask, dead_gray, npix,
                                                               out);
  EUNET_LAUNCH_CHECK("cell_mix_u8");
  return EUNET_OK;
}

}  // extern "C"
