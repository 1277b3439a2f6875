// Device-side data path of the training loader.
//
// Reference: dataset.py:133-321 (CellDataset.__getitem__), 355-361 (collate_fn).
// The reference runs all of it per sample on the host with cv2 / numpy /
// PIL (num_workers=0); at the GPU's img/s that loader is the bottleneck.  Here
// the decoded uint8 image and the LabelMe polygons go to the device once and
// everything per-pixel runs in HIP:
//   rasterize   LabelMe polygons -> semantic mask (instance order, last wins:
//               dataset.py:197-201) with cv2.fillPoly's rule (documented at the kernel)
//   flip        cv2.flip of image / mask (dataset.py:208-222)
//   augment_u8  the reference's numpy pixel ops in its order -- brightness
//               np.clip(img*alpha,0,255).astype(uint8) (:243), contrast
//               np.clip(img+beta,...) (:251), additive noise (:268), gamma LUT
//               (:273-276) -- each rounding to uint8 as numpy does (fp64 math)
//   to_tensor   transforms.ToTensor: HWC uint8 -> CHW float / 255 (:302-305)
//   resize_u8   cv2.resize INTER_LINEAR for 8U (dataset.py:151, 158): OpenCV's fixed-point
//               algorithm -- 11-bit coefficients, int row sums, the SIMD vertical rounding (and
//               the 2x-downscale INTER_AREA switch); oracle/data_ref.py resize_linear_u8.
// All are HBM-bound byte kernels: one thread per pixel, no reductions.
#include <climits>
#include <cmath>

#include "common.h"

namespace {

constexpr int NT = 256;

unsigned grid1(long long n) {
  long long b = (n + NT - 1) / NT;
  return (unsigned)(b > 65535 ? 65535 : (b < 1 ? 1 : b));
}

// Fill rule: cv2.fillPoly(mask, [points], 1) (dataset.py:184-186; LINE_8, shift 0) as OpenCV 4.x
// computes it (imgproc/src/drawing.cpp, 4.5.2 and later; oracle/data_ref.py fill_poly_u8 restates it):
//  * every edge (v[k-1], v[k]) is drawn with the 8-connected Line: LineIterator clips the endpoints
//    (clipLine), starts at the left one and runs Bresenham with err = dx - 2dy over dx + 1 pixels --
//    in closed form the pixel at major offset i has minor offset ceil((2 dmin i - dmaj) / (2 dmaj));
//  * the non-horizontal edges are collected in XY_SHIFT = 16 fixed point: x + 1/2 for an edge whose
//    endpoints are in the image, else the clipped endpoints (exact integers) re-projected to the
//    unclipped y0, dx = C-truncated (x1 - x0) / (y1 - y0); FillEdgeCollection then fills row y between
//    consecutive edges of the x-sorted active list (y0 <= y < y1), from x_a >> 16 to x_b >> 16.
// Per pixel that fill is a count: with a_e = x_e(y) >> 16 of the active edges, pixel x lies in a span
// iff #{a_e < x} is odd or some a_e == x follows an even count (#{a_e <= x} > #{a_e < x}).  Both
// rules are exact integer / fixed-point arithmetic; clipLine's double crossings match the CPU's IEEE
// ops (no contraction across the division).  pts: int32 (x, y) pairs; poly_off[i]..poly_off[i+1] the
// vertices of polygon i; labels[i] in {1 live, 2 dead}.
__device__ bool cv_clip_line(int w, int h, long long& x1, long long& y1, long long& x2, long long& y2) {
  const long long right = w - 1, bottom = h - 1;
  int c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
  int c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
  if ((c1 & c2) == 0 && (c1 | c2) != 0) {
    long long a;
    if (c1 & 12) {
      a = c1 < 8 ? 0 : bottom;
      x1 += (long long)((double)(a - y1) * (double)(x2 - x1) / (double)(y2 - y1));
      y1 = a;
      c1 = (x1 < 0) + (x1 > right) * 2;
    }
    if (c2 & 12) {
      a = c2 < 8 ? 0 : bottom;
      x2 += (long long)((double)(a - y2) * (double)(x2 - x1) / (double)(y2 - y1));
      y2 = a;
      c2 = (x2 < 0) + (x2 > right) * 2;
    }
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
      if (c1) {
        a = c1 == 1 ? 0 : right;
        y1 += (long long)((double)(a - x1) * (double)(y2 - y1) / (double)(x2 - x1));
        x1 = a;
        c1 = 0;
      }
      if (c2) {
        a = c2 == 1 ? 0 : right;
        y2 += (long long)((double)(a - x2) * (double)(y2 - y1) / (double)(x2 - x1));
        x2 = a;
        c2 = 0;
      }
    }
  }
  return (c1 | c2) == 0;
}

__device__ bool cv_fillpoly_covers(const int* pts, int b, int e, int x, int y, int h, int w) {
  bool on = false;
  int clt = 0, cle = 0;
  for (int k = b, j = e - 1; k < e; j = k++) {
    const long long X0 = pts[2 * j], Y0 = pts[2 * j + 1], X1 = pts[2 * k], Y1 = pts[2 * k + 1];
    const bool inimg = X0 >= 0 && X0 < w && X1 >= 0 && X1 < w && Y0 >= 0 && Y0 < h && Y1 >= 0 && Y1 < h;
    long long cx0 = X0, cy0 = Y0, cx1 = X1, cy1 = Y1;  // clipLine's copies (Line and the edge)
    bool vis = true;
    if (!inimg) vis = cv_clip_line(w, h, cx0, cy0, cx1, cy1);
    if (vis) {  // Line(img, t0, t1, 1, 8): left endpoint first
      long long lx1 = cx0, ly1 = cy0, lx2 = cx1, ly2 = cy1;
      if (lx2 < lx1) {
        lx1 = cx1; ly1 = cy1; lx2 = cx0; ly2 = cy0;
      }
      const long long ddx = lx2 - lx1, ddy = ly2 - ly1, ady = ddy < 0 ? -ddy : ddy;
      if (ady > ddx) {  // y major
        const long long i = ddy < 0 ? ly1 - y : y - ly1;
        if (i >= 0 && i <= ady) on |= x == lx1 + (2 * ddx * i + ady - 1) / (2 * ady);
      } else {
        const long long i = x - lx1;
        if (i >= 0 && i <= ddx) {
          const long long m = ddx ? (2 * ady * i + ddx - 1) / (2 * ddx) : 0;
          on |= y == (ddy < 0 ? ly1 - m : ly1 + m);
        }
      }
    }
    if (Y0 != Y1) {  // CollectPolyEdges' PolyEdge, then its x at row y
      long long c0x, c0y, c1x, c1y;
      if (inimg) {
        c0x = (X0 << 16) + 32768; c0y = Y0; c1x = (X1 << 16) + 32768; c1y = Y1;
      } else if (cy0 != cy1) {
        c0x = cx0 << 16; c0y = cy0; c1x = cx1 << 16; c1y = cy1;
      } else {
        c0x = X0 << 16; c0y = Y0; c1x = X1 << 16; c1y = Y1;
      }
      const long long dx = (c1x - c0x) / (c1y - c0y);  // C division: truncation toward zero
      long long y0, y1, x0;
      if (Y0 < Y1) {
        y0 = Y0; y1 = Y1; x0 = c0x + (Y0 - c0y) * dx;
      } else {
        y0 = Y1; y1 = Y0; x0 = c1x + (Y1 - c1y) * dx;
      }
      if (y >= y0 && y < y1) {
        const long long a = (x0 + (y - y0) * dx) >> 16;  // arithmetic shift: floor
        clt += a < x;
        cle += a <= x;
      }
    }
  }
  return on || (clt & 1) || cle > clt;
}

// Polygon i can only paint pixels inside its vertex bounding box: a Line pixel lies on its (clipped)
// segment's box, and a filled span runs between edge x values that truncation toward zero keeps
// within [min x, max x] of the edge's endpoints (x + 1/2 < max x + 1).
// Both rasterisers cull by it: the work is ~ sum of the polygons' box areas x edges, not
// pixels x all edges (a 640x480 LabelMe image with 40 cells: 205 -> ~10 us).
//
// Bounding boxes of polygons [p0, p0 + n) into LDS bb[0 .. n): the chunk's vertices split over the
// block's threads (coalesced), each vertex's polygon found by binary search in the LDS copy of
// poly_off, LDS integer min / max.  The caller syncs before (bb / offs reuse) and after.
constexpr int RCH = NT;  // polygons per LDS chunk
__device__ void chunk_bboxes(const int* pts, const int* poly_off, int p0, int n, int* offs, int4* bb) {
  for (int t = threadIdx.x; t <= n; t += NT) offs[t] = poly_off[p0 + t];
  for (int t = threadIdx.x; t < n; t += NT) bb[t] = make_int4(INT_MAX, INT_MAX, INT_MIN, INT_MIN);
  __syncthreads();
  const int v0 = offs[0], v1 = offs[n];
  for (int v = v0 + (int)threadIdx.x; v < v1; v += NT) {
    int lo = 0, hi = n - 1;  // the polygon t with offs[t] <= v < offs[t + 1] (empty polygons skipped)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (offs[mid] <= v) lo = mid;
      else hi = mid - 1;
    }
    const int x = pts[2 * v], y = pts[2 * v + 1];
    atomicMin(&bb[lo].x, x);
    atomicMin(&bb[lo].y, y);
    atomicMax(&bb[lo].z, x);
    atomicMax(&bb[lo].w, y);
  }
}

// semantic mask: one 16x16 pixel tile per block.  Per chunk of polygons the block keeps, in
// polygon order, those whose box meets the tile (ballot compaction), then every pixel tests only
// those: the last covering polygon wins, as dataset.py:197-201's loop paints.
constexpr int RT = 16;
__global__ __launch_bounds__(NT) void rasterize_kernel(const int* pts, const int* poly_off, const int* labels,
                                                       int npoly, int h, int w, int64_t* mask) {
  __shared__ int offs[RCH + 1];
  __shared__ int4 bb[RCH];
  __shared__ int list[RCH];
  __shared__ int wcnt[NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tx0 = blockIdx.x * RT, ty0 = blockIdx.y * RT;
  const int x = tx0 + (tid & (RT - 1)), y = ty0 + (tid >> 4);
  const int tx1 = min(tx0 + RT, w) - 1, ty1 = min(ty0 + RT, h) - 1;
  int64_t v = 0;
  for (int p0 = 0; p0 < npoly; p0 += RCH) {
    const int n = min(RCH, npoly - p0);
    __syncthreads();
    chunk_bboxes(pts, poly_off, p0, n, offs, bb);
    __syncthreads();
    bool hit = false;
    if (tid < n) {
      const int4 b = bb[tid];
      hit = b.x <= tx1 && b.z >= tx0 && b.y <= ty1 && b.w >= ty0;
    }
    const unsigned long long m = __ballot(hit);
    if (lane == 0) wcnt[wv] = __popcll(m);
    __syncthreads();
    int base = 0, cnt = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
      base += i < wv ? wcnt[i] : 0;
      cnt += wcnt[i];
    }
    if (hit) list[base + __popcll(m & ((1ull << lane) - 1ull))] = tid;
    __syncthreads();
    if (x < w && y < h)
      for (int j = 0; j < cnt; ++j) {
        const int t = list[j];
        const int4 b = bb[t];
        if (x < b.x || x > b.z || y < b.y || y > b.w) continue;
        if (cv_fillpoly_covers(pts, offs[t], offs[t + 1], x, y, h, w)) v = labels[p0 + t];
      }
  }
  if (x < w && y < h) mask[(long long)y * w + x] = v;
}

// one uint8 mask per polygon (dataset.py:184-186: cv2.fillPoly(mask, [points], 1)), same fill rule,
// with the training flips (dataset.py:209-222: every instance mask flipped like the image) applied
// as a mirrored read: out[i][y][x] = raster_i[flip_v ? h-1-y : y][flip_h ? w-1-x : x].
// blockIdx.y = polygon, blockIdx.x = a run of 4 NT output bytes (4 per thread, one 4-byte store
// when the run is aligned); bytes outside the polygon's box are zeros without a test.
__global__ __launch_bounds__(NT) void rasterize_instances_kernel(const int* pts, const int* poly_off, int npoly, int h,
                                                                 int w, int flip_h, int flip_v, uint8_t* masks) {
  __shared__ int4 wbb[NT / 64];
  const int p = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = poly_off[p], e = poly_off[p + 1];
  int4 bx = make_int4(INT_MAX, INT_MAX, INT_MIN, INT_MIN);
  for (int k = b + tid; k < e; k += NT) {
    const int xx = pts[2 * k], yy = pts[2 * k + 1];
    bx = make_int4(min(bx.x, xx), min(bx.y, yy), max(bx.z, xx), max(bx.w, yy));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    bx.x = min(bx.x, __shfl_xor(bx.x, o, 64));
    bx.y = min(bx.y, __shfl_xor(bx.y, o, 64));
    bx.z = max(bx.z, __shfl_xor(bx.z, o, 64));
    bx.w = max(bx.w, __shfl_xor(bx.w, o, 64));
  }
  if (lane == 0) wbb[wv] = bx;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    const int4 o = wbb[i];
    bx = make_int4(min(bx.x, o.x), min(bx.y, o.y), max(bx.z, o.z), max(bx.w, o.w));
  }
  const long long hw = (long long)h * w;
  const long long r0 = ((long long)blockIdx.x * NT + tid) * 4;
  if (r0 >= hw) return;
  uint8_t out[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    out[j] = 0;
    const long long r = r0 + j;
    if (r >= hw) continue;
    const int yo = (int)(r / w), xo = (int)(r - (long long)yo * w);
    const int y = flip_v ? h - 1 - yo : yo, x = flip_h ? w - 1 - xo : xo;
    if (x < bx.x || x > bx.z || y < bx.y || y > bx.w) continue;
    out[j] = cv_fillpoly_covers(pts, b, e, x, y, h, w) ? 1 : 0;
  }
  uint8_t* dst = masks + (long long)p * hw + r0;
  if (r0 + 4 <= hw && (((uintptr_t)dst) & 3) == 0) {
    *(uint32_t*)dst = (uint32_t)out[0] | ((uint32_t)out[1] << 8) | ((uint32_t)out[2] << 16) | ((uint32_t)out[3] << 24);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (r0 + j < hw) dst[j] = out[j];
  }
}

// flip a [h][w][c] byte image / int64 mask: mode 1 = horizontal (cv2.flip(., 1)), 0 = vertical
template <typename T>
__global__ __launch_bounds__(NT) void flip_kernel(const T* src, T* dst, int h, int w, int c, int mode) {
  const long long total = (long long)h * w * c;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int ch = (int)(i % c);
    const long long p = i / c;
    const int y = (int)(p / w), x = (int)(p - (long long)y * w);
    const int sy = mode == 0 ? h - 1 - y : y, sx = mode == 1 ? w - 1 - x : x;
    dst[i] = src[((long long)sy * w + sx) * c + ch];
  }
}

__device__ __forceinline__ uint8_t clip_u8(double v) {
  v = v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v);
  return (uint8_t)v;  // astype(np.uint8) truncates
}

// the numpy pixel ops in the reference's order; flags bit 0 alpha, 1 beta, 2 noise, 3 gamma LUT
__global__ __launch_bounds__(NT) void augment_kernel(uint8_t* img, long long n, int flags, double alpha,
                                                     double beta, const float* noise, const uint8_t* lut) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    uint8_t v = img[i];
    if (flags & 1) v = clip_u8((double)v * alpha);
    if (flags & 2) v = clip_u8((double)v + beta);
    if (flags & 4) v = clip_u8((double)((float)v + noise[i]));  // float32 image + float32 noise (:268)
    if (flags & 8) v = lut[v];
    img[i] = v;
  }
}

// dataset.py:225-257 with the live ratio read on the device: counts = eunet_semantic_counts of the
// (flipped) mask, live_ratio = #live / (#live + #dead) (0.5 without cells, :227-229); alpha / beta =
// random.uniform(a, b) = a + (b - a) u for the reference's ratio-dependent ranges, with u the
// host's random.random() draw -- the same double the reference forms (its uniform() draws exactly
// once in every branch), evaluated without FMA contraction as CPython does.  No host round trip.
__device__ __forceinline__ double uniform_ab(double a, double b, double u) { return __dadd_rn(a, __dmul_rn(b - a, u)); }

__global__ __launch_bounds__(NT) void augment_ratio_kernel(uint8_t* img, long long n, const long long* counts,
                                                           int flags, double ua, double ub) {
  const long long live = counts[3], dead = counts[6];  // counts[c][0] = #pixels of class c
  const long long total = live + dead;
  const double ratio = total > 0 ? (double)live / (double)total : 0.5;
  const double alpha = ratio > 0.6 ? uniform_ab(0.8, 1.3, ua) : (ratio < 0.4 ? uniform_ab(0.6, 1.1, ua) : uniform_ab(0.7, 1.3, ua));
  const double beta = ratio < 0.4 ? uniform_ab(-20.0, 40.0, ub) : uniform_ab(-30.0, 30.0, ub);
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    uint8_t v = img[i];
    if (flags & 1) v = clip_u8((double)v * alpha);
    if (flags & 2) v = clip_u8((double)v + beta);
    img[i] = v;
  }
}

// HWC uint8 -> CHW float32 / 255 (transforms.ToTensor), into out[c][h][w]
__global__ __launch_bounds__(NT) void to_tensor_kernel(const uint8_t* img, int h, int w, int c, float* out) {
  const long long hw = (long long)h * w, total = hw * c;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int ch = (int)(i / hw);
    const long long p = i - ch * hw;
    out[i] = (float)img[p * c + ch] / 255.f;
  }
}

// cv::resize coefficients of one axis (resize.cpp): fx = (float)((d + 0.5) * scale - 0.5) in double
// arithmetic with one cast, sx = floor(fx), fx -= sx; the caller clamps.  a = saturate_cast<short>
// ((1.f - fx, fx) * 2048): round half to even.
struct RCoef { int s, a0, a1; };
__device__ __forceinline__ RCoef resize_coef(int d, double scale) {
#pragma clang fp contract(off)
  float f = (float)(((double)d + 0.5) * scale - 0.5);
  const float fl = floorf(f);
  const int s = (int)fl;
  f = f - fl;
  return RCoef{s, __float2int_rn((1.f - f) * 2048.f), __float2int_rn(f * 2048.f)};
}

// one thread per output element.  mode 0: fixed-point bilinear (HResizeLinear rows, then the SIMD
// VResizeLinearVec_32s8u rounding for x < xvec, the scalar FixedPtCast tail after it); mode 1: the
// exact 2x downscale cv2 runs as INTER_AREA: (a + b + c + d + 2) >> 2.
__global__ __launch_bounds__(NT) void resize_u8_kernel(const uint8_t* src, int hi, int wi, int c, uint8_t* dst,
                                                       int ho, int wo, double scale_x, double scale_y, int mode,
                                                       int xvec) {
  const long long total = (long long)ho * wo * c;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int ch = (int)(i % c);
    const long long p = i / c;
    const int y = (int)(p / wo), x = (int)(p - (long long)y * wo);
    if (mode == 1) {
      const uint8_t* s0 = src + ((long long)(2 * y) * wi + 2 * x) * c + ch;
      const uint8_t* s1 = s0 + (long long)wi * c;
      dst[i] = (uint8_t)((s0[0] + s0[c] + s1[0] + s1[c] + 2) >> 2);
      continue;
    }
    RCoef cx = resize_coef(x, scale_x);
    if (cx.s < 0) cx = RCoef{0, 2048, 0};
    if (cx.s >= wi - 1) cx = RCoef{wi - 1, 2048, 0};
    const int sx1 = min(cx.s + 1, wi - 1);
    const RCoef cy = resize_coef(y, scale_y);
    const int y0 = min(max(cy.s, 0), hi - 1), y1 = min(max(cy.s + 1, 0), hi - 1);
    const uint8_t* r0 = src + (long long)y0 * wi * c + ch;
    const uint8_t* r1 = src + (long long)y1 * wi * c + ch;
    const int d0 = r0[(long long)cx.s * c] * cx.a0 + r0[(long long)sx1 * c] * cx.a1;
    const int d1 = r1[(long long)cx.s * c] * cx.a0 + r1[(long long)sx1 * c] * cx.a1;
    int v;
    if (x * c + ch < xvec) {  // 16-bit mulhi of the rows >> 4 (v_mul_hi), + 2 >> 2 (v_rshr_pack_u<2>)
      v = ((((d0 >> 4) * cy.a0) >> 16) + (((d1 >> 4) * cy.a1) >> 16) + 2) >> 2;
    } else {
      v = (cy.a0 * d0 + cy.a1 * d1 + (1 << 21)) >> 22;
    }
    dst[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

}  // namespace

extern "C" {

int eunet_rasterize_polygons(const int* pts, const int* poly_off, const int* labels, int npoly, int h, int w,
                             int64_t* mask, void* stream) {
  EUNET_REQUIRE(mask && h > 0 && w > 0 && npoly >= 0 && (npoly == 0 || (pts && poly_off && labels)),
                "rasterize_polygons: bad args");
  const dim3 g((unsigned)cdiv(w, RT), (unsigned)cdiv(h, RT));
  rasterize_kernel<<<g, NT, 0, (hipStream_t)stream>>>(pts, poly_off, labels, npoly, h, w, mask);
  EUNET_LAUNCH_CHECK("rasterize_polygons");
  return EUNET_OK;
}

int eunet_rasterize_instances(const int* pts, const int* poly_off, int npoly, int h, int w, int flip_h,
                              int flip_v, uint8_t* masks, void* stream) {
  EUNET_REQUIRE(masks && h > 0 && w > 0 && npoly > 0 && pts && poly_off, "rasterize_instances: bad args");
  EUNET_REQUIRE(npoly <= 65535 && ((long long)h * w + 4 * NT - 1) / (4 * NT) < (1ll << 31),
                "rasterize_instances: too many polygons / pixels");
  const dim3 g((unsigned)(((long long)h * w + 4 * NT - 1) / (4 * NT)), (unsigned)npoly);
  rasterize_instances_kernel<<<g, NT, 0, (hipStream_t)stream>>>(pts, poly_off, npoly, h, w, flip_h, flip_v, masks);
  EUNET_LAUNCH_CHECK("rasterize_instances");
  return EUNET_OK;
}

int eunet_flip_u8(const uint8_t* src, uint8_t* dst, int h, int w, int c, int mode, void* stream) {
  EUNET_REQUIRE(src && dst && src != dst && h > 0 && w > 0 && c > 0 && (mode == 0 || mode == 1),
                "flip_u8: bad args");
  flip_kernel<uint8_t><<<grid1((long long)h * w * c), NT, 0, (hipStream_t)stream>>>(src, dst, h, w, c, mode);
  EUNET_LAUNCH_CHECK("flip_u8");
  return EUNET_OK;
}

int eunet_flip_mask(const int64_t* src, int64_t* dst, int h, int w, int mode, void* stream) {
  EUNET_REQUIRE(src && dst && src != dst && h > 0 && w > 0 && (mode == 0 || mode == 1), "flip_mask: bad args");
  flip_kernel<int64_t><<<grid1((long long)h * w), NT, 0, (hipStream_t)stream>>>(src, dst, h, w, 1, mode);
  EUNET_LAUNCH_CHECK("flip_mask");
  return EUNET_OK;
}

int eunet_augment_u8(uint8_t* img, long long n, int flags, double alpha, double beta, const float* noise,
                     const uint8_t* lut, void* stream) {
  EUNET_REQUIRE(img && n > 0 && (!(flags & 4) || noise) && (!(flags & 8) || lut), "augment_u8: bad args");
  augment_kernel<<<grid1(n), NT, 0, (hipStream_t)stream>>>(img, n, flags, alpha, beta, noise, lut);
  EUNET_LAUNCH_CHECK("augment_u8");
  return EUNET_OK;
}

int eunet_augment_ratio_u8(uint8_t* img, long long n, const long long* counts, int flags, double u_alpha,
                           double u_beta, void* stream) {
  EUNET_REQUIRE(img && n > 0 && counts && (flags & ~3) == 0, "augment_ratio_u8: bad args");
  augment_ratio_kernel<<<grid1(n), NT, 0, (hipStream_t)stream>>>(img, n, counts, flags, u_alpha, u_beta);
  EUNET_LAUNCH_CHECK("augment_ratio_u8");
  return EUNET_OK;
}

int eunet_to_tensor(const uint8_t* img, int h, int w, int c, float* out, void* stream) {
  EUNET_REQUIRE(img && out && h > 0 && w > 0 && c > 0, "to_tensor: bad args");
  to_tensor_kernel<<<grid1((long long)h * w * c), NT, 0, (hipStream_t)stream>>>(img, h, w, c, out);
  EUNET_LAUNCH_CHECK("to_tensor");
  return EUNET_OK;
}

int eunet_resize_u8(const uint8_t* src, int hi, int wi, int c, uint8_t* dst, int ho, int wo, void* stream) {
  EUNET_REQUIRE(src && dst && hi > 0 && wi > 0 && ho > 0 && wo > 0 && c > 0, "resize_u8: bad args");
  if (hi == ho && wi == wo) {  // cv::resize copies
    const hipError_t e = hipMemcpyAsync(dst, src, (size_t)hi * wi * c, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    EUNET_REQUIRE(e == hipSuccess, "resize_u8: copy failed");
    return EUNET_OK;
  }
  // cv::hal::resize: scale = 1 / inv_scale, inv_scale = dsize / ssize; an exact 2x downscale in both
  // directions runs as INTER_AREA
  const double scale_x = 1.0 / ((double)wo / wi), scale_y = 1.0 / ((double)ho / hi);
  const double ix = std::nearbyint(scale_x), iy = std::nearbyint(scale_y);
  const double eps = 2.220446049250313e-16;
  const int mode = std::fabs(scale_x - ix) < eps && std::fabs(scale_y - iy) < eps && ix == 2.0 && iy == 2.0;
  // elements of a row the 128-bit vector loops of VResizeLinearVec_32s8u cover (16, then 8 at a time)
  const int width = wo * c;
  int xvec = width >= 16 ? width / 16 * 16 : 0;
  while (xvec < width - 8) xvec += 8;
  resize_u8_kernel<<<grid1((long long)ho * wo * c), NT, 0, (hipStream_t)stream>>>(src, hi, wi, c, dst, ho, wo,
                                                                                   scale_x, scale_y, mode, xvec);
  EUNET_LAUNCH_CHECK("resize_u8");
  return EUNET_OK;
}

}  // extern "C"
