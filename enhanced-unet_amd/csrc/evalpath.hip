// Evaluation path: semantic metrics, test-time-augmentation resampling, softmax
// and the thresholded probability -> mask conversion.
//
// Reference: metrics.py:12-58 (calculate_iou / calculate_dice /
// calculate_semantic_metrics), train_eval.py:397-453 (_run_model_single,
// _run_tta_inference), train_eval.py:455-568 (_convert_probs_to_mask).
// All of it is HBM-bound integer / per-pixel work: one pass per op, 16-byte or
// 8-byte lanes, block-level integer reductions (exact, order-free).
#include "common.h"

namespace {

constexpr int NT = 256;

// ---- semantic counts: per sample, per class c in {0,1,2}:
//      [pred == c], [gt == c], [pred == c && gt == c]   (metrics.py:38-45)
__global__ __launch_bounds__(NT) void semantic_counts_kernel(const int64_t* pred, const int64_t* gt, long long hw,
                                                             unsigned long long* counts) {
  const int n = blockIdx.y;
  const int64_t* p = pred + (long long)n * hw;
  const int64_t* g = gt + (long long)n * hw;
  unsigned int c[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) c[i] = 0;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < hw; i += (long long)gridDim.x * NT) {
    const int64_t a = p[i], b = g[i];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      c[k * 3 + 0] += a == k;
      c[k * 3 + 1] += b == k;
      c[k * 3 + 2] += (a == k) & (b == k);
    }
  }
  __shared__ unsigned int red[NT / 64][9];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    unsigned int v = c[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wv][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < 9) {
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += red[w][threadIdx.x];
    if (t) atomicAdd(counts + n * 9 + threadIdx.x, t);
  }
}

// ---- binary overlap of two integer masks (metrics.py:12-26): out = (#(a!=0 & b!=0),
//      #(a!=0 | b!=0), sum a, sum b); the Dice denominator is the sum of the VALUES.
__global__ __launch_bounds__(NT) void binary_overlap_kernel(const int64_t* a, const int64_t* b, long long n,
                                                            unsigned long long* out) {
  unsigned long long c[4] = {0, 0, 0, 0};
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const int64_t x = a[i], y = b[i];
    c[0] += (x != 0) & (y != 0);
    c[1] += (x != 0) | (y != 0);
    c[2] += (unsigned long long)x;
    c[3] += (unsigned long long)y;
  }
  __shared__ unsigned long long red[NT / 64][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned long long v = c[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wv][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += red[w][threadIdx.x];
    if (t) atomicAdd(out + threadIdx.x, t);
  }
}

// ---- bilinear resample, PyTorch upsample_bilinear2d semantics (align_corners=False):
// src = max(scale * (dst + 0.5) - 0.5, 0); i0 = (int)src; i1 = i0 + (i0 < in-1);
// l1 = src - i0.  scale = 1/scale_factor when F.interpolate got scale_factor, else in/out.
// Optional flips of the destination index (torch.flip composed with the copy).
__device__ __forceinline__ void src_index(int d, int in, float scale, int& i0, int& i1, float& l1) {
  float s = scale * ((float)d + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = (int)s;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
}

__global__ __launch_bounds__(NT) void resize_bilinear_kernel(const float* x, int planes, int hin, int win, float* y,
                                                             int hout, int wout, float sh, float sw, int flip_h,
                                                             int flip_w) {
  const long long total = (long long)planes * hout * wout;
  for (long long id = (long long)blockIdx.x * NT + threadIdx.x; id < total; id += (long long)gridDim.x * NT) {
    const int ox = (int)(id % wout);
    const long long r = id / wout;
    const int oy = (int)(r % hout);
    const long long pl = r / hout;
    const int dy = flip_h ? hout - 1 - oy : oy, dx = flip_w ? wout - 1 - ox : ox;
    int y0, y1, x0, x1;
    float ly1, lx1;
    src_index(dy, hin, sh, y0, y1, ly1);
    src_index(dx, win, sw, x0, x1, lx1);
    const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
    const float* p = x + pl * hin * win;
    const float v = ly0 * (lx0 * p[(long long)y0 * win + x0] + lx1 * p[(long long)y0 * win + x1]) +
                    ly1 * (lx0 * p[(long long)y1 * win + x0] + lx1 * p[(long long)y1 * win + x1]);
    y[id] = v;
  }
}

// ---- softmax over K of a cropped (and optionally flipped) logit map:
// logits [K][hp][wp] -> probs [K][h][w], probs[k][y][x] = softmax(logits[:, y', x'])[k]
// with y' = flip_h ? h-1-y : y (the crop keeps rows/cols < h, w; train_eval.py:412-415, 430-437)
template <int K>
__global__ __launch_bounds__(NT) void softmax_crop_kernel(const float* logits, int hp, int wp, int h, int w,
                                                          int flip_h, int flip_w, float* probs) {
  const long long total = (long long)h * w;
  for (long long id = (long long)blockIdx.x * NT + threadIdx.x; id < total; id += (long long)gridDim.x * NT) {
    const int x = (int)(id % w), yy = (int)(id / w);
    const int sy = flip_h ? h - 1 - yy : yy, sx = flip_w ? w - 1 - x : x;
    const long long s = (long long)sy * wp + sx;
    float v[K], m = -INFINITY;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      v[k] = logits[(long long)k * hp * wp + s];
      m = fmaxf(m, v[k]);
    }
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      v[k] = expf(v[k] - m);
      sum += v[k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) probs[(long long)k * total + id] = v[k] / sum;
  }
}

// acc = mode 0: p ; mode 1: acc + p ; mode 2: (acc + p) / count
__global__ __launch_bounds__(NT) void accumulate_kernel(float* acc, const float* p, long long n, int mode,
                                                        float count) {
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float v = mode == 0 ? p[i] : acc[i] + p[i];
    if (mode == 2) v = v / count;
    acc[i] = v;
  }
}

// ---- _convert_probs_to_mask, pass 1 (train_eval.py:465-531): per-pixel rules up to the
// very-low-confidence cleanup; counts[0..1] = #live, #dead pixels of that mask.
// K = 2 generalisation: dead_prob = 0 (the reference indexes probs[2] and needs K = 3).
template <int K>
__global__ __launch_bounds__(NT) void probs_mask_pass1(const float* probs, long long hw, int64_t* mask,
                                                       unsigned long long* counts) {
  unsigned int nl = 0, nd = 0;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < hw; i += (long long)gridDim.x * NT) {
    const float bg = probs[i], live = probs[hw + i];
    const float dead = K == 3 ? probs[2 * hw + i] : 0.f;
    // argmax, first index wins ties (torch.argmax)
    int pm = 0;
    float mx = bg;
    if (live > mx) { pm = 1; mx = live; }
    if (K == 3 && dead > mx) { pm = 2; mx = dead; }
    const float max_prob = mx;  // torch.max(probs, 0)[0]
    if (pm == 1 && (live < 0.42f || live <= bg * 1.15f)) pm = 0;
    if (pm == 2 && (dead < 0.5f || dead <= bg * 1.3f || bg > 0.3f || live > dead * 0.9f)) pm = 0;
    const bool bg_high_live = pm == 0 && live > 0.42f && live > bg * 1.15f && live > dead * 1.05f;
    if (bg_high_live) pm = 1;
    const bool bg_high_dead = pm == 0 && dead > 0.5f && dead > bg * 1.3f && dead > live * 1.1f && bg < 0.3f &&
                              !bg_high_live;
    if (bg_high_dead) pm = 2;
    if (pm == 1 && dead > live * 1.15f && dead > 0.45f) pm = 2;
    if (pm == 2 && live > dead * 1.15f && live > 0.42f) pm = 1;
    if (max_prob < 0.3f) pm = 0;
    mask[i] = pm;
    nl += pm == 1;
    nd += pm == 2;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nl += __shfl_xor(nl, o, 64);
    nd += __shfl_xor(nd, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (nl) atomicAdd(counts + 0, (unsigned long long)nl);
    if (nd) atomicAdd(counts + 1, (unsigned long long)nd);
  }
}

// pass 2 (train_eval.py:533-563): the pixel-ratio-conditioned refinement.  Both ratios are
// taken from the pass-1 mask (the reference computes them before either filter) in fp64.
template <int K>
__global__ __launch_bounds__(NT) void probs_mask_pass2(const float* probs, long long hw, int64_t* mask,
                                                       const unsigned long long* counts) {
  const double live_ratio = (double)counts[0] / (double)hw, dead_ratio = (double)counts[1] / (double)hw;
  const bool flive = live_ratio > 0.5, fdead = dead_ratio > 0.15;
  if (!flive && !fdead) return;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < hw; i += (long long)gridDim.x * NT) {
    const int64_t pm = mask[i];
    const float bg = probs[i], live = probs[hw + i];
    const float dead = K == 3 ? probs[2 * hw + i] : 0.f;
    if (flive && pm == 1) {
      const bool hc = live > 0.5f && live > bg * 1.3f && bg < 0.3f;
      if (!hc) mask[i] = 0;
    }
    if (fdead && pm == 2) {
      bool hc;
      if (dead_ratio > 0.4)
        hc = dead > 0.65f && dead > bg * 1.6f && bg < 0.2f && live < dead * 0.7f;
      else if (dead_ratio > 0.25)
        hc = dead > 0.6f && dead > bg * 1.5f && bg < 0.25f && live < dead * 0.8f;
      else
        hc = dead > 0.55f && dead > bg * 1.4f && bg < 0.25f;
      if (!hc) mask[i] = 0;
    }
  }
}

unsigned grid_for(long long n) {
  long long b = (n + NT - 1) / NT;
  if (b > 8192) b = 8192;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

extern "C" {

int eunet_semantic_counts(const int64_t* pred, const int64_t* gt, int n, long long hw, int64_t* counts,
                          void* stream) {
  EUNET_REQUIRE(pred && gt && counts && n > 0 && hw > 0, "semantic_counts: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(counts, 0, sizeof(int64_t) * 9 * n, s) != hipSuccess) {
    eunet::set_error("semantic_counts: memset failed");
    return EUNET_ERR_HIP;
  }
  long long bx = (hw + NT - 1) / NT;
  if (bx > 1024) bx = 1024;
  semantic_counts_kernel<<<dim3((unsigned)bx, n), NT, 0, s>>>(pred, gt, hw, (unsigned long long*)counts);
  EUNET_LAUNCH_CHECK("semantic_counts");
  return EUNET_OK;
}

int eunet_binary_overlap(const int64_t* a, const int64_t* b, long long n, int64_t* out, void* stream) {
  EUNET_REQUIRE(a && b && out && n > 0, "binary_overlap: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(out, 0, 4 * sizeof(int64_t), s) != hipSuccess) {
    eunet::set_error("binary_overlap: memset failed");
    return EUNET_ERR_HIP;
  }
  binary_overlap_kernel<<<grid_for(n) > 1024 ? 1024 : grid_for(n), NT, 0, s>>>(a, b, n, (unsigned long long*)out);
  EUNET_LAUNCH_CHECK("binary_overlap");
  return EUNET_OK;
}

int eunet_resize_bilinear(const float* x, int planes, int hin, int win, float* y, int hout, int wout, float scale_h,
                          float scale_w, int flip_h, int flip_w, void* stream) {
  EUNET_REQUIRE(x && y && planes > 0 && hin > 0 && win > 0 && hout > 0 && wout > 0 && scale_h > 0.f &&
                    scale_w > 0.f,
                "resize_bilinear: bad args");
  const long long total = (long long)planes * hout * wout;
  resize_bilinear_kernel<<<grid_for(total), NT, 0, (hipStream_t)stream>>>(x, planes, hin, win, y, hout, wout, scale_h,
                                                                          scale_w, flip_h, flip_w);
  EUNET_LAUNCH_CHECK("resize_bilinear");
  return EUNET_OK;
}

int eunet_softmax_crop(const float* logits, int k, int hp, int wp, int h, int w, int flip_h, int flip_w,
                       float* probs, void* stream) {
  EUNET_REQUIRE(logits && probs && (k == 2 || k == 3) && h > 0 && w > 0 && h <= hp && w <= wp,
                "softmax_crop: bad args (K must be 2 or 3, crop inside the map)");
  const unsigned g = grid_for((long long)h * w);
  if (k == 3)
    softmax_crop_kernel<3><<<g, NT, 0, (hipStream_t)stream>>>(logits, hp, wp, h, w, flip_h, flip_w, probs);
  else
    softmax_crop_kernel<2><<<g, NT, 0, (hipStream_t)stream>>>(logits, hp, wp, h, w, flip_h, flip_w, probs);
  EUNET_LAUNCH_CHECK("softmax_crop");
  return EUNET_OK;
}

int eunet_accumulate(float* acc, const float* p, long long n, int mode, float count, void* stream) {
  EUNET_REQUIRE(acc && p && n > 0 && mode >= 0 && mode <= 2 && count > 0.f, "accumulate: bad args");
  accumulate_kernel<<<grid_for(n), NT, 0, (hipStream_t)stream>>>(acc, p, n, mode, count);
  EUNET_LAUNCH_CHECK("accumulate");
  return EUNET_OK;
}

int eunet_probs_to_mask(const float* probs, int k, int h, int w, int64_t* mask, int64_t* counts, void* stream) {
  EUNET_REQUIRE(probs && mask && counts && (k == 2 || k == 3) && h > 0 && w > 0, "probs_to_mask: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(counts, 0, 2 * sizeof(int64_t), s) != hipSuccess) {
    eunet::set_error("probs_to_mask: memset failed");
    return EUNET_ERR_HIP;
  }
  const long long hw = (long long)h * w;
  const unsigned g = grid_for(hw);
  unsigned long long* c = (unsigned long long*)counts;
  if (k == 3) {
    probs_mask_pass1<3><<<g, NT, 0, s>>>(probs, hw, mask, c);
    probs_mask_pass2<3><<<g, NT, 0, s>>>(probs, hw, mask, c);
  } else {
    probs_mask_pass1<2><<<g, NT, 0, s>>>(probs, hw, mask, c);
    probs_mask_pass2<2><<<g, NT, 0, s>>>(probs, hw, mask, c);
  }
  EUNET_LAUNCH_CHECK("probs_to_mask");
  return EUNET_OK;
}

}  // extern "C"
