// The 2x-resolution tail of EnhancedUNet (fallback), fused and recomputed.
//
// Reference: models.py:236 (d1 = dec1(upsample(d2))), 308-313 + 336-337
// (out = d1 + enhance(d1), enhance = Conv3x3(K->64)+BN+ReLU+Conv1x1(64->K)),
// train_eval.py:306-310 (bilinear 2H->H resize, == exact 2x2 mean).
//
// dec1 commutes with the upsample, so the host passes z = dec1(d2) at H
// (K channels).  Everything at 2H -- u = up(z), the 64-channel conv output h,
// BN, ReLU, the 1x1, the residual and the 2x2 mean -- is recomputed per 16x16
// tile from z and never stored: the largest tensor of the network (64 ch at
// 2H) costs no HBM traffic.  Passes: fwd = stats, out; bwd = bwd1 (1x1 and BN
// reductions), bwd2 (g_h, gW1, and g_u = W1^T g_h + g_o) + upsample adjoint.
// All fp32 (vector ALU; ~1.5 % of the step FLOPs).
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr int T2 = 16;  // tile side at 2H
constexpr int MID = 64;

struct HeadArgs {
  const float* z; int N, h, w, K;
  const float* w1; const float* b1;
  const float* gamma; const float* beta; const float* w2; const float* b2;
  const float* mean; const float* istd;   // bwd
  const float* scale; const float* shift; // fwd out
  const float* glog; const float* gout2h;
  const float* dbeta; const float* dgamma; // bwd2
  float* stats; float* out2h; float* logits; float* part; float* gu;
  int tx, ty, ntiles;
};

__device__ __forceinline__ float up_val(const HeadArgs& a, int n, int oy, int ox, int k) {
  int y0, y1, x0, x1;
  float ly, lx;
  up2_src(oy, a.h, y0, y1, ly);
  up2_src(ox, a.w, x0, x1, lx);
  const float* zb = a.z + (long long)n * a.h * a.w * a.K;
  const float v00 = zb[((long long)y0 * a.w + x0) * a.K + k], v01 = zb[((long long)y0 * a.w + x1) * a.K + k];
  const float v10 = zb[((long long)y1 * a.w + x0) * a.K + k], v11 = zb[((long long)y1 * a.w + x1) * a.K + k];
  return (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
}

// fill su[(R x R) region starting at (oy0-off, ox0-off)][K], zero outside the image
__device__ void fill_u(const HeadArgs& a, float* su, int n, int oy0, int ox0, int R, int off) {
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  for (int i = threadIdx.x; i < R * R; i += NT) {
    const int hy = i / R, hx = i - hy * R;
    const int oy = oy0 + hy - off, ox = ox0 + hx - off;
    const bool in = oy >= 0 && oy < H2 && ox >= 0 && ox < W2;
    for (int k = 0; k < a.K; ++k) su[i * 3 + k] = in ? up_val(a, n, oy, ox, k) : 0.f;
  }
}

// h[c] for the pixel whose 3x3 window starts at su cell (sy, sx) (region width R)
template <int K>
__device__ __forceinline__ void conv_h(const float* su, const float* w1s, const float* b1s, int sy, int sx, int R,
                                       float (&h)[MID]) {
  float uk[K * 9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ky = t / 3, kx = t - ky * 3;
#pragma unroll
    for (int k = 0; k < K; ++k) uk[k * 9 + t] = su[((sy + ky) * R + sx + kx) * 3 + k];
  }
#pragma unroll
  for (int c = 0; c < MID; ++c) {
    float s = b1s[c];
#pragma unroll
    for (int j = 0; j < K * 9; ++j) s = fmaf(w1s[c * K * 9 + j], uk[j], s);
    h[c] = s;
  }
}

__device__ __forceinline__ void tile_coords(const HeadArgs& a, int tile, int& n, int& oy0, int& ox0) {
  const int tpi = a.tx * a.ty;
  n = tile / tpi;
  const int r = tile - n * tpi;
  oy0 = (r / a.tx) * T2;
  ox0 = (r % a.tx) * T2;
}

// thread -> pixel inside a 16x16 tile, 2x2 quads on lanes 4j..4j+3
__device__ __forceinline__ void quad_pixel(int tid, int& r, int& c) {
  const int blk = tid >> 2, sub = tid & 3;
  r = 2 * (blk >> 3) + (sub >> 1);
  c = 2 * (blk & 7) + (sub & 1);
}

template <int K>
__global__ __launch_bounds__(NT) void head_stats_kernel(HeadArgs a) {
  __shared__ float w1s[MID * K * 9], b1s[MID], su[18 * 18 * 3];
  __shared__ float red[4][MID], meanb[MID], sums[MID];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int n, oy0, ox0;
  tile_coords(a, blockIdx.x, n, oy0, ox0);
  for (int i = tid; i < MID * K * 9; i += NT) w1s[i] = a.w1[i];
  if (tid < MID) b1s[tid] = a.b1[tid];
  fill_u(a, su, n, oy0, ox0, 18, 1);
  __syncthreads();
  const int r = tid / T2, c = tid % T2;
  const bool pv = oy0 + r < 2 * a.h && ox0 + c < 2 * a.w;
  float h[MID];
  conv_h<K>(su, w1s, b1s, r, c, 18, h);
  float v[MID];
#pragma unroll
  for (int i = 0; i < MID; ++i) v[i] = pv ? h[i] : 0.f;
  red[wv][lane] = wave_transpose_reduce64(v);
  __syncthreads();
  const float cnt = (float)(min(T2, 2 * a.h - oy0) * min(T2, 2 * a.w - ox0));
  if (tid < MID) {
    sums[tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    meanb[tid] = sums[tid] / cnt;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < MID; ++i) {
    const float d = h[i] - meanb[i];
    v[i] = pv ? d * d : 0.f;
  }
  const float m2 = wave_transpose_reduce64(v);
  __syncthreads();
  red[wv][lane] = m2;
  __syncthreads();
  if (tid < MID) {
    a.stats[((long long)blockIdx.x * 2 + 0) * MID + tid] = sums[tid];
    a.stats[((long long)blockIdx.x * 2 + 1) * MID + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    if (tid == 0) a.stats[(long long)2 * MID * a.ntiles + blockIdx.x] = cnt;
  }
}

template <int K>
__global__ __launch_bounds__(NT) void head_out_kernel(HeadArgs a) {
  __shared__ float w1s[MID * K * 9], b1s[MID], su[18 * 18 * 3], sc[MID], sh[MID], w2s[K * MID];
  const int tid = threadIdx.x;
  int n, oy0, ox0;
  tile_coords(a, blockIdx.x, n, oy0, ox0);
  for (int i = tid; i < MID * K * 9; i += NT) w1s[i] = a.w1[i];
  for (int i = tid; i < K * MID; i += NT) w2s[i] = a.w2[i];
  if (tid < MID) {
    b1s[tid] = a.b1[tid];
    sc[tid] = a.scale[tid];
    sh[tid] = a.shift[tid];
  }
  fill_u(a, su, n, oy0, ox0, 18, 1);
  __syncthreads();
  int r, c;
  quad_pixel(tid, r, c);
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  const int oy = oy0 + r, ox = ox0 + c;
  const bool pv = oy < H2 && ox < W2;
  float h[MID];
  conv_h<K>(su, w1s, b1s, r, c, 18, h);
  float o[K];
#pragma unroll
  for (int k = 0; k < K; ++k) o[k] = a.b2[k];
#pragma unroll
  for (int i = 0; i < MID; ++i) {
    const float act = fmaxf(fmaf(h[i], sc[i], sh[i]), 0.f);
#pragma unroll
    for (int k = 0; k < K; ++k) o[k] = fmaf(w2s[k * MID + i], act, o[k]);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float u = su[((r + 1) * 18 + c + 1) * 3 + k];
    const float val = u + o[k];
    if (pv && a.out2h) a.out2h[(((long long)n * K + k) * H2 + oy) * W2 + ox] = val;
    float s = val + __shfl_xor(val, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (pv && a.logits && (tid & 3) == 0)
      a.logits[(((long long)n * K + k) * a.h + (oy >> 1)) * a.w + (ox >> 1)] = 0.25f * s;
  }
}

__device__ __forceinline__ float g_out(const HeadArgs& a, int K, int n, int k, int oy, int ox) {
  if (a.glog) return 0.25f * a.glog[(((long long)n * K + k) * a.h + (oy >> 1)) * a.w + (ox >> 1)];
  return a.gout2h[(((long long)n * K + k) * (2 * a.h) + oy) * (2 * a.w) + ox];
}

// pass 1: gW2, gb2 and the BN backward sums (dbeta = sum g_bn, dgamma = sum g_bn*xhat)
template <int K>
__global__ __launch_bounds__(NT) void head_bwd1_kernel(HeadArgs a) {
  __shared__ float w1s[MID * K * 9], b1s[MID], su[18 * 18 * 3], ga[MID], be[MID], mu[MID], is[MID], w2s[K * MID];
  __shared__ float acc_s[(K + 2) * MID + K];
  const int tid = threadIdx.x, lane = tid & 63;
  int n, oy0, ox0;
  tile_coords(a, blockIdx.x, n, oy0, ox0);
  for (int i = tid; i < MID * K * 9; i += NT) w1s[i] = a.w1[i];
  for (int i = tid; i < K * MID; i += NT) w2s[i] = a.w2[i];
  for (int i = tid; i < (K + 2) * MID + K; i += NT) acc_s[i] = 0.f;
  if (tid < MID) {
    b1s[tid] = a.b1[tid];
    ga[tid] = a.gamma[tid];
    be[tid] = a.beta[tid];
    mu[tid] = a.mean[tid];
    is[tid] = a.istd[tid];
  }
  fill_u(a, su, n, oy0, ox0, 18, 1);
  __syncthreads();
  int r, c;
  quad_pixel(tid, r, c);
  const int oy = oy0 + r, ox = ox0 + c;
  const bool pv = oy < 2 * a.h && ox < 2 * a.w;
  float h[MID];
  conv_h<K>(su, w1s, b1s, r, c, 18, h);
  float go[K];
#pragma unroll
  for (int k = 0; k < K; ++k) go[k] = pv ? g_out(a, K, n, k, oy, ox) : 0.f;
  float v[MID];
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int i = 0; i < MID; ++i) {
      const float xh = (h[i] - mu[i]) * is[i];
      v[i] = go[k] * fmaxf(fmaf(ga[i], xh, be[i]), 0.f);
    }
    atomicAdd(&acc_s[k * MID + lane], wave_transpose_reduce64(v));
  }
  // g_bn = (W2^T go) * [a > 0]
#pragma unroll
  for (int i = 0; i < MID; ++i) {
    const float xh = (h[i] - mu[i]) * is[i];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) s = fmaf(w2s[k * MID + i], go[k], s);
    v[i] = (fmaf(ga[i], xh, be[i]) > 0.f) ? s : 0.f;
  }
  // keep g_bn in h (h no longer needed after computing xhat * g_bn)
#pragma unroll
  for (int i = 0; i < MID; ++i) {
    const float xh = (h[i] - mu[i]) * is[i];
    h[i] = v[i] * xh;
  }
  atomicAdd(&acc_s[K * MID + lane], wave_transpose_reduce64(v));
  atomicAdd(&acc_s[(K + 1) * MID + lane], wave_transpose_reduce64(h));
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float s = wave_sum(go[k]);
    if (lane == 0) atomicAdd(&acc_s[(K + 2) * MID + k], s);
  }
  __syncthreads();
  const int stride = (K + 2) * MID + K;
  for (int i = tid; i < stride; i += NT) a.part[(long long)blockIdx.x * stride + i] = acc_s[i];
}

// pass 2: g_h on the tile + 1-px halo -> gW1/gb1 partials and g_u (written to a.gu)
template <int K>
__global__ __launch_bounds__(NT) void head_bwd2_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float dyn[];
  float* sgh = dyn;                  // [324][65]
  float* su = sgh + 324 * 65;        // [400][3]
  float* w1s = su + 400 * 3;         // [64*K*9]
  float* b1s = w1s + MID * K * 9;    // [64]
  float* prm = b1s + MID;            // ga, be, mu, is, dbeta, dgamma [6][64]
  float* w2s = prm + 6 * MID;        // [K*64]
  const int tid = threadIdx.x;
  int n, oy0, ox0;
  tile_coords(a, blockIdx.x, n, oy0, ox0);
  for (int i = tid; i < MID * K * 9; i += NT) w1s[i] = a.w1[i];
  for (int i = tid; i < K * MID; i += NT) w2s[i] = a.w2[i];
  if (tid < MID) {
    b1s[tid] = a.b1[tid];
    prm[0 * MID + tid] = a.gamma[tid];
    prm[1 * MID + tid] = a.beta[tid];
    prm[2 * MID + tid] = a.mean[tid];
    prm[3 * MID + tid] = a.istd[tid];
    prm[4 * MID + tid] = a.dbeta[tid];
    prm[5 * MID + tid] = a.dgamma[tid];
  }
  fill_u(a, su, n, oy0, ox0, 20, 2);
  __syncthreads();
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  const float inv_cnt = 1.f / ((float)a.N * (float)H2 * (float)W2);
  for (int i = tid; i < 18 * 18; i += NT) {
    const int gy = i / 18, gx = i - gy * 18;
    const int oy = oy0 + gy - 1, ox = ox0 + gx - 1;
    float* dst = sgh + i * 65;
    if (oy < 0 || oy >= H2 || ox < 0 || ox >= W2) {
      for (int ch = 0; ch < MID; ++ch) dst[ch] = 0.f;
      continue;
    }
    float h[MID];
    conv_h<K>(su, w1s, b1s, gy, gx, 20, h);
    float go[K];
#pragma unroll
    for (int k = 0; k < K; ++k) go[k] = g_out(a, K, n, k, oy, ox);
#pragma unroll
    for (int ch = 0; ch < MID; ++ch) {
      const float xh = (h[ch] - prm[2 * MID + ch]) * prm[3 * MID + ch];
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) s = fmaf(w2s[k * MID + ch], go[k], s);
      const float gbn = (fmaf(prm[ch], xh, prm[MID + ch]) > 0.f) ? s : 0.f;
      dst[ch] = prm[ch] * prm[3 * MID + ch] *
                (gbn - prm[4 * MID + ch] * inv_cnt - xh * prm[5 * MID + ch] * inv_cnt);
    }
  }
  __syncthreads();
  // g_u for the interior pixel of this thread
  {
    const int r = tid / T2, c = tid % T2;
    const int oy = oy0 + r, ox = ox0 + c;
    if (oy < H2 && ox < W2) {
      float acc[K];
#pragma unroll
      for (int k = 0; k < K; ++k) acc[k] = g_out(a, K, n, k, oy, ox);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t - ky * 3;
        const float* gp = sgh + ((r - ky + 2) * 18 + (c - kx + 2)) * 65;
        for (int ch = 0; ch < MID; ++ch) {
          const float g = gp[ch];
#pragma unroll
          for (int k = 0; k < K; ++k) acc[k] = fmaf(w1s[ch * K * 9 + k * 9 + t], g, acc[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < K; ++k) a.gu[(((long long)n * H2 + oy) * W2 + ox) * K + k] = acc[k];
    }
  }
  // gW1 / gb1 partials
  {
    const int ch = tid & 63, tg = tid >> 6;
    float acc[3][K];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int k = 0; k < K; ++k) acc[j][k] = 0.f;
    float gb = 0.f;
    for (int p = 0; p < T2 * T2; ++p) {
      const int r = p / T2, c = p - r * T2;
      const float g = sgh[((r + 1) * 18 + c + 1) * 65 + ch];
      gb += g;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int t = tg + 4 * j;
        if (t < 9) {
          const int ky = t / 3, kx = t - ky * 3;
          const float* up = su + ((r + ky + 1) * 20 + c + kx + 1) * 3;
#pragma unroll
          for (int k = 0; k < K; ++k) acc[j][k] = fmaf(g, up[k], acc[j][k]);
        }
      }
    }
    const int stride = MID * K * 9 + MID;
    float* out = a.part + (long long)blockIdx.x * stride;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int t = tg + 4 * j;
      if (t < 9)
#pragma unroll
        for (int k = 0; k < K; ++k) out[(ch * K + k) * 9 + t] = acc[j][k];
    }
    if (tg == 0) out[MID * K * 9 + ch] = gb;
  }
}

struct WsLayout {
  size_t stats, part1, part2, gu, scale, shift, total;
};
WsLayout ws_layout(int N, int h, int w, int K) {
  const int tiles = N * cdiv(2 * w, T2) * cdiv(2 * h, T2);
  WsLayout L;
  size_t off = 0;
  auto take = [&](size_t floats) {
    size_t o = off;
    off += (floats + 63) / 64 * 64;
    return o;
  };
  L.stats = take((size_t)tiles * (2 * MID + 1));
  L.part1 = take((size_t)tiles * ((K + 2) * MID + K));
  L.part2 = take((size_t)tiles * (MID * K * 9 + MID));
  L.gu = take((size_t)N * 4 * h * w * K);
  L.scale = take(MID);
  L.shift = take(MID);
  L.total = off * sizeof(float);
  return L;
}

}  // namespace

extern "C" int eunet_bn_finalize(const float*, int, int, const float*, const float*, float, float, float*, float*,
                                 float*, float*, float*, float*, void*);
extern "C" int eunet_bn_eval_affine(int, const float*, const float*, const float*, const float*, float, float*,
                                    float*, void*);
int eunet_colsum_ld(const float* part, int rows, int cols, int ld, float* out, hipStream_t s);
extern "C" int eunet_upsample_bwd(const eunet_act* ghi, const eunet_act* glo, void* stream);

extern "C" {

int eunet_head_workspace_bytes(int n, int h, int w, int k, size_t* bytes) {
  EUNET_REQUIRE(bytes && n > 0 && h > 0 && w > 0 && k >= 1 && k <= 3, "head_workspace_bytes: bad args");
  *bytes = ws_layout(n, h, w, k).total;
  return EUNET_OK;
}

int eunet_head_fwd(const float* z, int n, int h, int w, int k, const float* w1, const float* b1, const float* gamma,
                   const float* beta, const float* w2, const float* b2, int training, float eps, float momentum,
                   float* run_mean, float* run_var, float* mean, float* invstd, float* out2h, float* logits,
                   void* ws, void* stream) {
  EUNET_REQUIRE(z && w1 && b1 && gamma && beta && w2 && b2 && ws && k >= 1 && k <= 3, "head_fwd: bad args");
  EUNET_REQUIRE(out2h || logits, "head_fwd: nothing to write");
  EUNET_REQUIRE(!training || (mean && invstd), "head_fwd: training needs mean/invstd outputs");
  const WsLayout L = ws_layout(n, h, w, k);
  float* wsf = (float*)ws;
  HeadArgs a = {};
  a.z = z; a.N = n; a.h = h; a.w = w; a.K = k;
  a.w1 = w1; a.b1 = b1; a.gamma = gamma; a.beta = beta; a.w2 = w2; a.b2 = b2;
  a.tx = cdiv(2 * w, T2); a.ty = cdiv(2 * h, T2); a.ntiles = n * a.tx * a.ty;
  a.stats = wsf + L.stats; a.out2h = out2h; a.logits = logits;
  a.scale = wsf + L.scale; a.shift = wsf + L.shift;
  hipStream_t s = (hipStream_t)stream;
  if (training) {
    if (k == 1) head_stats_kernel<1><<<a.ntiles, NT, 0, s>>>(a);
    else if (k == 2) head_stats_kernel<2><<<a.ntiles, NT, 0, s>>>(a);
    else head_stats_kernel<3><<<a.ntiles, NT, 0, s>>>(a);
    EUNET_LAUNCH_CHECK("head_stats");
    int rc = eunet_bn_finalize(a.stats, a.ntiles, MID, gamma, beta, eps, momentum, run_mean, run_var, mean, invstd,
                               wsf + L.scale, wsf + L.shift, stream);
    if (rc) return rc;
  } else {
    EUNET_REQUIRE(run_mean && run_var, "head_fwd: eval needs running stats");
    int rc = eunet_bn_eval_affine(MID, gamma, beta, run_mean, run_var, eps, wsf + L.scale, wsf + L.shift, stream);
    if (rc) return rc;
  }
  if (k == 1) head_out_kernel<1><<<a.ntiles, NT, 0, s>>>(a);
  else if (k == 2) head_out_kernel<2><<<a.ntiles, NT, 0, s>>>(a);
  else head_out_kernel<3><<<a.ntiles, NT, 0, s>>>(a);
  EUNET_LAUNCH_CHECK("head_out");
  return EUNET_OK;
}

int eunet_head_bwd(const float* z, int n, int h, int w, int k, const float* w1, const float* b1, const float* gamma,
                   const float* beta, const float* w2, const float* mean, const float* invstd, const float* g_logits,
                   const float* g_out2h, float* gz, float* gw1, float* gb1, float* ggamma, float* gbeta, float* gw2,
                   float* gb2, void* ws, void* stream) {
  EUNET_REQUIRE(z && w1 && b1 && gamma && beta && w2 && mean && invstd && gz && gw1 && gb1 && ggamma && gbeta &&
                    gw2 && gb2 && ws && k >= 1 && k <= 3,
                "head_bwd: bad args");
  EUNET_REQUIRE((g_logits != nullptr) != (g_out2h != nullptr), "head_bwd: exactly one of g_logits/g_out2h");
  const WsLayout L = ws_layout(n, h, w, k);
  float* wsf = (float*)ws;
  HeadArgs a = {};
  a.z = z; a.N = n; a.h = h; a.w = w; a.K = k;
  a.w1 = w1; a.b1 = b1; a.gamma = gamma; a.beta = beta; a.w2 = w2;
  a.mean = mean; a.istd = invstd; a.glog = g_logits; a.gout2h = g_out2h;
  a.tx = cdiv(2 * w, T2); a.ty = cdiv(2 * h, T2); a.ntiles = n * a.tx * a.ty;
  hipStream_t s = (hipStream_t)stream;
  a.part = wsf + L.part1;
  if (k == 1) head_bwd1_kernel<1><<<a.ntiles, NT, 0, s>>>(a);
  else if (k == 2) head_bwd1_kernel<2><<<a.ntiles, NT, 0, s>>>(a);
  else head_bwd1_kernel<3><<<a.ntiles, NT, 0, s>>>(a);
  EUNET_LAUNCH_CHECK("head_bwd1");
  const int ld1 = (k + 2) * MID + k;
  int rc;
  if ((rc = eunet_colsum_ld(a.part, a.ntiles, k * MID, ld1, gw2, s))) return rc;
  if ((rc = eunet_colsum_ld(a.part + k * MID, a.ntiles, MID, ld1, gbeta, s))) return rc;
  if ((rc = eunet_colsum_ld(a.part + (k + 1) * MID, a.ntiles, MID, ld1, ggamma, s))) return rc;
  if ((rc = eunet_colsum_ld(a.part + (k + 2) * MID, a.ntiles, k, ld1, gb2, s))) return rc;
  a.dbeta = gbeta; a.dgamma = ggamma;
  a.part = wsf + L.part2;
  a.gu = wsf + L.gu;
  const size_t lds = (324 * 65 + 400 * 3 + MID * k * 9 + MID + 6 * MID + k * MID) * sizeof(float);
  allow_lds(head_bwd2_kernel<1>, lds);
  allow_lds(head_bwd2_kernel<2>, lds);
  allow_lds(head_bwd2_kernel<3>, lds);
  if (k == 1) head_bwd2_kernel<1><<<a.ntiles, NT, lds, s>>>(a);
  else if (k == 2) head_bwd2_kernel<2><<<a.ntiles, NT, lds, s>>>(a);
  else head_bwd2_kernel<3><<<a.ntiles, NT, lds, s>>>(a);
  EUNET_LAUNCH_CHECK("head_bwd2");
  const int ld2 = MID * k * 9 + MID;
  if ((rc = eunet_colsum_ld(a.part, a.ntiles, MID * k * 9, ld2, gw1, s))) return rc;
  if ((rc = eunet_colsum_ld(a.part + MID * k * 9, a.ntiles, MID, ld2, gb1, s))) return rc;
  eunet_act ghi = {a.gu, n, 2 * h, 2 * w, k, k, 0, EUNET_F32};
  eunet_act glo = {gz, n, h, w, k, k, 0, EUNET_F32};
  return eunet_upsample_bwd(&ghi, &glo, stream);
}

}  // extern "C"
