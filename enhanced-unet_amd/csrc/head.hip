// The 2x-resolution tail of EnhancedUNet (fallback), fused and recomputed.
//
// Reference: models.py:236 (d1 = dec1(upsample(d2))), 308-313 + 336-337
// (out = d1 + enhance(d1), enhance = Conv3x3(K->64)+BN+ReLU+Conv1x1(64->K)),
// train_eval.py:306-310 (bilinear 2H->H resize, == exact 2x2 mean).
//
// dec1 commutes with the upsample, so the host passes z = dec1(d2) at H
// (K channels).  u = up(z), the 64-channel conv output h, BN, ReLU, the 1x1,
// the residual and the 2x2 mean are recomputed per 16x16 tile (at 2H) from z;
// the 64-channel forward tensors at 2H are never stored.
// Kernels (persistent grids of <= 1024 blocks; one partial row per block):
//   fwd : stats (Chan-combined per-block BN partials) -> bn_finalize -> out
//   bwd : bwd1  -> gW2, gb2, dbeta, dgamma (BN backward sums)
//         gh    -> g_h (dtype T, stored once) and the per-tap products
//                  v[p][k][t] = sum_c W1[c][k][t] g_h[p][c]
//         gu    -> g_u[q] = g_o[q] + sum_t v[q - d_t][t]   (conv3x3 dgrad as a stencil)
//         wgrad -> gW1, gb1 via MFMA (K = pixels; im2col of u built in LDS)
//         upsample adjoint g_u -> g_z.
#include "common.h"

EUNET_DEBUG_UNIT(head)

namespace {
constexpr int NT = 256;
constexpr int T2 = 16;  // tile side at 2H
constexpr int MID = 64;
constexpr int HEAD_BLOCKS = 768;  // persistent grid: 3 resident blocks x 256 CUs (no second round)
constexpr int HEAD_BLOCKS4 = 1024;  // the bf16 stats / out kernels: 4 resident blocks per CU

struct HeadArgs {
  const float* z; int N, h, w, K;
  const float* w1; const float* b1;
  const float* gamma; const float* beta; const float* w2; const float* b2;
  const float* mean; const float* istd;    // bwd
  const float* scale; const float* shift;  // fwd out
  const float* glog; const float* gout2h;
  const float* dbeta; const float* dgamma;  // bwd gh
  float* stats; float* out2h; float* logits; float* part;
  void* gh; float* v; float* gu;
  float* patch;  // bf16 path: per-tile low-res adjoint patches [tile][10][10][K] (head_gh_mfma_kernel)
  float* gram;   // bf16 path: per-block im2col second-moment rows [block][GRAM_LD] (head_gram_mfma_kernel)
  int tx, ty, ntiles;
};

// u = up(z) at one point from its four z taps (rows y0 / y1, columns x0 / x1) as one explicit fmaf sequence, the
// same in every head kernel: the forward and the recomputing backward kernels get bit-equal u whatever
// contraction the compiler would choose for the expression in each of them
__device__ __forceinline__ float up_lerp(float ly, float lx, float v00, float v01, float v10, float v11) {
  const float r0 = fmaf(lx, v01, (1.f - lx) * v00);
  const float r1 = fmaf(lx, v11, (1.f - lx) * v10);
  return fmaf(ly, r1, (1.f - ly) * r0);
}

__device__ __forceinline__ float up_val(const HeadArgs& a, int n, int oy, int ox, int k) {
  int y0, y1, x0, x1;
  float ly, lx;
  up2_src(oy, a.h, y0, y1, ly);
  up2_src(ox, a.w, x0, x1, lx);
  const float* zb = a.z + (long long)n * a.h * a.w * a.K;
  const float v00 = zb[((long long)y0 * a.w + x0) * a.K + k], v01 = zb[((long long)y0 * a.w + x1) * a.K + k];
  const float v10 = zb[((long long)y1 * a.w + x0) * a.K + k], v11 = zb[((long long)y1 * a.w + x1) * a.K + k];
  return up_lerp(ly, lx, v00, v01, v10, v11);
}

// su[(18 x 18) region starting at (oy0-1, ox0-1)][3], zero outside the image
__device__ void fill_u(const HeadArgs& a, float* su, int n, int oy0, int ox0) {
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  for (int i = threadIdx.x; i < 18 * 18; i += NT) {
    const int hy = i / 18, hx = i - hy * 18;
    const int oy = oy0 + hy - 1, ox = ox0 + hx - 1;
    const bool in = oy >= 0 && oy < H2 && ox >= 0 && ox < W2;
    for (int k = 0; k < a.K; ++k) su[i * 3 + k] = in ? up_val(a, n, oy, ox, k) : 0.f;
  }
}


__device__ __forceinline__ void tile_coords(const HeadArgs& a, int tile, int& n, int& oy0, int& ox0) {
  const int tpi = a.tx * a.ty;
  n = tile / tpi;
  const int r = tile - n * tpi;
  oy0 = (r / a.tx) * T2;
  ox0 = (r % a.tx) * T2;
}

// The z region a 16x16 tile at 2H interpolates from: 10 x 10 pixels x K (<= 3) at H, edge-
// clamped.  Each thread holds <= 2 of its values; the next tile's are loaded into registers
// while the current tile computes, so fill_u no longer waits on global memory.
constexpr int ZR = 10;
template <int K>
__device__ __forceinline__ void zload(const HeadArgs& a, int tile, float (&zv)[2]) {
  if (tile >= a.ntiles) return;
  int n, oy0, ox0;
  tile_coords(a, tile, n, oy0, ox0);
  const int zy0 = oy0 / 2 - 1, zx0 = ox0 / 2 - 1;
  const float* zb = a.z + (long long)n * a.h * a.w * K;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + j * NT;
    if (idx < ZR * ZR * K) {
      const int k = idx % K, pix = idx / K, i = pix / ZR, c = pix - i * ZR;
      const int yy = min(max(zy0 + i, 0), a.h - 1), xx = min(max(zx0 + c, 0), a.w - 1);
      zv[j] = zb[((long long)yy * a.w + xx) * K + k];
    }
  }
}

// stage the prefetched z region, prefetch the next tile's, then u = up(z) over the 18x18 halo
// from LDS (as fill_u; the caller syncs before and after)
template <int K>
__device__ void stage_u(const HeadArgs& a, float* su, float* zs, float (&zv)[2], int tile, int oy0, int ox0) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + j * NT;
    if (idx < ZR * ZR * K) zs[idx] = zv[j];
  }
  __syncthreads();
  zload<K>(a, tile + gridDim.x, zv);
  const int H2 = 2 * a.h, W2 = 2 * a.w, zy0 = oy0 / 2 - 1, zx0 = ox0 / 2 - 1;
  for (int i = threadIdx.x; i < 18 * 18; i += NT) {
    const int hy = i / 18, hx = i - hy * 18;
    const int oy = oy0 + hy - 1, ox = ox0 + hx - 1;
    const bool in = oy >= 0 && oy < H2 && ox >= 0 && ox < W2;
    int y0, y1, x0, x1;
    float ly, lx;
    up2_src_i(in ? oy : 0, a.h, y0, y1, ly);
    up2_src_i(in ? ox : 0, a.w, x0, x1, lx);
    const float* r0 = zs + ((y0 - zy0) * ZR) * K;
    const float* r1 = zs + ((y1 - zy0) * ZR) * K;
    const int c0 = (x0 - zx0) * K, c1 = (x1 - zx0) * K;
#pragma unroll
    for (int k = 0; k < K; ++k)
      su[i * 3 + k] = in ? up_lerp(ly, lx, r0[c0 + k], r0[c1 + k], r1[c0 + k], r1[c1 + k]) : 0.f;
  }
}

__device__ __forceinline__ float g_out(const HeadArgs& a, int K, int n, int k, int oy, int ox) {
  if (a.glog) return 0.25f * a.glog[(((long long)n * K + k) * a.h + (oy >> 1)) * a.w + (ox >> 1)];
  return a.gout2h[(((long long)n * K + k) * (2 * a.h) + oy) * (2 * a.w) + ox];
}
// the same without the 2x2-mean factor (g_scale): a prefetching caller's bounds-checked load then
// has no dependent instruction in its branch, so it does not wait there for the load
__device__ __forceinline__ float g_raw(const HeadArgs& a, int K, int n, int k, int oy, int ox) {
  if (a.glog) return a.glog[(((long long)n * K + k) * a.h + (oy >> 1)) * a.w + (ox >> 1)];
  return a.gout2h[(((long long)n * K + k) * (2 * a.h) + oy) * (2 * a.w) + ox];
}
__device__ __forceinline__ float g_scale(const HeadArgs& a) { return a.glog ? 0.25f : 1.f; }

// Thread mapping: 8 lanes per pixel, lane group g = lane & 7 owns channels 8g..8g+7;
// a 256-thread block covers 32 pixels per pass, 8 passes per 16x16 tile.
// Quad order (pixel slots 4q..4q+3 = one 2x2 quad) so the 2x2 mean is a
// lane reduction (xor 8, 16).
__device__ __forceinline__ void pass_pixel(int pass, int tid, int& r, int& c) {
  const int ps = tid >> 3;  // pixel slot 0..31
  const int q = pass * 8 + (ps >> 2), sub = ps & 3;
  r = 2 * (q >> 3) + (sub >> 1);
  c = 2 * (q & 7) + (sub & 1);
}

// W1 transposed in LDS: w1t[j][64], j = k*9 + t; b1s[64]
template <int K>
__device__ __forceinline__ void load_w1t(const HeadArgs& a, float* w1t, float* b1s) {
  for (int i = threadIdx.x; i < MID * K * 9; i += NT) {
    const int c = i / (K * 9), j = i - c * (K * 9);
    w1t[j * MID + c] = a.w1[i];
  }
  if (threadIdx.x < MID) b1s[threadIdx.x] = a.b1[threadIdx.x];
}

// h[e] = conv3x3(u) for channels 8g+e of the pixel whose 3x3 window starts at su (r, c)
template <int K>
__device__ __forceinline__ void conv_h8(const float* su, const float* w1t, const float* b1s, int r, int c, int g,
                                        float (&h)[8]) {
  const float4 b0 = *(const float4*)(b1s + 8 * g), b1 = *(const float4*)(b1s + 8 * g + 4);
  h[0] = b0.x; h[1] = b0.y; h[2] = b0.z; h[3] = b0.w; h[4] = b1.x; h[5] = b1.y; h[6] = b1.z; h[7] = b1.w;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - ky * 3;
      const float u = su[((r + ky) * 18 + c + kx) * 3 + k];
      const float4 w0 = *(const float4*)(w1t + (k * 9 + t) * MID + 8 * g);
      const float4 w1 = *(const float4*)(w1t + (k * 9 + t) * MID + 8 * g + 4);
      h[0] = fmaf(w0.x, u, h[0]); h[1] = fmaf(w0.y, u, h[1]); h[2] = fmaf(w0.z, u, h[2]); h[3] = fmaf(w0.w, u, h[3]);
      h[4] = fmaf(w1.x, u, h[4]); h[5] = fmaf(w1.y, u, h[5]); h[6] = fmaf(w1.z, u, h[6]); h[7] = fmaf(w1.w, u, h[7]);
    }
}

__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// sum over the 8 pixel slots of a wave (lanes with equal g)
__device__ __forceinline__ float sum_pixels(float v) {
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
// sum over the 8 channel groups of one pixel
__device__ __forceinline__ float sum_groups(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

// ---------------------------------------------------------------------------
// forward statistics: per-thread Welford over its pixels (8 channels), Chan
// combine across lanes / waves, one (sum, M2, count) row per block
// ---------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(NT) void head_stats_kernel(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float w1t[K * 9 * MID];
  __shared__ __attribute__((aligned(16))) float b1s[MID];
  __shared__ float su[18 * 18 * 3];
  __shared__ float wn_s[4], wm_s[4][MID], wq_s[4][MID];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane & 7;
  load_w1t<K>(a, w1t, b1s);
  float n = 0.f, mean[8], m2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { mean[e] = 0.f; m2[e] = 0.f; }
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int nn, oy0, ox0;
    tile_coords(a, tile, nn, oy0, ox0);
    __syncthreads();
    fill_u(a, su, nn, oy0, ox0);
    __syncthreads();
    for (int pass = 0; pass < 8; ++pass) {
      int r, c;
      pass_pixel(pass, tid, r, c);
      if (oy0 + r >= 2 * a.h || ox0 + c >= 2 * a.w) continue;
      float h[8];
      conv_h8<K>(su, w1t, b1s, r, c, g, h);
      n += 1.f;
      const float inv = 1.f / n;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = h[e] - mean[e];
        mean[e] = fmaf(d, inv, mean[e]);
        m2[e] = fmaf(d, h[e] - mean[e], m2[e]);
      }
    }
  }
#pragma unroll
  for (int off = 8; off <= 32; off <<= 1) {
    const float nb = __shfl_xor(n, off, 64);
    const float nt = n + nb;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float mb = __shfl_xor(mean[e], off, 64), qb = __shfl_xor(m2[e], off, 64);
      const float d = mb - mean[e];
      if (nt > 0.f) {
        mean[e] += d * nb / nt;
        m2[e] += qb + d * d * n * nb / nt;
      }
    }
    n = nt;
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      wm_s[wv][8 * g + e] = mean[e];
      wq_s[wv][8 * g + e] = m2[e];
    }
    if (lane == 0) wn_s[wv] = n;
  }
  __syncthreads();
  if (tid < MID) {
    double bn = 0.0, bm = 0.0, bq = 0.0;
    for (int w = 0; w < 4; ++w) {
      const double nb = wn_s[w];
      if (nb <= 0.0) continue;
      const double d = (double)wm_s[w][tid] - bm, nt = bn + nb;
      bm += d * nb / nt;
      bq += (double)wq_s[w][tid] + d * d * bn * nb / nt;
      bn = nt;
    }
    a.stats[((long long)blockIdx.x * 2 + 0) * MID + tid] = (float)(bm * bn);
    a.stats[((long long)blockIdx.x * 2 + 1) * MID + tid] = (float)bq;
    if (tid == 0) a.stats[(long long)2 * MID * gridDim.x + blockIdx.x] = (float)bn;
  }
}

template <int K>
__global__ __launch_bounds__(NT) void head_out_kernel(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float w1t[K * 9 * MID];
  __shared__ __attribute__((aligned(16))) float b1s[MID], sc[MID], sh[MID], w2s[K * MID];
  __shared__ float su[18 * 18 * 3];
  const int tid = threadIdx.x, lane = tid & 63, g = lane & 7;
  load_w1t<K>(a, w1t, b1s);
  for (int i = tid; i < K * MID; i += NT) w2s[i] = a.w2[i];
  if (tid < MID) {
    sc[tid] = a.scale[tid];
    sh[tid] = a.shift[tid];
  }
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int n, oy0, ox0;
    tile_coords(a, tile, n, oy0, ox0);
    __syncthreads();
    fill_u(a, su, n, oy0, ox0);
    __syncthreads();
    for (int pass = 0; pass < 8; ++pass) {
      int r, c;
      pass_pixel(pass, tid, r, c);
      const int oy = oy0 + r, ox = ox0 + c;
      const bool pv = oy < H2 && ox < W2;
      float h[8], s8[8], t8[8];
      conv_h8<K>(su, w1t, b1s, r, c, g, h);
      load8(sc + 8 * g, s8);
      load8(sh + 8 * g, t8);
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = fmaxf(fmaf(h[e], s8[e], t8[e]), 0.f);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float w8[8];
        load8(w2s + k * MID + 8 * g, w8);
        float o = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) o = fmaf(w8[e], h[e], o);
        o = sum_groups(o);
        const float val = su[((r + 1) * 18 + c + 1) * 3 + k] + a.b2[k] + o;
        if (pv && g == 0 && a.out2h) a.out2h[(((long long)n * K + k) * H2 + oy) * W2 + ox] = val;
        float q = val + __shfl_xor(val, 8, 64);
        q += __shfl_xor(q, 16, 64);
        if (pv && g == 0 && ((lane >> 3) & 3) == 0 && a.logits)
          a.logits[(((long long)n * K + k) * a.h + (oy >> 1)) * a.w + (ox >> 1)] = 0.25f * q;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward pass 1: gW2, gb2, dbeta = sum g_bn, dgamma = sum g_bn * xhat
// (per-thread register accumulators over the block's pixels)
// ---------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(NT) void head_bwd1_kernel(HeadArgs a) {
  constexpr int STRIDE = (K + 2) * MID + K;
  __shared__ __attribute__((aligned(16))) float w1t[K * 9 * MID];
  __shared__ __attribute__((aligned(16))) float b1s[MID], ga[MID], be[MID], mu[MID], is[MID], w2s[K * MID];
  __shared__ float su[18 * 18 * 3];
  __shared__ float red[4][STRIDE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane & 7;
  load_w1t<K>(a, w1t, b1s);
  for (int i = tid; i < K * MID; i += NT) w2s[i] = a.w2[i];
  if (tid < MID) {
    ga[tid] = a.gamma[tid];
    be[tid] = a.beta[tid];
    mu[tid] = a.mean[tid];
    is[tid] = a.istd[tid];
  }
  float aw2[K][8], agb[8], agx[8], ab2[K];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    agb[e] = 0.f;
    agx[e] = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) aw2[k][e] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) ab2[k] = 0.f;
  __syncthreads();
  float ga8[8], be8[8], mu8[8], is8[8];
  load8(ga + 8 * g, ga8);
  load8(be + 8 * g, be8);
  load8(mu + 8 * g, mu8);
  load8(is + 8 * g, is8);
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int n, oy0, ox0;
    tile_coords(a, tile, n, oy0, ox0);
    __syncthreads();
    fill_u(a, su, n, oy0, ox0);
    __syncthreads();
    for (int pass = 0; pass < 8; ++pass) {
      int r, c;
      pass_pixel(pass, tid, r, c);
      const int oy = oy0 + r, ox = ox0 + c;
      if (oy >= 2 * a.h || ox >= 2 * a.w) continue;
      float h[8];
      conv_h8<K>(su, w1t, b1s, r, c, g, h);
      float go[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        go[k] = g_out(a, K, n, k, oy, ox);
        ab2[k] += (g == 0) ? go[k] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (h[e] - mu8[e]) * is8[e];
        const float pre = fmaf(ga8[e], xh, be8[e]);
        const float act = fmaxf(pre, 0.f);
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          aw2[k][e] = fmaf(go[k], act, aw2[k][e]);
          s = fmaf(w2s[k * MID + 8 * g + e], go[k], s);
        }
        const float gbn = pre > 0.f ? s : 0.f;
        agb[e] += gbn;
        agx[e] = fmaf(gbn, xh, agx[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    agb[e] = sum_pixels(agb[e]);
    agx[e] = sum_pixels(agx[e]);
#pragma unroll
    for (int k = 0; k < K; ++k) aw2[k][e] = sum_pixels(aw2[k][e]);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) ab2[k] = sum_pixels(ab2[k]);
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int k = 0; k < K; ++k) red[wv][k * MID + 8 * g + e] = aw2[k][e];
      red[wv][K * MID + 8 * g + e] = agb[e];
      red[wv][(K + 1) * MID + 8 * g + e] = agx[e];
    }
    if (g == 0)
#pragma unroll
      for (int k = 0; k < K; ++k) red[wv][(K + 2) * MID + k] = ab2[k];
  }
  __syncthreads();
  for (int i = tid; i < STRIDE; i += NT)
    a.part[(long long)blockIdx.x * STRIDE + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

// ---------------------------------------------------------------------------
// backward: g_h (stored, dtype T) and the per-tap products v[p][k*9+t]
// ---------------------------------------------------------------------------
template <int K, typename T>
__global__ __launch_bounds__(NT) void head_bwd_gh_kernel(HeadArgs a) {
  constexpr int GLD = MID + 4;  // padded row of the per-pass g_h staging tile
  __shared__ __attribute__((aligned(16))) float w1t[K * 9 * MID];
  __shared__ __attribute__((aligned(16))) float b1s[MID], ga[MID], be[MID], mu[MID], is[MID], c1[MID], c2[MID];
  __shared__ __attribute__((aligned(16))) float w2s[K * MID];
  __shared__ __attribute__((aligned(16))) float gls[32 * GLD];
  __shared__ float su[18 * 18 * 3];
  const int tid = threadIdx.x, lane = tid & 63, g = lane & 7, ps = tid >> 3;
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  const float inv_cnt = 1.f / ((float)a.N * (float)H2 * (float)W2);
  load_w1t<K>(a, w1t, b1s);
  for (int i = tid; i < K * MID; i += NT) w2s[i] = a.w2[i];
  if (tid < MID) {
    ga[tid] = a.gamma[tid];
    be[tid] = a.beta[tid];
    mu[tid] = a.mean[tid];
    is[tid] = a.istd[tid];
    c1[tid] = a.dbeta[tid] * inv_cnt;
    c2[tid] = a.dgamma[tid] * inv_cnt;
  }
  __syncthreads();
  float ga8[8], be8[8], mu8[8], is8[8], c18[8], c28[8];
  load8(ga + 8 * g, ga8);
  load8(be + 8 * g, be8);
  load8(mu + 8 * g, mu8);
  load8(is + 8 * g, is8);
  load8(c1 + 8 * g, c18);
  load8(c2 + 8 * g, c28);
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int n, oy0, ox0;
    tile_coords(a, tile, n, oy0, ox0);
    __syncthreads();
    fill_u(a, su, n, oy0, ox0);
    __syncthreads();
    for (int pass = 0; pass < 8; ++pass) {
      int r, c;
      pass_pixel(pass, tid, r, c);
      const int oy = oy0 + r, ox = ox0 + c;
      const bool pv = oy < H2 && ox < W2;
      float h[8];
      conv_h8<K>(su, w1t, b1s, r, c, g, h);
      float go[K];
#pragma unroll
      for (int k = 0; k < K; ++k) go[k] = pv ? g_out(a, K, n, k, oy, ox) : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (h[e] - mu8[e]) * is8[e];
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) s = fmaf(w2s[k * MID + 8 * g + e], go[k], s);
        const float gbn = (fmaf(ga8[e], xh, be8[e]) > 0.f) ? s : 0.f;
        h[e] = ga8[e] * is8[e] * (gbn - c18[e] - xh * c28[e]);  // g_h
      }
      const long long p = ((long long)n * H2 + oy) * W2 + ox;
      if (pv) {
        T* ghp = (T*)a.gh + p * MID + 8 * g;
        *(uint4*)ghp = Vec16<T>::pack(h);
        if constexpr (sizeof(T) == 4) *(uint4*)(ghp + 4) = Vec16<T>::pack(h + 4);
      }
      *(float4*)(gls + ps * GLD + 8 * g) = make_float4(h[0], h[1], h[2], h[3]);
      *(float4*)(gls + ps * GLD + 8 * g + 4) = make_float4(h[4], h[5], h[6], h[7]);
      __syncthreads();
      // per-tap products v[j] = sum_c W1[c][j] g_h[c], lane g takes j = 4g..4g+3
      float vj[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int c4 = 0; c4 < MID; c4 += 4) {
        const float4 gv = *(const float4*)(gls + ps * GLD + c4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int j = 4 * g + i;
          if (j < K * 9) {
            const float4 wv = *(const float4*)(w1t + j * MID + c4);
            vj[i] = fmaf(wv.x, gv.x, fmaf(wv.y, gv.y, fmaf(wv.z, gv.z, fmaf(wv.w, gv.w, vj[i]))));
          }
        }
      }
      if (pv) {  // planar v[j][pixel] (coalesced gather in head_bwd_gu_kernel)
        const long long P2 = (long long)a.N * 4 * a.h * a.w;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (4 * g + i < K * 9) a.v[(long long)(4 * g + i) * P2 + p] = vj[i];
      }
      __syncthreads();
    }
  }
}

// g_u[q][k] = g_o[q][k] + sum_t v[q - d_t][k*9+t]   (d_t = (ky-1, kx-1)); v fp32 or bf16
template <int K, typename TV>
__global__ void head_bwd_gu_kernel(HeadArgs a) {
  const TV* vp = (const TV*)a.v;
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long long)a.N * H2 * W2) return;
  const int ox = (int)(id % W2);
  const int oy = (int)((id / W2) % H2);
  const int n = (int)(id / ((long long)W2 * H2));
  float acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = g_out(a, K, n, k, oy, ox);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ky = t / 3, kx = t - ky * 3;
    const int py = oy - ky + 1, px = ox - kx + 1;
    if (py < 0 || py >= H2 || px < 0 || px >= W2) continue;
    const long long P2 = (long long)a.N * H2 * W2, pix = ((long long)n * H2 + py) * W2 + px;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] += Elem<TV>::ld(vp + (long long)(k * 9 + t) * P2 + pix);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) a.gu[id * K + k] = acc[k];
}

// ---------------------------------------------------------------------------
// gW1[c][k][t] = sum_p g_h[p][c] u[p + d_t][k],  gb1[c] = sum_p g_h[p][c]
// MFMA with the pixels as the reduction dimension; im2col(u) [256 px][32] in LDS
// ---------------------------------------------------------------------------
template <int K, typename T>
__global__ __launch_bounds__(NT) void head_wgrad_kernel(HeadArgs a) {
  constexpr int E = Vec16<T>::N;
  constexpr int STRIDE = MID * K * 9 + MID;
  __shared__ __attribute__((aligned(16))) T gs[T2 * T2 * MID];  // g_h tile [256 px][64]
  __shared__ __attribute__((aligned(16))) T cs[T2 * T2 * 32];   // im2col [256 px][32]
  __shared__ float su[18 * 18 * 3];
  __shared__ float dbs[4][MID];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  f32x4 acc[2];
  acc[0] = (f32x4){0.f, 0.f, 0.f, 0.f};
  acc[1] = acc[0];
  float dbacc = 0.f;
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int n, oy0, ox0;
    tile_coords(a, tile, n, oy0, ox0);
    __syncthreads();
    fill_u(a, su, n, oy0, ox0);
    for (int id = tid; id < T2 * T2 * MID / E; id += NT) {  // stage g_h (zero outside the image)
      const int px = id / (MID / E), u = id - px * (MID / E);
      const int oy = oy0 + px / T2, ox = ox0 + px % T2;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (oy < H2 && ox < W2)
        val = *(const uint4*)((const T*)a.gh + (((long long)n * H2 + oy) * W2 + ox) * MID + u * E);
      *(uint4*)(gs + px * MID + u * E) = val;
    }
    __syncthreads();
    for (int id = tid; id < T2 * T2 * 32; id += NT) {  // im2col of u
      const int px = id >> 5, j = id & 31;
      float val = 0.f;
      if (j < K * 9) {
        const int k = j / 9, t = j - k * 9;
        const int ky = t / 3, kx = t - ky * 3;
        val = su[((px / T2 + ky) * 18 + (px % T2) + kx) * 3 + k];
      }
      Elem<T>::st(cs + id, val);
    }
    __syncthreads();
    for (int px = wv; px < T2 * T2; px += 4) dbacc += Elem<T>::ld(gs + px * MID + lane);
    const int cw = wv * 16;
    if constexpr (sizeof(T) == 2) {
      const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
#pragma unroll 2
      for (int ks = 0; ks < T2 * T2 / 32; ++ks) {
        const int pxa = ks * 32 + 8 * g + q4;
        const s16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, (char*)gs + (pxa * MID + cw + 4 * p4) * 2));
        const s16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, (char*)gs + ((pxa + 4) * MID + cw + 4 * p4) * 2));
        const bf16x8 af = cat_bf16x4(alo, ahi);
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
          const s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              LDS_PTR(s16x4, (char*)cs + (pxa * 32 + jt * 16 + 4 * p4) * 2));
          const s16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              LDS_PTR(s16x4, (char*)cs + ((pxa + 4) * 32 + jt * 16 + 4 * p4) * 2));
          acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, cat_bf16x4(blo, bhi), acc[jt], 0, 0, 0);
        }
      }
    } else {
      const int kq = lane >> 4, i = lane & 15;
#pragma unroll 4
      for (int ks = 0; ks < T2 * T2 / 4; ++ks) {
        const int px = ks * 4 + kq;
        const float av = ((const float*)gs)[px * MID + cw + i];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
          acc[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, ((const float*)cs)[px * 32 + jt * 16 + i], acc[jt],
                                                          0, 0, 0);
      }
    }
  }
  float* out = a.part + (long long)blockIdx.x * STRIDE;
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = wv * 16 + g * 4 + e, j = jt * 16 + li;
      if (j < K * 9) out[c * K * 9 + j] = acc[jt][e];
    }
  __syncthreads();
  dbs[wv][lane] = dbacc;
  __syncthreads();
  if (tid < MID) out[MID * K * 9 + tid] = dbs[0][tid] + dbs[1][tid] + dbs[2][tid] + dbs[3][tid];
}

// ===========================================================================
// bf16 MFMA head (dtype EUNET_BF16; the reference's autocast runs these convs in
// bf16).  Per 16-pixel row segment the 64-channel conv is one GEMM,
//   h^T[c][px] = W1[c][j] * im2col^T[j][px]    (v_mfma_f32_16x16x32_bf16,
//   4 channel blocks, j = k*9+t zero-padded to 32),
// leaving lane l with channels c = 16cb + 4q + i (q = l>>4, i = 0..3) of pixel
// x = l&15.  Those 16 values, converted to bf16 in the order (cb = 2ch, i),
// (cb = 2ch+1, i), ARE the B operand of the next GEMM over channels when its A
// operand is loaded with the same channel permutation (perm_c) -- the 1x1 conv,
// the per-tap products v and the backward g_a all chain without transposes.
// Wave w of a 256-thread block owns rows 4w..4w+3 of the 16x16 tile.
// ===========================================================================
__device__ __forceinline__ int perm_c(int q, int ch, int jj) { return 16 * (2 * ch + (jj >> 2)) + 4 * q + (jj & 3); }

// C-layout values v[cb][i] -> B fragment over channel chunk ch
__device__ __forceinline__ bf16x8 cfrag(const f32x4 (&v)[4], int ch) {
  bf16x8 b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    b[i] = (__bf16)v[2 * ch][i];
    b[4 + i] = (__bf16)v[2 * ch + 1][i];
  }
  return b;
}

// A operand of h^T: row c = 16cb + (l&15), k = j = 8q + jj
// Weight fragments are loaded once per block, all loads first at clamped (valid) indices, an empty asm
// on the values so the compiler cannot sink each load into the branch of its select (which made every
// load wait for the previous one: ~50 serialized L2 round trips in a block's prologue), then the selects.
template <int N>
__device__ __forceinline__ void keep_loads(float (&f)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}

template <int K>
__device__ __forceinline__ void load_a_w1(const float* w1, int lane, bf16x8 (&A)[4]) {
  const int r = lane & 15, q = lane >> 4;
  float f[32];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int j = 8 * q + jj;
      f[8 * cb + jj] = w1[(16 * cb + r) * K * 9 + (j < K * 9 ? j : 0)];
    }
  keep_loads(f);
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) A[cb][jj] = (__bf16)(8 * q + jj < K * 9 ? f[8 * cb + jj] : 0.f);
}

// per-lane su offsets of im2col^T[j = 8q + jj][px] relative to the pixel's window corner (su row stride RS).
// The padding entries j >= 9K read the window corner (offset 0) instead of a zero: every consumer's W1
// fragment (load_a_w1) is zero at those k, and the staged u is finite, so they add exact zeros -- the
// fragment is 8 reads and 4 v_cvt_pk_bf16_f32 with no per-entry select and repack.
template <int K, int RS = 18>
__device__ __forceinline__ void im2col_offsets(int q, int (&off)[8]) {
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int j = 8 * q + jj;
    if (j < K * 9) {
      const int k = j / 9, t = j - 9 * k, ky = t / 3, kx = t - 3 * ky;
      off[jj] = (ky * RS + kx) * 3 + k;
    } else {
      off[jj] = 0;
    }
  }
}

__device__ __forceinline__ bf16x8 im2col_frag(const float* su, int base, const int (&off)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = pk_bf16(su[base + off[2 * i]], su[base + off[2 * i + 1]]);
  return __builtin_bit_cast(bf16x8, (u32x4){w[0], w[1], w[2], w[3]});
}

// h^T (bias excluded) for the pixel row segment whose window corner is su[base]
__device__ __forceinline__ void conv_h_mfma(const float* su, int base, const int (&off)[8], const bf16x8 (&Ah)[4],
                                            f32x4 (&acc)[4]) {
  const bf16x8 b = im2col_frag(su, base, off);
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah[cb], b, z, 0, 0, 0);
}

// A operand of s^T[c][px] = sum_k W2[k][c] g_o[k][px]: row c = 16cb + (l&15), k = class 8q + jj
template <int K>
__device__ __forceinline__ void load_a_w2t(const float* w2, int lane, bf16x8 (&A)[4]) {
  const int r = lane & 15, q = lane >> 4;
  float f[32];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int kk = 8 * q + jj;
      f[8 * cb + jj] = w2[(kk < K ? kk : 0) * MID + 16 * cb + r];
    }
  keep_loads(f);
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) A[cb][jj] = (__bf16)(8 * q + jj < K ? f[8 * cb + jj] : 0.f);
}

template <int K>
__device__ __forceinline__ bf16x8 go_frag(int q, const float (&go)[K]) {
  bf16x8 b;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) b[jj] = (__bf16)0.f;
  if (q == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) b[k] = (__bf16)go[k];
  }
  return b;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ float f4(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
// packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two channels per instruction, each element
// rounded as the scalar op would round it)
__device__ __forceinline__ f32x4 ld4v(const float* p) { return *(const f32x4*)p; }
__device__ __forceinline__ f32x2 half2(const f32x4& v, int hp) { return hp ? v.hi : v.lo; }
__device__ __forceinline__ f32x2 pkfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
// per 16-bit half of a (halves >= 0): 1 where nonzero, else 0 (v_pk_min_u16; inline asm here and below: written
// in C the compiler turns the per-half ops into a compare and a select per half)
__device__ __forceinline__ uint32_t pk_nonzero_one(uint32_t a) {
  uint32_t m;  // (the 1 comes from a register: an inline constant would give the high half 0)
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(a), "s"(0x00010001u));
  return m;
}
// per 16-bit half: a * b mod 2^16 (v_pk_mul_lo_u16; with b in {0, 1} a select of a or 0)
__device__ __forceinline__ uint32_t pk_mul_u16(uint32_t a, uint32_t b) {
  uint32_t m;
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(m) : "v"(a), "v"(b));
  return m;
}
__device__ __forceinline__ uint32_t pk_mul_u16s(uint32_t a, uint32_t b) {  // b wave-uniform (an SGPR)
  uint32_t m;
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(m) : "v"(a), "s"(b));
  return m;
}
__device__ __forceinline__ f32x2 relu_sel(f32x2 pre, f32x2 v) {  // v where pre > 0, else 0
  return (f32x2){pre.x > 0.f ? v.x : 0.f, pre.y > 0.f ? v.y : 0.f};
}

// sum over the 16 pixel lanes of a row (lanes with equal q)
__device__ __forceinline__ float sum_x16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

// Per lane shifted sums S1 = sum (h - s), S2 = sum (h - s)^2 over its pixels, with the shift s =
// the lane's first computed value (any finite shift is exact in real arithmetic; one near the
// mean keeps S2 - S1^2 / n free of cancellation), then (mean, M2) per lane and Chan's combine
// across lanes and waves.  Full tiles (every 2H tile of a multiple-of-16 image) take a branch-free
// path with two rows' MFMAs issued ahead of their VALU work; the count is kept per lane.
template <int K>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void head_stats_mfma_kernel(HeadArgs a) {
  __shared__ float su[18 * 18 * 3];
  __shared__ float zs[ZR * ZR * 3];
  __shared__ float wn_s[4], wm_s[4][MID], wq_s[4][MID];
  __shared__ __attribute__((aligned(16))) float shs[4][MID];  // per-wave shift of each channel
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4, x = lane & 15;
  bf16x8 Ah[4];
  load_a_w1<K>(a.w1, lane, Ah);
  int off[8];
  im2col_offsets<K>(q, off);
  float n = 0.f, s1[16], s2[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  const float* shw = shs[wv];
  bool first = true;
  float zv[2] = {0.f, 0.f};
  zload<K>(a, blockIdx.x, zv);
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int nn, oy0, ox0;
    tile_coords(a, tile, nn, oy0, ox0);
    __syncthreads();
    stage_u<K>(a, su, zs, zv, tile, oy0, ox0);
    __syncthreads();
    if (first) {  // the wave's shift per channel: its first row's pixel 0 (a zero-padded 0 at an edge)
      f32x4 acc[4];
      conv_h_mfma(su, ((4 * wv) * 18 + x) * 3, off, Ah, acc);
      if (x == 0)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) shs[wv][16 * cb + 4 * q + i] = acc[cb][i];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes (wave-private row)
      __builtin_amdgcn_wave_barrier();
      first = false;
    }
    const bool full = oy0 + T2 <= H2 && ox0 + T2 <= W2;  // uniform (every tile of a multiple-of-16 image)
#pragma unroll 1
    for (int rr = 0; rr < 4; ++rr) {
      const int r = 4 * wv + rr;
      f32x4 acc[4];
      conv_h_mfma(su, (r * 18 + x) * 3, off, Ah, acc);
      const float m = (full || (oy0 + r < H2 && ox0 + x < W2)) ? 1.f : 0.f;
      n += m;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const float4 s4 = ld4(shw + 16 * cb + 4 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = 4 * cb + i;
          const float d = (acc[cb][i] - f4(s4, i)) * m;
          s1[e] += d;
          s2[e] = fmaf(d, d, s2[e]);
        }
      }
    }
  }
  // the lanes of a row share the wave's shifts: their shifted sums add directly
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    s1[e] = sum_x16(s1[e]);
    s2[e] = sum_x16(s2[e]);
  }
  n = sum_x16(n);
  if (x == 0) {
    const float inv = n > 0.f ? 1.f / n : 0.f;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 16 * cb + 4 * q + i, e = 4 * cb + i;
        wm_s[wv][c] = fmaf(s1[e], inv, shs[wv][c]) + a.b1[c];
        wq_s[wv][c] = fmaxf(fmaf(-s1[e] * inv, s1[e], s2[e]), 0.f);
      }
    if (q == 0) wn_s[wv] = n;
  }
  __syncthreads();
  if (tid < MID) {
    double bn = 0.0, bm = 0.0, bq = 0.0;
    for (int w = 0; w < 4; ++w) {
      const double nb = wn_s[w];
      if (nb <= 0.0) continue;
      const double d = (double)wm_s[w][tid] - bm, nt = bn + nb;
      bm += d * nb / nt;
      bq += (double)wq_s[w][tid] + d * d * bn * nb / nt;
      bn = nt;
    }
    a.stats[((long long)blockIdx.x * 2 + 0) * MID + tid] = (float)(bm * bn);
    a.stats[((long long)blockIdx.x * 2 + 1) * MID + tid] = (float)bq;
    if (tid == 0) a.stats[(long long)2 * MID * gridDim.x + blockIdx.x] = (float)bn;
  }
}

// ---------------------------------------------------------------------------
// bf16 forward statistics from the second moments of the conv's input columns.  The head conv is
// linear in the im2col column col(p) (the 9K values of u around pixel p, zero outside the image):
//   mean_c = w_c . m + b1_c,   var_c = w_c^T Cov w_c,   m = E[col],  Cov = E[col col^T] - m m^T,
// with w_c = bf16(W1[c]) -- the operands head_out / bwd multiply -- so one pass accumulating
// G = sum_p col(p) col(p)^T over the valid pixels (bf16 col values are exact, their products exact
// in fp32) replaces computing and reducing all 64 channels of h per pixel.  The column is padded to
// 32 (two MFMA fragments); entry 31 is the pixel's validity (1 / 0), so G[j][31] = sum_p col_j and
// G[31][31] = the pixel count.  One partial row per block: the 00, 01 and 11 16x16 blocks of the
// symmetric 32x32 G, C layout (row 4q + i, column x), summed over the block's 4 waves.
// ---------------------------------------------------------------------------
constexpr int GRAM_LD = 3 * 256;

// su offset of column entry j = 16 jb + x relative to a pixel's window corner; -1: zero entry,
// -2: the validity entry (j = 31)
template <int K, int RS>
__device__ __forceinline__ void gram_offsets(int x, int (&o)[2]) {
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const int j = 16 * jb + x;
    if (j < K * 9) {
      const int k = j / 9, t = j - 9 * k, ky = t / 3, kx = t - 3 * ky;
      o[jb] = (ky * RS + kx) * 3 + k;
    } else {
      o[jb] = j == 31 ? -2 : -1;
    }
  }
}

// one 32-pixel group of a region with row stride RS (RS - 2 pixels per tile row): W = 16, tile rows r0,
// r0 + 1 (slot px = 8q + jj -> (r0 + (px >> 4), px & 15)); W = 32, tile row r0 (px -> (r0, px)).
// Lane (q, x) holds col_{16 jb + x} of slots 8q..8q+7: the A fragment of G's rows and, unchanged,
// the B fragment of its columns.
template <int RS>
__device__ __forceinline__ void gram_group(const float* su, int r0, int q, const int (&o)[2], int vh, int vw,
                                           f32x4& c00, f32x4& c01, f32x4& c11) {
  constexpr int W = RS - 2;
  bf16x8 f0, f1;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int px = 8 * q + jj, r = r0 + px / W, c = px % W;
    const bool valid = r < vh && c < vw;
    const int base = (r * RS + c) * 3;
    const float v0 = su[base + (o[0] < 0 ? 0 : o[0])];
    const float v1 = su[base + (o[1] < 0 ? 0 : o[1])];
    f0[jj] = (__bf16)(valid && o[0] >= 0 ? v0 : 0.f);
    f1[jj] = (__bf16)(!valid ? 0.f : o[1] >= 0 ? v1 : o[1] == -2 ? 1.f : 0.f);
  }
  c00 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, f0, c00, 0, 0, 0);
  c01 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, f1, c01, 0, 0, 0);
  c11 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1, f1, c11, 0, 0, 0);
}

// the same for a group whose 32 pixels are all inside the image (every group of a full tile): no validity
// factor, and the padding entries 9K <= j < 31 read the window corner instead of a selected zero -- they only
// reach G's rows / columns 9K .. 30, which nothing reads (each G entry is its own dot product over the
// pixels); the validity entry j = 31 (lanes with o1 == -2) is the constant 1.0 pair.  8 v_cvt_pk_bf16_f32
// per group instead of a select chain per entry; the G entries that are read are the same values.
template <int RS>
__device__ __forceinline__ void gram_group_full(const float* su, int r0, int q, int o0, int o1, bool one,
                                                f32x4& c00, f32x4& c01, f32x4& c11) {
  static_assert(RS - 2 == 32, "one tile row per 32-pixel group");
  const int base = (r0 * RS + 8 * q) * 3;
  uint32_t w0[4], w1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = base + 6 * i;
    w0[i] = pk_bf16(su[b + o0], su[b + 3 + o0]);
    const uint32_t v1 = pk_bf16(su[b + o1], su[b + 3 + o1]);
    w1[i] = one ? 0x3F803F80u : v1;
  }
  const bf16x8 f0 = __builtin_bit_cast(bf16x8, (u32x4){w0[0], w0[1], w0[2], w0[3]});
  const bf16x8 f1 = __builtin_bit_cast(bf16x8, (u32x4){w1[0], w1[1], w1[2], w1[3]});
  c00 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, f0, c00, 0, 0, 0);
  c01 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, f1, c01, 0, 0, 0);
  c11 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1, f1, c11, 0, 0, 0);
}

// the block's three G blocks -> one partial row (fixed-order sum of the 4 waves)
__device__ __forceinline__ void gram_store(float* red, float* row, const f32x4& c00, const f32x4& c01,
                                           const f32x4& c11) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4, x = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = (4 * q + i) * 16 + x;
    red[wv * GRAM_LD + e] = c00[i];
    red[wv * GRAM_LD + 256 + e] = c01[i];
    red[wv * GRAM_LD + 512 + e] = c11[i];
  }
  __syncthreads();
  for (int e = tid; e < GRAM_LD; e += NT)
    row[e] = (red[e] + red[GRAM_LD + e]) + (red[2 * GRAM_LD + e] + red[3 * GRAM_LD + e]);
}

// 32 x 32 tiles at 2H (4x the pixels of the other head kernels' tiles per barrier set): the 18 x 18 x K
// z region is staged, u = up(z) over the 34 x 34 region (zero outside the image, up2_src as stage_u),
// then each wave accumulates 8 rows of 32 pixels.  tx / ty / ntiles of HeadArgs describe these tiles.
constexpr int GT = 32, GR = GT + 2, GZ = GT / 2 + 2;
template <int K>
struct Z32 {
  static constexpr int ZN = GZ * GZ * K, ZI = (ZN + NT - 1) / NT;  // z values of a tile's region, per thread
};
__device__ __forceinline__ void tile32_coords(const HeadArgs& a, int tile, int& n, int& oy0, int& ox0) {
  const int tpi = a.tx * a.ty;  // (a.tx / a.ty count 32 x 32 tiles)
  n = tile / tpi;
  const int r = tile - n * tpi;
  oy0 = (r / a.tx) * GT;
  ox0 = (r % a.tx) * GT;
}
// the 18 x 18 x K z region a 32 x 32 tile interpolates from, edge-clamped, into registers
template <int K>
__device__ __forceinline__ void zfetch32(const HeadArgs& a, int tile, float (&zv)[Z32<K>::ZI]) {
  if (tile >= a.ntiles) return;
  int n, oy0, ox0;
  tile32_coords(a, tile, n, oy0, ox0);
  const int zy0 = oy0 / 2 - 1, zx0 = ox0 / 2 - 1;
  const float* zb = a.z + (long long)n * a.h * a.w * K;
#pragma unroll
  for (int j = 0; j < Z32<K>::ZI; ++j) {
    const int idx = threadIdx.x + j * NT;
    if (idx < Z32<K>::ZN) {
      const int k = idx % K, pix = idx / K, i = pix / GZ, c = pix - i * GZ;
      const int yy = min(max(zy0 + i, 0), a.h - 1), xx = min(max(zx0 + c, 0), a.w - 1);
      zv[j] = zb[((long long)yy * a.w + xx) * K + k];
    }
  }
}
// stage the prefetched z region, prefetch the next tile's, then u = up(z) over the 34 x 34 region from LDS
// (zero outside the image); the caller syncs before (su / zs free) and after (su complete)
template <int K>
__device__ void stage_u32(const HeadArgs& a, float* su, float* zs, float (&zv)[Z32<K>::ZI], int tile, int oy0,
                          int ox0) {
  const int tid = threadIdx.x, H2 = 2 * a.h, W2 = 2 * a.w;
#pragma unroll
  for (int j = 0; j < Z32<K>::ZI; ++j)
    if (tid + j * NT < Z32<K>::ZN) zs[tid + j * NT] = zv[j];
  __syncthreads();
  zfetch32<K>(a, tile + gridDim.x, zv);
  const int zy0 = oy0 / 2 - 1, zx0 = ox0 / 2 - 1;
  for (int i = tid; i < GR * GR; i += NT) {
    const int hy = i / GR, hx = i - hy * GR;
    const int oy = oy0 + hy - 1, ox = ox0 + hx - 1;
    const bool in = oy >= 0 && oy < H2 && ox >= 0 && ox < W2;
    int y0, y1, x0, x1;
    float ly, lx;
    up2_src_i(in ? oy : 0, a.h, y0, y1, ly);
    up2_src_i(in ? ox : 0, a.w, x0, x1, lx);
    const float* r0 = zs + ((y0 - zy0) * GZ) * K;
    const float* r1 = zs + ((y1 - zy0) * GZ) * K;
    const int c0 = (x0 - zx0) * K, c1 = (x1 - zx0) * K;
#pragma unroll
    for (int k = 0; k < K; ++k)
      su[i * 3 + k] = in ? up_lerp(ly, lx, r0[c0 + k], r0[c1 + k], r1[c0 + k], r1[c1 + k]) : 0.f;
  }
}
template <int K>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void head_gram_mfma_kernel(HeadArgs a) {
  __shared__ float su[GR * GR * 3];
  __shared__ float zs[GZ * GZ * 3];
  __shared__ float red[4 * GRAM_LD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4, x = lane & 15;
  int o[2];
  gram_offsets<K, GR>(x, o);
  const int o0c = o[0] < 0 ? 0 : o[0], o1c = o[1] < 0 ? 0 : o[1];
  const bool one = o[1] == -2;
  f32x4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c11 = c00;
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  float zv[Z32<K>::ZI];
  zfetch32<K>(a, blockIdx.x, zv);
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int n, oy0, ox0;
    tile32_coords(a, tile, n, oy0, ox0);
    __syncthreads();  // the previous tile's su reads are done
    stage_u32<K>(a, su, zs, zv, tile, oy0, ox0);
    __syncthreads();
    const int vh = min(GT, H2 - oy0), vw = min(GT, W2 - ox0);
    if (vh == GT && vw == GT) {
#pragma unroll 2
      for (int rr = 0; rr < GT / 4; ++rr)
        gram_group_full<GR>(su, 8 * wv + rr, q, o0c, o1c, one, c00, c01, c11);
    } else {
#pragma unroll 2
      for (int rr = 0; rr < GT / 4; ++rr) gram_group<GR>(su, 8 * wv + rr, q, o, vh, vw, c00, c01, c11);
    }
  }
  EUNET_DASSERT(a.gram != nullptr);
  gram_store(red, a.gram + (long long)blockIdx.x * GRAM_LD, c00, c01, c11);
}

// G (the column sums of the partial rows, fp32) -> one (sum, M2, count) statistics row for
// bn_finalize: per channel c (thread c) mean and variance of h_c = bf16(W1[c]) . col + b1[c], in fp64
__device__ __forceinline__ double gram_at(const float* g, int j, int jp) {
  if (j > jp) { const int t = j; j = jp; jp = t; }  // symmetric: the stored blocks are 00, 01, 11
  if (jp < 16) return (double)g[j * 16 + jp];
  if (j < 16) return (double)g[256 + j * 16 + (jp - 16)];
  return (double)g[512 + (j - 16) * 16 + (jp - 16)];
}

template <int K>
__global__ __launch_bounds__(MID) void head_gram_stats_kernel(const float* g, const float* w1, const float* b1,
                                                              float* stats) {
  constexpr int KJ = K * 9;
  __shared__ double cov[KJ][KJ], m[KJ];
  const int tid = threadIdx.x;
  const double n = (double)g[512 + 15 * 16 + 15];
  const double inv = n > 0.0 ? 1.0 / n : 0.0;
  if (tid < KJ) m[tid] = gram_at(g, tid, 31) * inv;
  __syncthreads();
  for (int e = tid; e < KJ * KJ; e += MID) {
    const int j = e / KJ, jp = e - j * KJ;
    cov[j][jp] = gram_at(g, j, jp) * inv - m[j] * m[jp];
  }
  __syncthreads();
  double wb[KJ];
#pragma unroll
  for (int j = 0; j < KJ; ++j) wb[j] = (double)(float)(__bf16)w1[tid * KJ + j];
  double mean = 0.0, var = 0.0;
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    mean += wb[j] * m[j];
    double t = 0.0;
#pragma unroll
    for (int jp = 0; jp < KJ; ++jp) t += cov[j][jp] * wb[jp];
    var += wb[j] * t;
  }
  stats[tid] = (float)((mean + (double)b1[tid]) * n);
  stats[MID + tid] = (float)(fmax(var, 0.0) * n);
  if (tid == 0) stats[2 * MID] = (float)n;
}

// bf16 forward output: h = conv3x3(u) by MFMA, BN + ReLU, the 1x1 by MFMA, residual, 2H output and the 2x2
// mean.  32 x 32 tiles (a.tx / a.ty / a.ntiles count them): one z and u stage per 1024 pixels (16 x 16
// tiles: 334 vs 281 us/launch at the bench shape, profiles/r03_ab.txt); wave w runs rows 8w .. 8w+7 as
// row pairs of 16-pixel segments.
template <int K>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void head_out32_mfma_kernel(HeadArgs a) {
  __shared__ float su[GR * GR * 3];
  __shared__ float zs[GZ * GZ * 3];
  __shared__ __attribute__((aligned(16))) float scs[MID], shs[MID];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4, x = lane & 15;
  if (tid < MID) {
    scs[tid] = a.scale[tid];
    shs[tid] = fmaf(a.b1[tid], a.scale[tid], a.shift[tid]);  // b1 folded into the shift
  }
  bf16x8 Ah[4], Ao[2];
  load_a_w1<K>(a.w1, lane, Ah);
  {
    float f[16];
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) f[8 * ch + jj] = a.w2[(x < K ? x : 0) * MID + perm_c(q, ch, jj)];
    keep_loads(f);
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) Ao[ch][jj] = (__bf16)(x < K ? f[8 * ch + jj] : 0.f);
  }
  int off[8];
  im2col_offsets<K, GR>(q, off);
  float b2k[K];
#pragma unroll
  for (int k = 0; k < K; ++k) b2k[k] = a.b2[k];
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  float zv[Z32<K>::ZI];
  zfetch32<K>(a, blockIdx.x, zv);
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int n, oy0, ox0;
    tile32_coords(a, tile, n, oy0, ox0);
    __syncthreads();
    stage_u32<K>(a, su, zs, zv, tile, oy0, ox0);
    __syncthreads();
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int rp = it >> 1, sx = 16 * (it & 1);
      float lsum[K];
#pragma unroll
      for (int k = 0; k < K; ++k) lsum[k] = 0.f;
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int r = 8 * wv + 2 * rp + rr, oy = oy0 + r, ox = ox0 + sx + x;
        f32x4 acc[4];
        conv_h_mfma(su, (r * GR + sx + x) * 3, off, Ah, acc);
        // BN + ReLU straight into the 1x1's B fragments (cfrag order): packed fp32 FMA per channel pair,
        // one v_cvt_pk_bf16_f32, ReLU on the rounded pair (round(max(v, 0)) == max(round(v), 0))
        uint32_t bw[4][2];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const f32x4 s4 = ld4v(scs + 16 * cb + 4 * q), t4 = ld4v(shs + 16 * cb + 4 * q);
#pragma unroll
          for (int hp = 0; hp < 2; ++hp) {
            const f32x2 v = pkfma(half2(acc[cb], hp), half2(s4, hp), half2(t4, hp));
            const s16x2 b = __builtin_bit_cast(s16x2, pk_bf16(v.x, v.y));
            bw[cb][hp] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(b, (s16x2){0, 0}));
          }
        }
        const bf16x8 f0 = __builtin_bit_cast(bf16x8, (u32x4){bw[0][0], bw[0][1], bw[1][0], bw[1][1]});
        const bf16x8 f1 = __builtin_bit_cast(bf16x8, (u32x4){bw[2][0], bw[2][1], bw[3][0], bw[3][1]});
        f32x4 o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ao[0], f0, z4, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ao[1], f1, o, 0, 0, 0);
        // lanes q == 0 hold o[k = i][pixel x]
        const bool pv = q == 0 && oy < H2 && ox < W2;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float val = o[k] + b2k[k] + su[((r + 1) * GR + sx + x + 1) * 3 + k];
          if (pv && a.out2h) a.out2h[(((long long)n * K + k) * H2 + oy) * W2 + ox] = val;
          lsum[k] += val;
        }
      }
      const int oy = oy0 + 8 * wv + 2 * rp, ox = ox0 + sx + x;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float t = lsum[k] + __shfl_xor(lsum[k], 1, 64);
        if (q == 0 && (x & 1) == 0 && oy < H2 && ox < W2 && a.logits)
          a.logits[(((long long)n * K + k) * a.h + (oy >> 1)) * a.w + (ox >> 1)] = 0.25f * t;
      }
    }
  }
}

// BN backward parameters, per channel: xhat = h*is + off, pre = h*P + Q (h without b1)
__device__ __forceinline__ void bwd_params(const HeadArgs& a, int c, float& is, float& off, float& P, float& Q) {
  is = a.istd[c];
  off = (a.b1[c] - a.mean[c]) * is;
  P = a.gamma[c] * is;
  Q = fmaf(a.gamma[c], off, a.beta[c]);
}

// g_o (the loss gradient w.r.t. the 2H output) over a tile's 16x16 pixels, K x 256 values,
// <= 3 per thread, held in registers one tile ahead and staged in LDS per tile: the per-row
// MFMA -> VALU chains of head_bwd1 / head_gh no longer wait on global loads.
template <int K>
__device__ __forceinline__ void goload(const HeadArgs& a, int tile, float (&gv)[3]) {
  if (tile >= a.ntiles) return;
  int n, oy0, ox0;
  tile_coords(a, tile, n, oy0, ox0);
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int p = threadIdx.x, oy = oy0 + (p >> 4), ox = ox0 + (p & 15);
    gv[j] = (oy < 2 * a.h && ox < 2 * a.w) ? g_raw(a, K, n, j, oy, ox) : 0.f;  // x g_scale when staged
  }
}

// bf16 backward pass 1: gW2, gb2, dbeta = sum g_bn, dgamma = sum g_bn * xhat.  The GEMMs are transposed: the
// im2col / g_o fragments are the A operands and W1 / W2^T the B operands, so lane (q, x) receives
// h[pixel 4q + i][channel 16cb + x]; its 4 channels are fixed for the whole kernel, the BN-backward
// constants (is, off, P, Q) live in VGPRs and each per-channel sum needs 4 accumulators, reduced over the 4
// lane groups q at the end.  32 x 32 tiles (a.tx / a.ty / a.ntiles count them): one z, u and g_o stage per
// 1024 pixels (16 x 16 tiles: 557 vs 497 us/launch, profiles/r03_ab.txt); wave w runs rows 8w .. 8w+7 as
// 16-pixel segments.  The g_o tile is loaded into registers before the u stage and stored after it, so its
// global latency hides behind the interpolation.
template <int K>
__global__ __launch_bounds__(NT, 3) void head_bwd1t32_mfma_kernel(HeadArgs a) {
  constexpr int STRIDE = (K + 2) * MID + K;
  constexpr int GO = GT * GT / NT;  // g_o values per thread and class
  __shared__ float su[GR * GR * 3];
  __shared__ float zs[GZ * GZ * 3];
  __shared__ float red[STRIDE];
  __shared__ __attribute__((aligned(16))) float gos[K * GT * GT];
  __shared__ __attribute__((aligned(16))) bf16x8 fr[4][64];  // W1 fragments (B operands here)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4, x = lane & 15;
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  for (int i = tid; i < STRIDE; i += NT) red[i] = 0.f;
  if (wv == 0) {
    bf16x8 A4[4];
    load_a_w1<K>(a.w1, lane, A4);
#pragma unroll
    for (int f = 0; f < 4; ++f) fr[f][lane] = A4[f];
  }
  float kI[4], kO[4], kP[4], kQ[4];  // channel 16cb + x (op_sel broadcasts them to both pixel halves)
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) bwd_params(a, 16 * cb + x, kI[cb], kO[cb], kP[cb], kQ[cb]);
  int off[8];
  im2col_offsets<K, GR>(q, off);
  // Per-channel sums as MFMAs over pixels with a row's g_o as the A operand (class m = lane & 15 < K, pixels
  // 4q .. 4q+3 of both 16-pixel segments): for channel c = 16cb + x
  //   gW2[k][c]    = sum_p g_o[p][k] relu(pre[p][c])                      (accA)
  //   dbeta[c]     = sum_p g_bn = sum_k W2[k][c] sum_p g_o[p][k] [pre > 0]  (accM)
  //   dgamma[c]    = sum_p g_bn xhat = sum_k W2[k][c] sum_p g_o[p][k] [pre > 0] xhat   (accN)
  // (g_bn = [pre > 0] s, s = W2^T g_o with the bf16 operands of the s GEMM it replaces); the B operands are
  // the bf16 pair of relu(pre), the mask (1.0 / 0) and the masked xhat, formed with 16-bit integer ops.
  f32x4 accA[4], accM[4], accN[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) accA[cb] = accM[cb] = accN[cb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float ab2 = 0.f;  // lanes x < K: sum of g_o of class x over this lane's pixels
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  const int gk = min(x, K - 1);
  const float gsc = g_scale(a);
  float zv[Z32<K>::ZI];
  zfetch32<K>(a, blockIdx.x, zv);
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int n, oy0, ox0;
    tile32_coords(a, tile, n, oy0, ox0);
    float gv[K][GO];
#pragma unroll
    for (int e = 0; e < GO; ++e) {
      const int p = tid + e * NT, oy = oy0 + p / GT, ox = ox0 + p % GT;
      const bool in = oy < H2 && ox < W2;
#pragma unroll
      for (int k = 0; k < K; ++k) gv[k][e] = in ? g_raw(a, K, n, k, oy, ox) : 0.f;  // x g_scale when staged
    }
    __syncthreads();  // the previous tile's su / gos reads are done
    stage_u32<K>(a, su, zs, zv, tile, oy0, ox0);
#pragma unroll
    for (int e = 0; e < GO; ++e)
#pragma unroll
      for (int k = 0; k < K; ++k) gos[k * GT * GT + tid + e * NT] = gv[k][e] * gsc;
    __syncthreads();
#pragma unroll 1
    for (int rr = 0; rr < GT / 4; ++rr) {  // row r: two 16-pixel segments, whose 8 pixels per lane fill the sums' k
      const int r = 8 * wv + rr;
      int fl = lane;
      asm volatile("" : "+v"(fl));  // keep the fragment reads in the loop (no LICM into registers)
      f32x4 acc[2][4];
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
        const bf16x8 b = im2col_frag(su, (r * GR + 16 * sg + x) * 3, off);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[sg][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, fr[cb][fl], z4, 0, 0, 0);
      }
      const bool kv = x < K;
      uint32_t gw[4];
#pragma unroll
      for (int sg = 0; sg < 2; ++sg) {
        const f32x4 gA = ld4v(gos + gk * GT * GT + r * GT + 16 * sg + 4 * q);  // 0 outside the image
        ab2 += kv ? (gA[0] + gA[1]) + (gA[2] + gA[3]) : 0.f;
        gw[2 * sg] = kv ? pk_bf16(gA[0], gA[1]) : 0u;
        gw[2 * sg + 1] = kv ? pk_bf16(gA[2], gA[3]) : 0u;
      }
      const bf16x8 ga = __builtin_bit_cast(bf16x8, (u32x4){gw[0], gw[1], gw[2], gw[3]});
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        uint32_t ba[4], bm[4], bx[4];
#pragma unroll
        for (int sg = 0; sg < 2; ++sg)
#pragma unroll
          for (int hp = 0; hp < 2; ++hp) {
            const f32x2 h = half2(acc[sg][cb], hp);
            const f32x2 xh = pkfma(h, (f32x2){kI[cb], kI[cb]}, (f32x2){kO[cb], kO[cb]});
            const f32x2 pre = pkfma(h, (f32x2){kP[cb], kP[cb]}, (f32x2){kQ[cb], kQ[cb]});
            // relu on the rounded pair; a half is nonzero iff pre > 0 (a positive fp32 rounds to a
            // positive bf16: the exponent ranges agree), so the mask comes from it in 16-bit integer ops
            const uint32_t act = __builtin_bit_cast(
                uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, pk_bf16(pre.x, pre.y)), (s16x2){0, 0}));
            const uint32_t m1 = pk_nonzero_one(act);
            ba[2 * sg + hp] = act;
            bm[2 * sg + hp] = pk_mul_u16s(m1, 0x3F803F80u);  // bf16 1.0 where pre > 0
            bx[2 * sg + hp] = pk_mul_u16(pk_bf16(xh.x, xh.y), m1);
          }
        accA[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, __builtin_bit_cast(bf16x8, (u32x4){ba[0], ba[1], ba[2], ba[3]}),
                                                           accA[cb], 0, 0, 0);
        accM[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, __builtin_bit_cast(bf16x8, (u32x4){bm[0], bm[1], bm[2], bm[3]}),
                                                           accM[cb], 0, 0, 0);
        accN[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, __builtin_bit_cast(bf16x8, (u32x4){bx[0], bx[1], bx[2], bx[3]}),
                                                           accN[cb], 0, 0, 0);
      }
    }
  }
  // lanes q == 0 hold class k = e of accX[cb][e] for channel 16cb + x
  float sgb[4], sgx[4], sw2[K][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    sgb[cb] = sgx[cb] = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float w2b = (float)(__bf16)a.w2[k * MID + 16 * cb + x];  // the s GEMM's bf16 W2
      sgb[cb] = fmaf(w2b, accM[cb][k], sgb[cb]);
      sgx[cb] = fmaf(w2b, accN[cb][k], sgx[cb]);
      sw2[k][cb] = accA[cb][k];
    }
  }
  ab2 += __shfl_xor(ab2, 16, 64);
  ab2 += __shfl_xor(ab2, 32, 64);
  for (int w = 0; w < 4; ++w) {
    __syncthreads();
    if (wv == w && q == 0) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int c = 16 * cb + x;
#pragma unroll
        for (int k = 0; k < K; ++k) red[k * MID + c] += sw2[k][cb];
        red[K * MID + c] += sgb[cb];
        red[(K + 1) * MID + c] += sgx[cb];
      }
      if (x < K) red[(K + 2) * MID + x] += ab2;
    }
  }
  __syncthreads();
  for (int i = tid; i < STRIDE; i += NT) a.part[(long long)blockIdx.x * STRIDE + i] = red[i];
}

// g_h (never stored), the per-tap products v = g_h * W1 and the W1/b1 gradients (MFMA over
// pixels from a wave-private bf16 g_h tile in LDS).  v stays on chip (as the H rows below): per tile
// the kernel forms g_u = g_o + sum_t v[q - d_t][t] over the 18x18 region the tile's pixels reach and
// applies the x2 upsample adjoint to it, writing the tile's 10x10 low-res patch of g_z;
// head_patch_gather adds the (at most four) patches covering each low-res pixel in a fixed order.  No
// v / g_u round trip through HBM (it was 0.6 GB written and read per step at 1024^2 x 4).
// Register budget (3 waves/SIMD to overlap the dependent MFMA -> VALU chains): the BN-backward
// algebra is folded into 4 per-channel constants, evaluated two channels per packed fp32 op,
//   pre = h P + Q,   g_h = P gbn + h D + E   (D = -P c2 is, E = -P (c2 off + c1)),
// and the constant A fragments (W1 for h, W2^T for s, W1^T for v) are read from LDS.
// The per-tap products are reduced over kx in registers as they leave the MFMA.
// The v MFMA's A rows are ordered so that lane (q, x) receives, for the combination cmb = (k, ky) =
// 4 jb + q, the three kx taps of pixel x (C rows 4q + kx); two row_shr DPP moves within the 16-lane
// pixel row give H[k][ky][r][cc] = sum_kx v[k][ky][kx][r][cc - kx] over the 18 region columns cc, kept
// in fp32.  The g_u pass then adds 3 rows of H per point and channel (9 bf16 taps before: 960 vs 900
// us/launch, and packed fp32 for the BN-backward algebra 1023 vs 900, profiles/r03_ab.txt).
__device__ __forceinline__ float dpp_shr(float v, int n) {  // lane x <- lane x - n of its 16-lane row, 0 below
  const int iv = __builtin_bit_cast(int, v);
  return __builtin_bit_cast(float, n == 1 ? __builtin_amdgcn_update_dpp(0, iv, 0x111, 0xf, 0xf, true)
                                          : __builtin_amdgcn_update_dpp(0, iv, 0x112, 0xf, 0xf, true));
}
// resident blocks per CU (K = 3: LDS allows 2).  Measured: 2 blocks / CU for K = 2, with or without the
// two rows of a pair unrolled, 1125-1141 vs 898-903 us (profiles/r04_ab.txt)
constexpr int gh_occ(int K) { return K == 3 ? 2 : 3; }
// Diagnostic build only (-DHEAD_STAMP=1, tools/head_stamps.py): per block of head_gh_mfma_kernel, wave 0's
// s_memtime sums over its tiles of staging (z / u / g_o, with the barriers), the row phase (h, s, BN
// backward, v, the W1-gradient MFMAs) and the tail (g_u, x2 upsample adjoint, patch store).
#ifndef HEAD_STAMP
#define HEAD_STAMP 0
#endif
#if HEAD_STAMP
__device__ unsigned long long g_head_stamps[1024 * 5];  // [block][total, staging, rows, tail, final reduction]
__device__ __forceinline__ unsigned long long head_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif
template <int K>
__global__ __launch_bounds__(NT, gh_occ(K)) void head_gh_mfma_kernel(HeadArgs a) {
  constexpr int STRIDE = MID * K * 9 + MID;
  constexpr int KJ = K * 9;
  __shared__ float su[18 * 18 * 3];
  __shared__ float zs[ZR * ZR * 3];
  __shared__ __attribute__((aligned(16))) float pP[MID], pQ[MID], pD[MID], pE[MID];
  constexpr int NJB = (3 * K + 3) / 4;  // v MFMAs: 4 (k, ky) combinations each
  __shared__ __attribute__((aligned(16))) bf16x8 fr[8 + 2 * NJB][64];  // Ah[4], As[4], Av[jb][ch] per lane
  constexpr int GLD = MID + 16;  // padded row: conflict-free transposed reads
  __shared__ __attribute__((aligned(16))) bf16_t gsw[4][32 * GLD];
  static_assert(STRIDE * 4 <= (int)sizeof(gsw), "red aliases gsw");
  float* red = (float*)&gsw[0][0];  // (used after the tile loop only)
  __shared__ float gos[K * T2 * T2];
  __shared__ float hb[3 * K][T2][18];   // H rows of the tile, [k * 3 + ky][tile row][region column]
  __shared__ float hxs[18 * 10 * 3];    // horizontal upsample adjoint of g_u [18 rows][10 cols][K]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, q = lane >> 4, x = lane & 15;
  const int H2 = 2 * a.h, W2 = 2 * a.w;
  if (tid < MID) {
    float is, of, P, Q;
    bwd_params(a, tid, is, of, P, Q);
    const float inv_cnt = 1.f / ((float)a.N * (float)H2 * (float)W2);
    const float c1 = a.dbeta[tid] * inv_cnt, c2 = a.dgamma[tid] * inv_cnt;
    pP[tid] = P; pQ[tid] = Q;
    pD[tid] = -P * c2 * is;
    pE[tid] = -P * fmaf(c2, of, c1);
  }
  if (wv == 0) {
    bf16x8 A4[4];
    load_a_w1<K>(a.w1, lane, A4);
#pragma unroll
    for (int f = 0; f < 4; ++f) fr[f][lane] = A4[f];
    load_a_w2t<K>(a.w2, lane, A4);
#pragma unroll
    for (int f = 0; f < 4; ++f) fr[4 + f][lane] = A4[f];
    float f[NJB * 16];
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
      const int cmb = 4 * jb + (x >> 2), kx = x & 3;  // A row x -> C row 4 (x >> 2) + kx
      const int j = (cmb < 3 * K && kx < 3) ? (cmb / 3) * 9 + (cmb % 3) * 3 + kx : KJ;
#pragma unroll
      for (int ch = 0; ch < 2; ++ch)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) f[16 * jb + 8 * ch + jj] = a.w1[perm_c(q, ch, jj) * KJ + (j < KJ ? j : 0)];
    }
    keep_loads(f);
#pragma unroll
    for (int jb = 0; jb < NJB; ++jb) {
      const int cmb = 4 * jb + (x >> 2), kx = x & 3;
      const bool jv = cmb < 3 * K && kx < 3;
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        bf16x8 v;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) v[jj] = (__bf16)(jv ? f[16 * jb + 8 * ch + jj] : 0.f);
        fr[8 + 2 * jb + ch][lane] = v;
      }
    }
  }
  int off[8];
  im2col_offsets<K>(q, off);
  // wgrad B operand: im2col[px slot 8q + jj][j = 16jb + x]; slot -> (row q>>1, col 8(q&1) + jj)
  int boff[2];
#pragma unroll
  for (int jb = 0; jb < 2; ++jb) {
    const int j = 16 * jb + x;
    if (j < KJ) {
      const int k = j / 9, t = j - 9 * k, ky = t / 3, kx = t - 3 * ky;
      boff[jb] = (((q >> 1) + ky) * 18 + 8 * (q & 1) + kx) * 3 + k;
    } else {
      boff[jb] = 0;
    }
  }
  f32x4 accW[4][2];
  float agb1[16];
#pragma unroll
  for (int pb = 0; pb < 4; ++pb) accW[pb][0] = accW[pb][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 16; ++e) agb1[e] = 0.f;
  f32x2 pgb1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) pgb1[e] = (f32x2){0.f, 0.f};
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  bf16_t* gw = gsw[wv];
  const int q4 = x >> 2, p4 = x & 3;
  float zv[2] = {0.f, 0.f}, gv[3] = {0.f, 0.f, 0.f};
  const float gsc = g_scale(a);
  zload<K>(a, blockIdx.x, zv);
  goload<K>(a, blockIdx.x, gv);
#if HEAD_STAMP
  const unsigned long long hs0 = head_stamp();
  unsigned long long hs_a = hs0, hs_b, hs_stage = 0, hs_rows = 0, hs_tail = 0;
#endif
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int n, oy0, ox0;
    tile_coords(a, tile, n, oy0, ox0);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) gos[k * T2 * T2 + tid] = gv[k] * gsc;
    stage_u<K>(a, su, zs, zv, tile, oy0, ox0);  // (syncs after staging z)
    goload<K>(a, tile + gridDim.x, gv);
    __syncthreads();
#if HEAD_STAMP
    hs_b = head_stamp();
    hs_stage += hs_b - hs_a;
#endif
#pragma unroll 1
    for (int rp = 0; rp < 2; ++rp) {
#pragma unroll 1
      for (int rr = 0; rr < 2; ++rr) {
        const int r = 4 * wv + 2 * rp + rr, oy = oy0 + r, ox = ox0 + x;
        const bool pv = oy < H2 && ox < W2;
        int fl = lane;
        asm volatile("" : "+v"(fl));  // keep the fragment reads in the loop (no LICM into registers)
        f32x4 acc[4];
        {
          const bf16x8 b = im2col_frag(su, (r * 18 + x) * 3, off);
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[cb][fl], b, z4, 0, 0, 0);
        }
        float go[K];
#pragma unroll
        for (int k = 0; k < K; ++k) go[k] = gos[k * T2 * T2 + r * T2 + x];  // 0 outside the image
        const bf16x8 gb = go_frag<K>(q, go);
        const f32x2 pvf = pv ? (f32x2){1.f, 1.f} : (f32x2){0.f, 0.f};
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const f32x4 sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[4 + cb][fl], gb, z4, 0, 0, 0);
          const int c0 = 16 * cb + 4 * q;
          const f32x4 P4 = ld4v(pP + c0), Q4 = ld4v(pQ + c0), D4 = ld4v(pD + c0), E4 = ld4v(pE + c0);
#pragma unroll
          for (int hp = 0; hp < 2; ++hp) {
            const f32x2 h = half2(acc[cb], hp), P = half2(P4, hp);
            const f32x2 gbn = relu_sel(pkfma(h, P, half2(Q4, hp)), half2(sv, hp));
            const f32x2 g = pkfma(P, gbn, pkfma(h, half2(D4, hp), half2(E4, hp))) * pvf;
            if (hp) acc[cb].hi = g; else acc[cb].lo = g;
            pgb1[2 * cb + hp] += g;
          }
        }
        const bf16x8 g0 = cfrag(acc, 0), g1 = cfrag(acc, 1);
        // every v MFMA first, then the g_h tile stores, then the kx reduction: the DPP reads of an MFMA result
        // no longer wait out its latency right behind it
        f32x4 vov[NJB];
#pragma unroll
        for (int jb = 0; jb < NJB; ++jb) {
          vov[jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[8 + 2 * jb][fl], g0, z4, 0, 0, 0);
          vov[jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[9 + 2 * jb][fl], g1, vov[jb], 0, 0, 0);
        }
        // wave-private g_h tile [32 px][64 positions], position 16q + 4cb + i <-> channel 16cb + 4q + i
        *(bf16x8*)(gw + (rr * 16 + x) * GLD + 16 * q) = g0;
        *(bf16x8*)(gw + (rr * 16 + x) * GLD + 16 * q + 8) = g1;
#pragma unroll
        for (int jb = 0; jb < NJB; ++jb) {
          const f32x4 vo = vov[jb];
          // (zero where the pixel is outside the image: g is)
          const float s1 = dpp_shr(vo[1], 1), s2 = dpp_shr(vo[2], 2), t1 = dpp_shr(vo[2], 1);
          const int cmb = 4 * jb + q;
          if (cmb < 3 * K) {
            float* hr = &hb[cmb][r][0];
            hr[x] = vo[0] + s1 + s2;
            if (x == 15) {
              hr[16] = vo[1] + t1;
              hr[17] = vo[2];
            }
          }
        }
      }
      // gw is wave-private: the wave's own LDS writes are in order before its reads (no block barrier)
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      const int r0 = 4 * wv + 2 * rp;
      bf16x8 Bw[2];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {  // (columns j >= 9K read finite u at boff 0; their sums are never stored)
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = pk_bf16(su[r0 * 54 + boff[jb] + 6 * i], su[r0 * 54 + boff[jb] + 6 * i + 3]);
        Bw[jb] = __builtin_bit_cast(bf16x8, (u32x4){w[0], w[1], w[2], w[3]});
      }
      const int pxa = 8 * q + q4;
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) {
        const s16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, (char*)gw + (pxa * GLD + 16 * pb + 4 * p4) * 2));
        const s16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, (char*)gw + ((pxa + 4) * GLD + 16 * pb + 4 * p4) * 2));
        const bf16x8 af = cat_bf16x4(alo, ahi);
        accW[pb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, Bw[0], accW[pb][0], 0, 0, 0);
        accW[pb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, Bw[1], accW[pb][1], 0, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();  // (the next rows' gw writes stay behind these reads)
    }
    __syncthreads();  // every wave's v rows are in vt and its Bw reads of su are done
#if HEAD_STAMP
    hs_a = head_stamp();
    hs_rows += hs_a - hs_b;
#endif
    // g_u over the region rows / cols oy0-1 .. oy0+16 (into su, free now), zero outside the image;
    // branch-free: out-of-tile taps read a clamped index and add zero
    for (int i = tid; i < 18 * 18; i += NT) {
      const int rr = i / 18, cc = i - rr * 18;
      const int oy = oy0 - 1 + rr, ox = ox0 - 1 + cc;
      const bool img = oy >= 0 && oy < H2 && ox >= 0 && ox < W2;
      const bool inner = img && rr >= 1 && rr <= T2 && cc >= 1 && cc <= T2;
      const int gi = inner ? (rr - 1) * T2 + cc - 1 : 0;
      float g[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float v = gos[k * T2 * T2 + gi];
        g[k] = inner ? v : 0.f;
      }
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {  // H rows of tile row rr - ky
        const int pr = rr - ky;
        const bool ok = img && pr >= 0 && pr < T2;
        const int ri = ok ? pr : 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const float v = hb[k * 3 + ky][ri][cc];
          g[k] += ok ? v : 0.f;
        }
      }
#pragma unroll
      for (int k = 0; k < K; ++k) su[i * 3 + k] = g[k];
    }
    __syncthreads();
    const int Y0 = oy0 / 2, X0 = ox0 / 2;
    // x2 upsample adjoint, columns first: hxs[rr][px] = sum_cc wx(ox, X) g_u[rr][cc], X = X0-1+px
    // (taps at high-res column 2X - 1 + d, region column cc; branch-free: a tap outside the region / image weighs 0)
    for (int i = tid; i < 18 * 10; i += NT) {
      const int rr = i / 10, px = i - rr * 10, X = X0 - 1 + px;
      const f32x4 wx4 = up2_adj_w4(X, a.w);
      const bool xv = X >= 0 && X < a.w;
      float hv[K];
#pragma unroll
      for (int k = 0; k < K; ++k) hv[k] = 0.f;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int cc = 2 * px - 2 + d;
        const bool ok = xv && cc >= 0 && cc < 18;
        const float wxv = ok ? wx4[d] : 0.f;
        const int ci = ok ? cc : 0;
#pragma unroll
        for (int k = 0; k < K; ++k) hv[k] = fmaf(wxv, su[(rr * 18 + ci) * 3 + k], hv[k]);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) hxs[i * 3 + k] = hv[k];
    }
    __syncthreads();
    if (tid < 100) {  // rows: patch[py][px] = sum_rr wy(oy, Y) hxs[rr][px], Y = Y0-1+py
      const int py = tid / 10, px = tid - py * 10, Y = Y0 - 1 + py;
      const f32x4 wy4 = up2_adj_w4(Y, a.h);
      const bool yv = Y >= 0 && Y < a.h;
      float pv[K];
#pragma unroll
      for (int k = 0; k < K; ++k) pv[k] = 0.f;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int rr = 2 * py - 2 + d;
        const bool ok = yv && rr >= 0 && rr < 18;
        const float wyv = ok ? wy4[d] : 0.f;
        const int ri = ok ? rr : 0;
#pragma unroll
        for (int k = 0; k < K; ++k) pv[k] = fmaf(wyv, hxs[(ri * 10 + px) * 3 + k], pv[k]);
      }
#pragma unroll
      EUNET_DASSERT(tile < a.ntiles && tid < 100);
#pragma unroll
      for (int k = 0; k < K; ++k) a.patch[((long long)tile * 100 + tid) * K + k] = pv[k];
    }
#if HEAD_STAMP
    hs_b = head_stamp();
    hs_tail += hs_b - hs_a;
    hs_a = hs_b;
#endif
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) agb1[e] = pgb1[e >> 1][e & 1];
#pragma unroll
  for (int e = 0; e < 16; ++e) agb1[e] = sum_x16(agb1[e]);
  __syncthreads();
  for (int i = tid; i < STRIDE; i += NT) red[i] = 0.f;
  for (int w = 0; w < 4; ++w) {
    __syncthreads();
    if (wv == w) {
      // accW[pb][jb][i]: row = position 16pb + 4q + i -> channel 16q + 4pb + i; col j = 16jb + x
#pragma unroll
      for (int pb = 0; pb < 4; ++pb)
#pragma unroll
        for (int jb = 0; jb < 2; ++jb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int c = 16 * q + 4 * pb + i, j = 16 * jb + x;
            if (j < KJ) red[c * KJ + j] += accW[pb][jb][i];
          }
      if (x == 0)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) red[MID * KJ + 16 * cb + 4 * q + i] += agb1[4 * cb + i];
    }
  }
  __syncthreads();
  for (int i = tid; i < STRIDE; i += NT) a.part[(long long)blockIdx.x * STRIDE + i] = red[i];
#if HEAD_STAMP
  const unsigned long long hs_e = head_stamp();
  if (tid == 0 && blockIdx.x < 1024) {
    unsigned long long* o = g_head_stamps + (size_t)blockIdx.x * 5;
    o[0] = hs_e - hs0;
    o[1] = hs_stage;
    o[2] = hs_rows;
    o[3] = hs_tail;
    o[4] = hs_e - hs_a;
  }
#endif
}

// g_z[n][y][x][k] = sum of the (at most four) tile patches covering low-res pixel (y, x), in a
// fixed order: tile rows y/8 - 1 .. y/8 + 1, then columns (a 16x16 tile at 2H covers low-res
// rows 8ty - 1 .. 8ty + 8)
template <int K>
__global__ __launch_bounds__(256) void head_patch_gather_kernel(const float* patch, float* gz, int N, int h, int w,
                                                                int tx, int ty) {
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long long)N * h * w) return;
  const int x = (int)(id % w);
  const int y = (int)((id / w) % h);
  const int n = (int)(id / ((long long)w * h));
  // the <= 4 covering patches' values, all 9 candidates loaded first (invalid ones from the buffer
  // start), then added in the fixed (dy, dx) order; +0.0 for a non-covering candidate leaves every
  // bit of the sum as skipping it did (the sum starts at +0.0 and never becomes -0.0)
  float v[9 * K];
  bool ok[9];
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      const int i = 3 * (dy + 1) + dx + 1;
      const int tr = y / 8 + dy, py = y - 8 * tr + 1, tc = x / 8 + dx, px = x - 8 * tc + 1;
      ok[i] = tr >= 0 && tr < ty && py >= 0 && py < 10 && tc >= 0 && tc < tx && px >= 0 && px < 10;
      const float* pp = ok[i] ? patch + ((((long long)n * ty + tr) * tx + tc) * 100 + py * 10 + px) * K : patch;
#pragma unroll
      for (int k = 0; k < K; ++k) v[i * K + k] = pp[k];
    }
  keep_loads(v);
  float acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.f;
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] += ok[i] ? v[i * K + k] : 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) gz[id * K + k] = acc[k];
}

struct WsLayout {
  size_t stats, part1, partw, gh, v, gu, patch, gram, gsum, scale, shift, cws, total;
  int grid, grid4;  // grid4: the bf16 forward kernels' grid (also the rows of the stats partials)
};
WsLayout ws_layout(int N, int h, int w, int K, int dtype) {
  const int tiles = N * cdiv(2 * w, T2) * cdiv(2 * h, T2);
  const int grid = tiles < HEAD_BLOCKS ? tiles : HEAD_BLOCKS;
  const size_t P2 = (size_t)N * 4 * h * w;
  WsLayout L;
  L.grid = grid;
  L.grid4 = dtype == EUNET_BF16 ? (tiles < HEAD_BLOCKS4 ? tiles : HEAD_BLOCKS4) : grid;
  size_t off = 0;
  auto take = [&](size_t floats) {
    size_t o = off;
    off += (floats + 63) / 64 * 64;
    return o;
  };
  L.stats = take((size_t)L.grid4 * (2 * MID + 1));
  L.part1 = take((size_t)grid * ((K + 2) * MID + K));
  L.partw = take((size_t)grid * (MID * K * 9 + MID));
  L.gh = take(dtype == EUNET_F32 ? P2 * MID : 0);  // the bf16 path never stores g_h
  // per-tap products v[j][pixel]: fp32 (fp32 path) / bf16 (bf16 path, the dgrad operand precision
  // of the reference's autocast)
  // fp32 path: per-tap products v[j][pixel] and g_u at 2H; the bf16 path keeps both on chip and
  // writes 10x10 low-res patches per tile instead
  L.v = take(dtype == EUNET_F32 ? P2 * ((K * 9 + 3) & ~3) : 0);
  L.gu = take(dtype == EUNET_F32 ? P2 * K : 0);
  L.patch = take(dtype == EUNET_F32 ? 0 : (size_t)tiles * 100 * K);
  L.gram = take(dtype == EUNET_F32 ? 0 : (size_t)L.grid4 * GRAM_LD);
  L.gsum = take(dtype == EUNET_F32 ? 0 : (size_t)GRAM_LD);
  L.scale = take(MID);
  L.shift = take(MID);
  // fp64 colsum stage-1 rows (<= 16 for <= 1024 rows)
  L.cws = take((size_t)2 * 16 * std::max(MID * K * 9 + MID, GRAM_LD));
  L.total = off * sizeof(float);
  return L;
}

}  // namespace

extern "C" int eunet_bn_eval_affine(int, const float*, const float*, const float*, const float*, float, float*,
                                    float*, void*);
extern "C" int eunet_upsample_bwd(const eunet_act* ghi, const eunet_act* glo, void* stream);

#define HEAD_DISPATCH(KERNEL, ...)                  \
  do {                                              \
    if (k == 1) KERNEL<1><<<__VA_ARGS__>>>(a);      \
    else if (k == 2) KERNEL<2><<<__VA_ARGS__>>>(a); \
    else KERNEL<3><<<__VA_ARGS__>>>(a);             \
  } while (0)
#define HEAD_DISPATCH_T(KERNEL, T, ...)                \
  do {                                                 \
    if (k == 1) KERNEL<1, T><<<__VA_ARGS__>>>(a);      \
    else if (k == 2) KERNEL<2, T><<<__VA_ARGS__>>>(a); \
    else KERNEL<3, T><<<__VA_ARGS__>>>(a);             \
  } while (0)

extern "C" {

#if HEAD_STAMP
int eunet_head_stamps(void* out, size_t bytes) {  // diagnostic builds only (tools/head_stamps.py)
  EUNET_REQUIRE(out && bytes <= sizeof(g_head_stamps), "head_stamps: bad args");
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_head_stamps), bytes, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return EUNET_ERR_HIP;
  return EUNET_OK;
}
#endif

int eunet_head_workspace_bytes(int n, int h, int w, int k, int dtype, size_t* bytes) {
  EUNET_REQUIRE(bytes && n > 0 && h > 0 && w > 0 && k >= 1 && k <= 3, "head_workspace_bytes: bad args");
  EUNET_REQUIRE(dtype == EUNET_F32 || dtype == EUNET_BF16, "head_workspace_bytes: dtype");
  *bytes = ws_layout(n, h, w, k, dtype).total;
  return EUNET_OK;
}

int eunet_head_fwd(const float* z, int n, int h, int w, int k, const float* w1, const float* b1, const float* gamma,
                   const float* beta, const float* w2, const float* b2, int training, float eps, float momentum,
                   float* run_mean, float* run_var, float* mean, float* invstd, float* out2h, float* logits,
                   int dtype, void* ws, void* stream) {
  EUNET_REQUIRE(z && w1 && b1 && gamma && beta && w2 && b2 && ws && k >= 1 && k <= 3, "head_fwd: bad args");
  EUNET_REQUIRE(out2h || logits, "head_fwd: nothing to write");
  EUNET_REQUIRE(!training || (mean && invstd), "head_fwd: training needs mean/invstd outputs");
  EUNET_REQUIRE(dtype == EUNET_F32 || dtype == EUNET_BF16, "head_fwd: dtype");
  const bool mf = dtype == EUNET_BF16;
  const WsLayout L = ws_layout(n, h, w, k, dtype);
  float* wsf = (float*)ws;
  HeadArgs a = {};
  a.z = z; a.N = n; a.h = h; a.w = w; a.K = k;
  a.w1 = w1; a.b1 = b1; a.gamma = gamma; a.beta = beta; a.w2 = w2; a.b2 = b2;
  a.tx = cdiv(2 * w, T2); a.ty = cdiv(2 * h, T2); a.ntiles = n * a.tx * a.ty;
  a.stats = wsf + L.stats; a.out2h = out2h; a.logits = logits;
  a.scale = wsf + L.scale; a.shift = wsf + L.shift;
  hipStream_t s = (hipStream_t)stream;
  if (training) {
    int rows = L.grid4;
    if (mf) {  // statistics from the im2col second moments (one stats row)
      a.gram = wsf + L.gram;
      HeadArgs ag = a;  // the Gram pass tiles 2H in 32 x 32
      ag.tx = cdiv(2 * w, GT); ag.ty = cdiv(2 * h, GT); ag.ntiles = n * ag.tx * ag.ty;
      {
        const HeadArgs a = ag;
        HEAD_DISPATCH(head_gram_mfma_kernel, L.grid4, NT, 0, s);
      }
      EUNET_LAUNCH_CHECK("head_gram");
      int rc = eunet_colsum_ld(a.gram, L.grid4, GRAM_LD, GRAM_LD, wsf + L.gsum, wsf + L.cws, s);
      if (rc) return rc;
      const float* gs = wsf + L.gsum;
      if (k == 1) head_gram_stats_kernel<1><<<1, MID, 0, s>>>(gs, w1, b1, a.stats);
      else if (k == 2) head_gram_stats_kernel<2><<<1, MID, 0, s>>>(gs, w1, b1, a.stats);
      else head_gram_stats_kernel<3><<<1, MID, 0, s>>>(gs, w1, b1, a.stats);
      rows = 1;
    } else {
      HEAD_DISPATCH(head_stats_kernel, L.grid, NT, 0, s);
    }
    EUNET_LAUNCH_CHECK("head_stats");
    int rc = eunet_bn_finalize(a.stats, rows, MID, gamma, beta, eps, momentum, run_mean, run_var, mean, invstd,
                               wsf + L.scale, wsf + L.shift, nullptr, stream);
    if (rc) return rc;
  } else {
    EUNET_REQUIRE(run_mean && run_var, "head_fwd: eval needs running stats");
    int rc = eunet_bn_eval_affine(MID, gamma, beta, run_mean, run_var, eps, wsf + L.scale, wsf + L.shift, stream);
    if (rc) return rc;
  }
  if (mf) {
    HeadArgs ag = a;  // 32 x 32 tiles
    ag.tx = cdiv(2 * w, GT); ag.ty = cdiv(2 * h, GT); ag.ntiles = n * ag.tx * ag.ty;
    const HeadArgs a = ag;
    HEAD_DISPATCH(head_out32_mfma_kernel, L.grid4, NT, 0, s);
  }
  else HEAD_DISPATCH(head_out_kernel, L.grid, NT, 0, s);
  EUNET_LAUNCH_CHECK("head_out");
  return EUNET_OK;
}

int eunet_head_bwd(const float* z, int n, int h, int w, int k, const float* w1, const float* b1, const float* gamma,
                   const float* beta, const float* w2, const float* mean, const float* invstd, const float* g_logits,
                   const float* g_out2h, float* gz, float* gw1, float* gb1, float* ggamma, float* gbeta, float* gw2,
                   float* gb2, int dtype, void* ws, void* stream) {
  EUNET_REQUIRE(z && w1 && b1 && gamma && beta && w2 && mean && invstd && gz && gw1 && gb1 && ggamma && gbeta &&
                    gw2 && gb2 && ws && k >= 1 && k <= 3,
                "head_bwd: bad args");
  EUNET_REQUIRE((g_logits != nullptr) != (g_out2h != nullptr), "head_bwd: exactly one of g_logits/g_out2h");
  EUNET_REQUIRE(dtype == EUNET_F32 || dtype == EUNET_BF16, "head_bwd: dtype");
  const bool mf = dtype == EUNET_BF16;
  const WsLayout L = ws_layout(n, h, w, k, dtype);
  float* wsf = (float*)ws;
  void* cws = wsf + L.cws;
  HeadArgs a = {};
  a.z = z; a.N = n; a.h = h; a.w = w; a.K = k;
  a.w1 = w1; a.b1 = b1; a.gamma = gamma; a.beta = beta; a.w2 = w2;
  a.mean = mean; a.istd = invstd; a.glog = g_logits; a.gout2h = g_out2h;
  a.tx = cdiv(2 * w, T2); a.ty = cdiv(2 * h, T2); a.ntiles = n * a.tx * a.ty;
  a.gh = wsf + L.gh; a.v = wsf + L.v; a.gu = wsf + L.gu; a.patch = wsf + L.patch;
  hipStream_t s = (hipStream_t)stream;
  int rc;
  a.part = wsf + L.part1;
  if (mf) {
    HeadArgs ag = a;  // 32 x 32 tiles
    ag.tx = cdiv(2 * w, GT); ag.ty = cdiv(2 * h, GT); ag.ntiles = n * ag.tx * ag.ty;
    const HeadArgs a = ag;
    HEAD_DISPATCH(head_bwd1t32_mfma_kernel, L.grid, NT, 0, s);
  }
  else HEAD_DISPATCH(head_bwd1_kernel, L.grid, NT, 0, s);
  EUNET_LAUNCH_CHECK("head_bwd1");
  const int ld1 = (k + 2) * MID + k;
  {  // one column sum over the packed row [gW2 | dbeta | dgamma | gb2]
    const ColSegs g = {{gw2, gbeta, ggamma, gb2}, {0, k * MID, (k + 1) * MID, (k + 2) * MID}, 4};
    if ((rc = eunet_colsum_segs(a.part, L.grid, ld1, ld1, g, cws, s))) return rc;
  }
  a.dbeta = gbeta; a.dgamma = ggamma;
  const long long P2 = (long long)n * 4 * h * w;
  // the gh grid: its resident blocks (256 CUs x gh_occ), no second partial round
  const int gridw = mf ? std::min(L.grid, 256 * gh_occ(k)) : L.grid;
  if (mf) {
    a.part = wsf + L.partw;  // g_h, v, the g_z patches and the W1/b1 partials in one pass
    HEAD_DISPATCH(head_gh_mfma_kernel, gridw, NT, 0, s);
    EUNET_LAUNCH_CHECK("head_gh_mfma");
  } else {
    HEAD_DISPATCH_T(head_bwd_gh_kernel, float, L.grid, NT, 0, s);
    EUNET_LAUNCH_CHECK("head_bwd_gh");
    HEAD_DISPATCH_T(head_bwd_gu_kernel, float, (unsigned)((P2 + 255) / 256), 256, 0, s);
    EUNET_LAUNCH_CHECK("head_bwd_gu");
    a.part = wsf + L.partw;
    HEAD_DISPATCH_T(head_wgrad_kernel, float, L.grid, NT, 0, s);
    EUNET_LAUNCH_CHECK("head_wgrad");
  }
  const int ldw = MID * k * 9 + MID;
  if ((rc = eunet_colsum_ld(a.part, gridw, MID * k * 9 + MID, ldw, gw1, cws, s, MID * k * 9, gb1))) return rc;
  if (mf) {
    const unsigned gg = (unsigned)(((long long)n * h * w + 255) / 256);
    if (k == 1) head_patch_gather_kernel<1><<<gg, 256, 0, s>>>(a.patch, gz, n, h, w, a.tx, a.ty);
    else if (k == 2) head_patch_gather_kernel<2><<<gg, 256, 0, s>>>(a.patch, gz, n, h, w, a.tx, a.ty);
    else head_patch_gather_kernel<3><<<gg, 256, 0, s>>>(a.patch, gz, n, h, w, a.tx, a.ty);
    EUNET_LAUNCH_CHECK("head_patch_gather");
    return EUNET_OK;
  }
  eunet_act ghi = {a.gu, n, 2 * h, 2 * w, k, k, 0, EUNET_F32};
  eunet_act glo = {gz, n, h, w, k, k, 0, EUNET_F32};
  return eunet_upsample_bwd(&ghi, &glo, stream);
}

}  // extern "C"
