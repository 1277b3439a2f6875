// Dual-branch fusion of the SMP-path EnhancedUNet (models.py:253-302, 316-333) and the
// consistency term of its auxiliary supervision (train_eval.py:199-234).
//
// Everything here is per-pixel work on 2K <= 6 channels (K = num_classes <= 3):
// HBM-bound, one thread per pixel, fp32 arithmetic.  The wide part of the fusion
// head (2K->256->128->64 3x3 convs) runs on the MFMA conv kernels (conv3x3.hip,
// bn_pool_up.hip); this file holds the narrow glue around it:
//   gate_conv_fwd   a  = conv3x3(ff, Wg1)          ff = cat(unetpp, deeplab)   models.py:280
//   gate_mid_fwd    b  = Wg2 gelu(bn1(a))                                      models.py:281-283
//   gate_out_fwd    f2 = ff * sigmoid(bn2(b))  (compute dtype, padded to 8 ch) models.py:284, 322-323
//   fusion_out_fwd  out = head 1x1(relu(bn3(y3))) + Wr f2 + br                models.py:294, 325-328
// and their backward.  Per-tile partial sums (BN statistics, weight gradients) are
// reduced in fixed order (block butterfly, then the fp64 colsum): deterministic.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int PPT = 8;             // pixels per thread
constexpr int TP = NT * PPT;       // pixels per tile (block)
constexpr int F2C = 8;             // channel stride of the f2 / g_f2 buffers (2K <= 6, 16-byte rows)

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

// fixed-order block sum of NV per-thread values; result in out[0..NV) (LDS), all threads synced
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* red /* [4][NV] */, float* out) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float x = v[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) red[wv * NV + i] = x;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NV; i += NT) out[i] = (red[i] + red[NV + i]) + (red[2 * NV + i] + red[3 * NV + i]);
  __syncthreads();
}

// BN statistics partials of one tile in the layout eunet_bn_finalize reads:
// st[tile][0][c] = sum, st[tile][1][c] = M2 about the tile mean, counts at st[2*C*tiles + tile]
template <int C>
__device__ __forceinline__ void tile_stats(float (&val)[PPT][C], const bool (&ok)[PPT], float cnt, float* red,
                                           float* buf, float* st, int tiles) {
  float s[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    s[c] = 0.f;
#pragma unroll
    for (int i = 0; i < PPT; ++i) s[c] += ok[i] ? val[i][c] : 0.f;
  }
  block_sum<C>(s, red, buf);
  float m2[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float mu = buf[c] / cnt;
    m2[c] = 0.f;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const float d = val[i][c] - mu;
      m2[c] += ok[i] ? d * d : 0.f;
    }
  }
  block_sum<C>(m2, red, buf + C);
  const int tile = blockIdx.x;
  if (threadIdx.x < C) {
    st[((long long)tile * 2 + 0) * C + threadIdx.x] = buf[threadIdx.x];
    st[((long long)tile * 2 + 1) * C + threadIdx.x] = buf[C + threadIdx.x];
  }
  if (threadIdx.x == 0) st[(long long)2 * C * tiles + tile] = cnt;
}

struct GateArgs {
  const float* za; const float* zb;  // branch outputs NHWC fp32 [N,H,W,K]
  int N, H, W;
  long long P;
  int tiles;
};

__device__ __forceinline__ float ff_at(const GateArgs& g, int K, long long pix, int j) {
  return j < K ? g.za[pix * K + j] : g.zb[pix * K + (j - K)];
}

// ---- forward ------------------------------------------------------------------------
// a[p][k] = sum_{t,j} Wg1[k][j][t] ff[p + d_t][j] (zero padding) + tile stats; also writes the
// aux outputs in NCHW (the _aux_outputs dict, models.py:329-332).
template <int K>
__global__ __launch_bounds__(NT) void gate_conv_fwd_kernel(GateArgs g, const float* w1, float* a, float* st,
                                                           float* aux_a, float* aux_b) {
  constexpr int C2 = 2 * K;
  __shared__ float ws[K * C2 * 9];
  __shared__ float red[4 * 2 * K], buf[2 * K];
  for (int i = threadIdx.x; i < K * C2 * 9; i += NT) ws[i] = w1[i];
  __syncthreads();
  const long long base = (long long)blockIdx.x * TP;
  const long long hw = (long long)g.H * g.W;
  float val[PPT][K];
  bool ok[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const long long p = base + i * NT + threadIdx.x;
    ok[i] = p < g.P;
#pragma unroll
    for (int k = 0; k < K; ++k) val[i][k] = 0.f;
    if (!ok[i]) continue;
    const int n = (int)(p / hw);
    const long long r = p - n * hw;
    const int y = (int)(r / g.W), x = (int)(r - (long long)y * g.W);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      if (yy < 0 || yy >= g.H || xx < 0 || xx >= g.W) continue;
      const long long q = (long long)n * hw + (long long)yy * g.W + xx;
#pragma unroll
      for (int j = 0; j < C2; ++j) {
        const float f = ff_at(g, K, q, j);
#pragma unroll
        for (int k = 0; k < K; ++k) val[i][k] = fmaf(ws[(k * C2 + j) * 9 + t], f, val[i][k]);
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      a[p * K + k] = val[i][k];
      aux_a[((long long)n * K + k) * hw + r] = g.za[p * K + k];
      aux_b[((long long)n * K + k) * hw + r] = g.zb[p * K + k];
    }
  }
  const float cnt = (float)min((long long)TP, g.P - base);
  tile_stats<K>(val, ok, cnt, red, buf, st, g.tiles);
}

// b[p][j] = sum_k Wg2[j][k] gelu(a[p][k] sc1[k] + sh1[k]) + tile stats (2K channels)
template <int K>
__global__ __launch_bounds__(NT) void gate_mid_fwd_kernel(GateArgs g, const float* a, const float* sc1,
                                                          const float* sh1, const float* w2, float* b, float* st) {
  constexpr int C2 = 2 * K;
  __shared__ float red[4 * 2 * C2], buf[2 * C2];
  const long long base = (long long)blockIdx.x * TP;
  float val[PPT][C2];
  bool ok[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const long long p = base + i * NT + threadIdx.x;
    ok[i] = p < g.P;
#pragma unroll
    for (int j = 0; j < C2; ++j) val[i][j] = 0.f;
    if (!ok[i]) continue;
    float v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = gelu_f(fmaf(a[p * K + k], sc1[k], sh1[k]));
#pragma unroll
    for (int j = 0; j < C2; ++j) {
#pragma unroll
      for (int k = 0; k < K; ++k) val[i][j] = fmaf(w2[j * K + k], v[k], val[i][j]);
      b[p * C2 + j] = val[i][j];
    }
  }
  const float cnt = (float)min((long long)TP, g.P - base);
  tile_stats<C2>(val, ok, cnt, red, buf, st, g.tiles);
}

// f2[p][j] = ff[p][j] sigmoid(b[p][j] sc2[j] + sh2[j]) -> compute dtype, [P][8] (pad = 0)
template <int K, typename T>
__global__ __launch_bounds__(NT) void gate_out_fwd_kernel(GateArgs g, const float* b, const float* sc2,
                                                          const float* sh2, T* f2) {
  constexpr int C2 = 2 * K;
  for (long long p = (long long)blockIdx.x * NT + threadIdx.x; p < g.P; p += (long long)gridDim.x * NT) {
    float o[F2C];
#pragma unroll
    for (int j = 0; j < F2C; ++j) o[j] = 0.f;
#pragma unroll
    for (int j = 0; j < C2; ++j) o[j] = ff_at(g, K, p, j) * sigmoid_f(fmaf(b[p * C2 + j], sc2[j], sh2[j]));
    T* d = f2 + p * F2C;
    if constexpr (sizeof(T) == 2) {
      *(uint4*)d = Vec16<T>::pack(o);
    } else {
      *(uint4*)d = Vec16<T>::pack(o);
      *(uint4*)(d + 4) = Vec16<T>::pack(o + 4);
    }
  }
}

// out[n][k][y][x] = b11[k] + sum_c W11[k][c] relu(y3 sc3 + sh3)[c] + br[k] + sum_j Wr[k][j] f2[j]
// (f2 recomputed in fp32 from b and ff; models.py:294, 325-328)
template <int K, typename T>
__global__ __launch_bounds__(NT) void fusion_out_fwd_kernel(GateArgs g, const T* y3, const float* sc3,
                                                            const float* sh3, const float* w11, const float* b11,
                                                            const float* b, const float* sc2, const float* sh2,
                                                            const float* wr, const float* br, float* out) {
  constexpr int C2 = 2 * K, CH = 64, E = Vec16<T>::N;
  __shared__ float s_sc[CH], s_sh[CH], s_w[K * CH];
  for (int i = threadIdx.x; i < CH; i += NT) { s_sc[i] = sc3[i]; s_sh[i] = sh3[i]; }
  for (int i = threadIdx.x; i < K * CH; i += NT) s_w[i] = w11[i];
  __syncthreads();
  const long long hw = (long long)g.H * g.W;
  for (long long p = (long long)blockIdx.x * NT + threadIdx.x; p < g.P; p += (long long)gridDim.x * NT) {
    float acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = b11[k] + br[k];
#pragma unroll
    for (int u = 0; u < CH / E; ++u) {
      float f[E];
      Vec16<T>::unpack(*(const uint4*)(y3 + p * CH + u * E), f);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int c = u * E + e;
        const float h = fmaxf(fmaf(f[e], s_sc[c], s_sh[c]), 0.f);
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = fmaf(s_w[k * CH + c], h, acc[k]);
      }
    }
#pragma unroll
    for (int j = 0; j < C2; ++j) {
      const float f2 = ff_at(g, K, p, j) * sigmoid_f(fmaf(b[p * C2 + j], sc2[j], sh2[j]));
#pragma unroll
      for (int k = 0; k < K; ++k) acc[k] = fmaf(wr[k * C2 + j], f2, acc[k]);
    }
    const int n = (int)(p / hw);
    const long long r = p - n * hw;
#pragma unroll
    for (int k = 0; k < K; ++k) out[((long long)n * K + k) * hw + r] = acc[k];
  }
}

// ---- backward -----------------------------------------------------------------------
// From d out (NCHW): gz [P][K] (NHWC, for the head 1x1 backward), g_f2res[p][j] =
// sum_k Wr[k][j] gout[k], partials [tile][K*2K + K] of dWr (k-major) and dbr.
template <int K>
__global__ __launch_bounds__(NT) void fusion_out_bwd_kernel(GateArgs g, const float* gout, const float* b,
                                                            const float* sc2, const float* sh2, const float* wr,
                                                            float* gz, float* gf2res, float* part) {
  constexpr int C2 = 2 * K, NV = K * C2 + K;
  __shared__ float red[4 * NV], buf[NV];
  const long long base = (long long)blockIdx.x * TP, hw = (long long)g.H * g.W;
  float acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.f;
  for (int i = 0; i < PPT; ++i) {
    const long long p = base + i * NT + threadIdx.x;
    if (p >= g.P) break;
    const int n = (int)(p / hw);
    const long long r = p - n * hw;
    float go[K], f2[C2];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      go[k] = gout[((long long)n * K + k) * hw + r];
      gz[p * K + k] = go[k];
      acc[K * C2 + k] += go[k];
    }
#pragma unroll
    for (int j = 0; j < C2; ++j) {
      f2[j] = ff_at(g, K, p, j) * sigmoid_f(fmaf(b[p * C2 + j], sc2[j], sh2[j]));
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        s = fmaf(wr[k * C2 + j], go[k], s);
        acc[k * C2 + j] = fmaf(go[k], f2[j], acc[k * C2 + j]);
      }
      gf2res[p * C2 + j] = s;
    }
  }
  block_sum<NV>(acc, red, buf);
  for (int i = threadIdx.x; i < NV; i += NT) part[(long long)blockIdx.x * NV + i] = buf[i];
}

// gate backward 1: g_f2 = g_f2conv + g_f2res; att = sigmoid(bn2(b)); g_ffd = g_f2 att;
// g_bhat = g_f2 ff att (1 - att) (gradient w.r.t. the BN2 output) + partials [tile][2][2K]
// (sum g_bhat, sum g_bhat xhat2) for the BN2 backward.
template <int K, typename T>
__global__ __launch_bounds__(NT) void gate_bwd1_kernel(GateArgs g, const T* gf2conv, const float* gf2res,
                                                       const float* b, const float* mean2, const float* istd2,
                                                       const float* gam2, const float* bet2, float* gffd,
                                                       float* gbhat, float* part) {
  constexpr int C2 = 2 * K, NV = 2 * C2;
  __shared__ float red[4 * NV], buf[NV];
  const long long base = (long long)blockIdx.x * TP;
  float acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.f;
  for (int i = 0; i < PPT; ++i) {
    const long long p = base + i * NT + threadIdx.x;
    if (p >= g.P) break;
    float gc[F2C];
    if constexpr (sizeof(T) == 2) {
      Vec16<T>::unpack(*(const uint4*)(gf2conv + p * F2C), gc);
    } else {
      Vec16<T>::unpack(*(const uint4*)(gf2conv + p * F2C), gc);
      Vec16<T>::unpack(*(const uint4*)(gf2conv + p * F2C + 4), gc + 4);
    }
#pragma unroll
    for (int j = 0; j < C2; ++j) {
      const float gf = gc[j] + gf2res[p * C2 + j];
      const float xh = (b[p * C2 + j] - mean2[j]) * istd2[j];
      const float at = sigmoid_f(fmaf(gam2[j], xh, bet2[j]));
      gffd[p * C2 + j] = gf * at;
      const float gb = gf * ff_at(g, K, p, j) * at * (1.f - at);
      gbhat[p * C2 + j] = gb;
      acc[j] += gb;
      acc[C2 + j] = fmaf(gb, xh, acc[C2 + j]);
    }
  }
  block_sum<NV>(acc, red, buf);
  if (threadIdx.x < C2) {
    part[((long long)blockIdx.x * 2 + 0) * C2 + threadIdx.x] = buf[threadIdx.x];
    part[((long long)blockIdx.x * 2 + 1) * C2 + threadIdx.x] = buf[C2 + threadIdx.x];
  }
}

// gate backward 2: g_b = BN2 backward; g_v = Wg2^T g_b; g_abn = g_v gelu'(bn1(a)) (stored);
// partials [tile][2K*K + 2K] = dWg2 (j-major, torch [2K][K]) and the BN1 reductions
// (sum g_abn, sum g_abn xhat1) laid out [2][K].
template <int K>
__global__ __launch_bounds__(NT) void gate_bwd2_kernel(GateArgs g, const float* gbhat, const float* b,
                                                       const float* mean2, const float* istd2, const float* gam2,
                                                       const float* dbet2, const float* dgam2, const float* a,
                                                       const float* mean1, const float* istd1, const float* gam1,
                                                       const float* bet1, const float* w2, float* gabn, float* part) {
  constexpr int C2 = 2 * K, NV = C2 * K + 2 * K;
  __shared__ float red[4 * NV], buf[NV];
  const long long base = (long long)blockIdx.x * TP;
  const float inv_n = 1.f / (float)g.P;
  float acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.f;
  for (int i = 0; i < PPT; ++i) {
    const long long p = base + i * NT + threadIdx.x;
    if (p >= g.P) break;
    float gb[C2];
#pragma unroll
    for (int j = 0; j < C2; ++j) {
      const float xh = (b[p * C2 + j] - mean2[j]) * istd2[j];
      gb[j] = gam2[j] * istd2[j] * (gbhat[p * C2 + j] - dbet2[j] * inv_n - xh * dgam2[j] * inv_n);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float xh = (a[p * K + k] - mean1[k]) * istd1[k];
      const float abn = fmaf(gam1[k], xh, bet1[k]);
      const float v = gelu_f(abn);
      float gv = 0.f;
#pragma unroll
      for (int j = 0; j < C2; ++j) {
        gv = fmaf(w2[j * K + k], gb[j], gv);
        acc[j * K + k] = fmaf(gb[j], v, acc[j * K + k]);
      }
      const float ga = gv * gelu_grad(abn);
      gabn[p * K + k] = ga;
      acc[C2 * K + k] += ga;
      acc[C2 * K + K + k] = fmaf(ga, xh, acc[C2 * K + K + k]);
    }
  }
  block_sum<NV>(acc, red, buf);
  for (int i = threadIdx.x; i < NV; i += NT) part[(long long)blockIdx.x * NV + i] = buf[i];
}

// gate backward 3 (one 16x32 pixel tile per block): g_a = BN1 backward of g_abn (applied while
// staging the tile + halo in LDS); g_ff[p][j] = g_ffd[p][j] + sum_{t,k} Wg1[k][j][t] g_a[p - d_t][k]
// (+ the aux-output gradients), split into the two branch gradients gz_a / gz_b (NHWC fp32);
// partials [tile][K*2K*9] of dWg1[k][j][t] = sum_q g_a[q][k] ff[q + d_t][j].
constexpr int GTH = 16, GTW = 32, GHP = (GTH + 2) * (GTW + 2);
template <int K>
__global__ __launch_bounds__(NT) void gate_bwd3_kernel(GateArgs g, const float* gabn, const float* a,
                                                       const float* mean1, const float* istd1, const float* gam1,
                                                       const float* dbet1, const float* dgam1, const float* w1,
                                                       const float* gffd, const float* gaux_a, const float* gaux_b,
                                                       float* gz_a, float* gz_b, float* part, int tx, int ty) {
  constexpr int C2 = 2 * K, NW = K * C2 * 9;
  __shared__ float sga[GHP * K];   // g_a over the tile + halo
  __shared__ float sff[GHP * C2];  // ff over the tile + halo
  __shared__ float ws[NW];
  const int tile = blockIdx.x, tpi = tx * ty;
  const int n = tile / tpi, trem = tile - n * tpi;
  const int y0 = (trem / tx) * GTH, x0 = (trem % tx) * GTW;
  const long long hw = (long long)g.H * g.W;
  const float inv_n = 1.f / (float)g.P;
  for (int i = threadIdx.x; i < NW; i += NT) ws[i] = w1[i];
  for (int hp = threadIdx.x; hp < GHP; hp += NT) {
    const int yy = y0 + hp / (GTW + 2) - 1, xx = x0 + hp % (GTW + 2) - 1;
    const bool in = yy >= 0 && yy < g.H && xx >= 0 && xx < g.W;
    const long long q = (long long)n * hw + (long long)yy * g.W + xx;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float v = 0.f;
      if (in) {
        const float xh = (a[q * K + k] - mean1[k]) * istd1[k];
        v = gam1[k] * istd1[k] * (gabn[q * K + k] - dbet1[k] * inv_n - xh * dgam1[k] * inv_n);
      }
      sga[hp * K + k] = v;
    }
#pragma unroll
    for (int j = 0; j < C2; ++j) sff[hp * C2 + j] = in ? ff_at(g, K, q, j) : 0.f;
  }
  __syncthreads();
  for (int px = threadIdx.x; px < GTH * GTW; px += NT) {
    const int r = px / GTW, c = px % GTW;
    const int yy = y0 + r, xx = x0 + c;
    if (yy >= g.H || xx >= g.W) continue;
    const long long p = (long long)n * hw + (long long)yy * g.W + xx;
    const long long rr = (long long)yy * g.W + xx;
    float gf[C2];
#pragma unroll
    for (int j = 0; j < C2; ++j) gf[j] = gffd[p * C2 + j];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // g_a at p - d_t: halo coordinates (r + 1 - dy, c + 1 - dx), d_t = (t/3 - 1, t%3 - 1)
      const int hp = (r + 2 - t / 3) * (GTW + 2) + (c + 2 - t % 3);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float ga = sga[hp * K + k];
#pragma unroll
        for (int j = 0; j < C2; ++j) gf[j] = fmaf(ws[(k * C2 + j) * 9 + t], ga, gf[j]);
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const long long o = ((long long)n * K + k) * hw + rr;
      gz_a[p * K + k] = gf[k] + (gaux_a ? gaux_a[o] : 0.f);
      gz_b[p * K + k] = gf[K + k] + (gaux_b ? gaux_b[o] : 0.f);
    }
  }
  // dWg1 partials: thread (k, j, t) sums over the tile's pixels (g_a at q, ff at q + d_t)
  if (threadIdx.x < NW) {
    const int k = threadIdx.x / (C2 * 9), rem = threadIdx.x % (C2 * 9), j = rem / 9, t = rem % 9;
    const int dy = t / 3, dx = t % 3;
    float s = 0.f;
    for (int px = 0; px < GTH * GTW; ++px) {
      const int r = px / GTW, c = px % GTW;
      const float ga = sga[((r + 1) * (GTW + 2) + c + 1) * K + k];
      s = fmaf(ga, sff[((r + dy) * (GTW + 2) + c + dx) * C2 + j], s);
    }
    part[(long long)tile * NW + threadIdx.x] = s;
  }
}

// ---- consistency term: c_b * mean((softmax(branch_b) - softmax(fused))^2) per sample --
// fwd partials [tile][N... ] -> sq[n][b] via per-(sample, tile) block sums
template <int K>
__global__ __launch_bounds__(NT) void consistency_fwd_kernel(const float* fused, const float* br0, const float* br1,
                                                             long long hw, float* part) {
  // grid: (tiles of one sample, N); part[n][tile][2]
  const int n = blockIdx.y;
  __shared__ float red[4 * 2], buf[2];
  float acc[2] = {0.f, 0.f};
  const long long base = (long long)blockIdx.x * TP;
  for (int i = 0; i < PPT; ++i) {
    const long long r = base + i * NT + threadIdx.x;
    if (r >= hw) break;
    float pf[K], m = -INFINITY, s = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { pf[k] = fused[((long long)n * K + k) * hw + r]; m = fmaxf(m, pf[k]); }
#pragma unroll
    for (int k = 0; k < K; ++k) { pf[k] = expf(pf[k] - m); s += pf[k]; }
#pragma unroll
    for (int k = 0; k < K; ++k) pf[k] /= s;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
      const float* bl = bi == 0 ? br0 : br1;
      float pb[K], mb = -INFINITY, sb = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) { pb[k] = bl[((long long)n * K + k) * hw + r]; mb = fmaxf(mb, pb[k]); }
#pragma unroll
      for (int k = 0; k < K; ++k) { pb[k] = expf(pb[k] - mb); sb += pb[k]; }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float d = pb[k] / sb - pf[k];
        acc[bi] = fmaf(d, d, acc[bi]);
      }
    }
  }
  block_sum<2>(acc, red, buf);
  if (threadIdx.x < 2) part[((long long)n * gridDim.x + blockIdx.x) * 2 + threadIdx.x] = buf[threadIdx.x];
}

// loss = sum_b coef[b] * (1/N) sum_n sq[n][b] / (K hw), partial sums in fixed order (fp64)
__global__ void consistency_finalize_kernel(const float* part, int N, int tiles, float c0, float c1, long long khw,
                                            float* loss) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double t0 = 0.0, t1 = 0.0;
  for (int n = 0; n < N; ++n)
    for (int t = 0; t < tiles; ++t) {
      t0 += (double)part[((long long)n * tiles + t) * 2 + 0];
      t1 += (double)part[((long long)n * tiles + t) * 2 + 1];
    }
  *loss = (float)(((double)c0 * t0 + (double)c1 * t1) / ((double)N * (double)khw));
}

// d/d branch_b = s_b J_b^T (pb - pf), d/d fused = sum_b s_b J_f^T (pf - pb),
// s_b = 2 coef_b gloss / (N K hw); J^T v = p (v - <v, p>).  Gradients are ACCUMULATED.
template <int K>
__global__ __launch_bounds__(NT) void consistency_bwd_kernel(const float* fused, const float* br0, const float* br1,
                                                             long long hw, long long total, float s0, float s1,
                                                             const float* gloss, float* gf, float* g0, float* g1) {
  const float gl = *gloss;
  for (long long id = (long long)blockIdx.x * NT + threadIdx.x; id < total; id += (long long)gridDim.x * NT) {
    const long long n = id / hw, r = id - n * hw;
    float pf[K], m = -INFINITY, s = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { pf[k] = fused[(n * K + k) * hw + r]; m = fmaxf(m, pf[k]); }
#pragma unroll
    for (int k = 0; k < K; ++k) { pf[k] = expf(pf[k] - m); s += pf[k]; }
#pragma unroll
    for (int k = 0; k < K; ++k) pf[k] /= s;
    float vf[K];
#pragma unroll
    for (int k = 0; k < K; ++k) vf[k] = 0.f;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
      const float* bl = bi == 0 ? br0 : br1;
      float* gb = bi == 0 ? g0 : g1;
      const float sc = (bi == 0 ? s0 : s1) * gl;
      float pb[K], mb = -INFINITY, sb = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) { pb[k] = bl[(n * K + k) * hw + r]; mb = fmaxf(mb, pb[k]); }
#pragma unroll
      for (int k = 0; k < K; ++k) { pb[k] = expf(pb[k] - mb); sb += pb[k]; }
      float v[K], dot = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        pb[k] /= sb;
        v[k] = sc * (pb[k] - pf[k]);
        dot = fmaf(v[k], pb[k], dot);
        vf[k] -= v[k];
      }
#pragma unroll
      for (int k = 0; k < K; ++k) gb[(n * K + k) * hw + r] += pb[k] * (v[k] - dot);
    }
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) dot = fmaf(vf[k], pf[k], dot);
#pragma unroll
    for (int k = 0; k < K; ++k) gf[(n * K + k) * hw + r] += pf[k] * (vf[k] - dot);
  }
}

// Dropout2d folded into the preceding BN+ReLU affine (models.py:287, 291): keep [n][c] in {0,1};
// per-sample sc' = sc keep/(1-p), sh' = sh keep/(1-p) (relu(x) m = relu(x m) for m >= 0) and the
// backward scale g = keep/(1-p) (nullable outputs)
__global__ void dropout_affine_kernel(const float* sc, const float* sh, const float* keep, int n, int c, float inv_q,
                                      float* osc, float* osh, float* og) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * c) return;
  const int ch = i % c;
  const float m = keep[i] * inv_q;
  osc[i] = sc[ch] * m;
  osh[i] = sh[ch] * m;
  if (og) og[i] = m;
}

unsigned grid_for(long long n) {
  long long b = (n + NT - 1) / NT;
  if (b > 16384) b = 16384;
  return (unsigned)(b < 1 ? 1 : b);
}

GateArgs gate_args(const float* za, const float* zb, int n, int h, int w) {
  GateArgs g;
  g.za = za; g.zb = zb; g.N = n; g.H = h; g.W = w;
  g.P = (long long)n * h * w;
  g.tiles = (int)((g.P + TP - 1) / TP);
  return g;
}

#define EUNET_K_DISPATCH(k, ...)        \
  do {                                  \
    if ((k) == 2) {                     \
      constexpr int KK = 2;             \
      __VA_ARGS__;                      \
    } else if ((k) == 3) {              \
      constexpr int KK = 3;             \
      __VA_ARGS__;                      \
    } else {                            \
      constexpr int KK = 1;             \
      __VA_ARGS__;                      \
    }                                   \
  } while (0)

}  // namespace

extern "C" {

int eunet_fusion_tiles(int n, int h, int w, int* tiles, int* gate_tiles) {
  EUNET_REQUIRE(n > 0 && h > 0 && w > 0 && tiles, "fusion_tiles: bad args");
  const long long P = (long long)n * h * w;
  *tiles = (int)((P + TP - 1) / TP);
  if (gate_tiles) *gate_tiles = n * cdiv(h, GTH) * cdiv(w, GTW);
  return EUNET_OK;
}

int eunet_gate_fwd(const float* za, const float* zb, int n, int h, int w, int k, const float* w1, float* a,
                   float* st1, float* aux_a, float* aux_b, void* stream) {
  EUNET_REQUIRE(za && zb && w1 && a && st1 && aux_a && aux_b && n > 0 && h > 0 && w > 0 && k >= 1 && k <= 3,
                "gate_fwd: bad args");
  GateArgs g = gate_args(za, zb, n, h, w);
  EUNET_K_DISPATCH(k, gate_conv_fwd_kernel<KK><<<g.tiles, NT, 0, (hipStream_t)stream>>>(g, w1, a, st1, aux_a, aux_b));
  EUNET_LAUNCH_CHECK("gate_fwd");
  return EUNET_OK;
}

int eunet_gate_mid_fwd(const float* za, const float* zb, int n, int h, int w, int k, const float* a,
                       const float* sc1, const float* sh1, const float* w2, float* b, float* st2, void* stream) {
  EUNET_REQUIRE(a && sc1 && sh1 && w2 && b && st2 && k >= 1 && k <= 3, "gate_mid_fwd: bad args");
  GateArgs g = gate_args(za, zb, n, h, w);
  EUNET_K_DISPATCH(k, gate_mid_fwd_kernel<KK><<<g.tiles, NT, 0, (hipStream_t)stream>>>(g, a, sc1, sh1, w2, b, st2));
  EUNET_LAUNCH_CHECK("gate_mid_fwd");
  return EUNET_OK;
}

int eunet_gate_out_fwd(const float* za, const float* zb, int n, int h, int w, int k, const float* b,
                       const float* sc2, const float* sh2, const eunet_act* f2, void* stream) {
  EUNET_REQUIRE(za && zb && b && sc2 && sh2 && f2 && f2->ptr && k >= 1 && k <= 3, "gate_out_fwd: bad args");
  EUNET_REQUIRE(f2->ctot == F2C && f2->coff == 0 && f2->c == 2 * k && f2->n == n && f2->h == h && f2->w == w,
                "gate_out_fwd: f2 must be [n,h,w,8] with c = 2K");
  GateArgs g = gate_args(za, zb, n, h, w);
  const unsigned gr = grid_for(g.P);
  if (f2->dtype == EUNET_BF16)
    EUNET_K_DISPATCH(k, gate_out_fwd_kernel<KK, bf16_t><<<gr, NT, 0, (hipStream_t)stream>>>(g, b, sc2, sh2,
                                                                                           (bf16_t*)f2->ptr));
  else
    EUNET_K_DISPATCH(k, gate_out_fwd_kernel<KK, float><<<gr, NT, 0, (hipStream_t)stream>>>(g, b, sc2, sh2,
                                                                                          (float*)f2->ptr));
  EUNET_LAUNCH_CHECK("gate_out_fwd");
  return EUNET_OK;
}

int eunet_fusion_out_fwd(const float* za, const float* zb, int k, const eunet_act* y3, const float* sc3,
                         const float* sh3, const float* w11, const float* b11, const float* b, const float* sc2,
                         const float* sh2, const float* wr, const float* br, float* out, void* stream) {
  EUNET_REQUIRE(za && zb && y3 && y3->ptr && sc3 && sh3 && w11 && b11 && b && sc2 && sh2 && wr && br && out &&
                    k >= 1 && k <= 3,
                "fusion_out_fwd: bad args");
  EUNET_REQUIRE(y3->c == 64 && y3->ctot == 64 && y3->coff == 0, "fusion_out_fwd: y3 must be [n,h,w,64]");
  GateArgs g = gate_args(za, zb, y3->n, y3->h, y3->w);
  const unsigned gr = grid_for(g.P);
  if (y3->dtype == EUNET_BF16)
    EUNET_K_DISPATCH(k, fusion_out_fwd_kernel<KK, bf16_t><<<gr, NT, 0, (hipStream_t)stream>>>(
                            g, (const bf16_t*)y3->ptr, sc3, sh3, w11, b11, b, sc2, sh2, wr, br, out));
  else
    EUNET_K_DISPATCH(k, fusion_out_fwd_kernel<KK, float><<<gr, NT, 0, (hipStream_t)stream>>>(
                            g, (const float*)y3->ptr, sc3, sh3, w11, b11, b, sc2, sh2, wr, br, out));
  EUNET_LAUNCH_CHECK("fusion_out_fwd");
  return EUNET_OK;
}

int eunet_fusion_out_bwd(const float* za, const float* zb, int n, int h, int w, int k, const float* gout,
                         const float* b, const float* sc2, const float* sh2, const float* wr, float* gz, float* gf2res,
                         float* part, void* stream) {
  EUNET_REQUIRE(za && zb && gout && b && sc2 && sh2 && wr && gz && gf2res && part && k >= 1 && k <= 3,
                "fusion_out_bwd: bad args");
  GateArgs g = gate_args(za, zb, n, h, w);
  EUNET_K_DISPATCH(k, fusion_out_bwd_kernel<KK><<<g.tiles, NT, 0, (hipStream_t)stream>>>(g, gout, b, sc2, sh2, wr,
                                                                                          gz, gf2res, part));
  EUNET_LAUNCH_CHECK("fusion_out_bwd");
  return EUNET_OK;
}

int eunet_gate_bwd1(const float* za, const float* zb, int k, const eunet_act* gf2conv, const float* gf2res,
                    const float* b, const float* mean2, const float* istd2, const float* gam2, const float* bet2,
                    float* gffd, float* gbhat, float* part, void* stream) {
  EUNET_REQUIRE(za && zb && gf2conv && gf2conv->ptr && gf2res && b && mean2 && istd2 && gam2 && bet2 && gffd &&
                    gbhat && part && k >= 1 && k <= 3,
                "gate_bwd1: bad args");
  EUNET_REQUIRE(gf2conv->ctot == F2C && gf2conv->coff == 0, "gate_bwd1: g_f2 must be [n,h,w,8]");
  GateArgs g = gate_args(za, zb, gf2conv->n, gf2conv->h, gf2conv->w);
  if (gf2conv->dtype == EUNET_BF16)
    EUNET_K_DISPATCH(k, gate_bwd1_kernel<KK, bf16_t><<<g.tiles, NT, 0, (hipStream_t)stream>>>(
                            g, (const bf16_t*)gf2conv->ptr, gf2res, b, mean2, istd2, gam2, bet2, gffd, gbhat, part));
  else
    EUNET_K_DISPATCH(k, gate_bwd1_kernel<KK, float><<<g.tiles, NT, 0, (hipStream_t)stream>>>(
                            g, (const float*)gf2conv->ptr, gf2res, b, mean2, istd2, gam2, bet2, gffd, gbhat, part));
  EUNET_LAUNCH_CHECK("gate_bwd1");
  return EUNET_OK;
}

int eunet_gate_bwd2(int n, int h, int w, int k, const float* gbhat, const float* b, const float* mean2,
                    const float* istd2, const float* gam2, const float* dbet2, const float* dgam2, const float* a,
                    const float* mean1, const float* istd1, const float* gam1, const float* bet1, const float* w2,
                    float* gabn, float* part, void* stream) {
  EUNET_REQUIRE(gbhat && b && mean2 && istd2 && gam2 && dbet2 && dgam2 && a && mean1 && istd1 && gam1 && bet1 &&
                    w2 && gabn && part && k >= 1 && k <= 3,
                "gate_bwd2: bad args");
  GateArgs g = gate_args(nullptr, nullptr, n, h, w);
  EUNET_K_DISPATCH(k, gate_bwd2_kernel<KK><<<g.tiles, NT, 0, (hipStream_t)stream>>>(
                          g, gbhat, b, mean2, istd2, gam2, dbet2, dgam2, a, mean1, istd1, gam1, bet1, w2, gabn, part));
  EUNET_LAUNCH_CHECK("gate_bwd2");
  return EUNET_OK;
}

int eunet_gate_bwd3(const float* za, const float* zb, int n, int h, int w, int k, const float* gabn, const float* a,
                    const float* mean1, const float* istd1, const float* gam1, const float* dbet1, const float* dgam1,
                    const float* w1, const float* gffd, const float* gaux_a, const float* gaux_b, float* gz_a,
                    float* gz_b, float* part, void* stream) {
  EUNET_REQUIRE(za && zb && gabn && a && mean1 && istd1 && gam1 && dbet1 && dgam1 && w1 && gffd && gz_a && gz_b &&
                    part && k >= 1 && k <= 3,
                "gate_bwd3: bad args");
  GateArgs g = gate_args(za, zb, n, h, w);
  const int tx = cdiv(w, GTW), ty = cdiv(h, GTH);
  EUNET_K_DISPATCH(k, gate_bwd3_kernel<KK><<<n * tx * ty, NT, 0, (hipStream_t)stream>>>(
                          g, gabn, a, mean1, istd1, gam1, dbet1, dgam1, w1, gffd, gaux_a, gaux_b, gz_a, gz_b, part,
                          tx, ty));
  EUNET_LAUNCH_CHECK("gate_bwd3");
  return EUNET_OK;
}

int eunet_dropout_affine(const float* scale, const float* shift, const float* keep, int n, int c, float p,
                         float* nscale, float* nshift, float* gscale, void* stream) {
  EUNET_REQUIRE(scale && shift && keep && nscale && nshift && n > 0 && c > 0 && p >= 0.f && p < 1.f,
                "dropout_affine: bad args");
  dropout_affine_kernel<<<cdiv(n * c, 256), 256, 0, (hipStream_t)stream>>>(scale, shift, keep, n, c, 1.f / (1.f - p),
                                                                           nscale, nshift, gscale);
  EUNET_LAUNCH_CHECK("dropout_affine");
  return EUNET_OK;
}

int eunet_consistency_tiles(int h, int w, int* tiles) {
  EUNET_REQUIRE(h > 0 && w > 0 && tiles, "consistency_tiles: bad args");
  *tiles = (int)(((long long)h * w + TP - 1) / TP);
  return EUNET_OK;
}

int eunet_consistency_fwd(const float* fused, const float* br0, const float* br1, int n, int k, int h, int w,
                          float c0, float c1, float* part, float* loss, void* stream) {
  EUNET_REQUIRE(fused && br0 && br1 && part && loss && n > 0 && k >= 1 && k <= 3, "consistency_fwd: bad args");
  const long long hw = (long long)h * w;
  const int tiles = (int)((hw + TP - 1) / TP);
  dim3 grid(tiles, n);
  EUNET_K_DISPATCH(k, consistency_fwd_kernel<KK><<<grid, NT, 0, (hipStream_t)stream>>>(fused, br0, br1, hw, part));
  consistency_finalize_kernel<<<1, 64, 0, (hipStream_t)stream>>>(part, n, tiles, c0, c1, (long long)k * hw, loss);
  EUNET_LAUNCH_CHECK("consistency_fwd");
  return EUNET_OK;
}

int eunet_consistency_bwd(const float* fused, const float* br0, const float* br1, int n, int k, int h, int w,
                          float c0, float c1, const float* gloss, float* gfused, float* g0, float* g1, void* stream) {
  EUNET_REQUIRE(fused && br0 && br1 && gloss && gfused && g0 && g1 && n > 0 && k >= 1 && k <= 3,
                "consistency_bwd: bad args");
  const long long hw = (long long)h * w, total = (long long)n * hw;
  const double denom = (double)n * k * hw;
  const float s0 = (float)(2.0 * c0 / denom), s1 = (float)(2.0 * c1 / denom);
  EUNET_K_DISPATCH(k, consistency_bwd_kernel<KK><<<grid_for(total), NT, 0, (hipStream_t)stream>>>(
                          fused, br0, br1, hw, total, s0, s1, gloss, gfused, g0, g1));
  EUNET_LAUNCH_CHECK("consistency_bwd");
  return EUNET_OK;
}

}  // extern "C"
