// Memory-bound kernels of the hot path (HBM-bound; NHWC, 16-byte vectors):
//   enc1.0 direct conv (Cin <= 4), BatchNorm statistics finalisation,
//   BN+ReLU fused into MaxPool / bilinear Upsample / dec1 1x1 consumers,
//   and their backward counterparts.
// Reference sites: models.py:203 (enc1.0), 214-215 (pool, upsample),
// 212/236 (dec1), 220-224 (BN+ReLU), autograd of all of them.
#include "common.h"

#include <algorithm>

EUNET_DEBUG_UNIT(bnpool)

namespace {

constexpr int NT = 256;
constexpr int STH = 8, STW = 32;  // wgrad tile of conv_small
constexpr int SFH = 16;           // forward tile SFH x STW = conv3x3 forward tiling (BN stats rows agree)
constexpr int SCI = 8;            // max input channels of the direct conv (enc1.0: in_ch; fusion_head.0: 2K)
constexpr int SJT = (SCI * 9 + 15) / 16;  // 16-column im2col MFMA tiles of its wgrad (5)

bool act_ok(const eunet_act* a) {
  return a && a->ptr && a->n > 0 && a->h > 0 && a->w > 0 && a->c > 0 && a->coff >= 0 &&
         a->coff + a->c <= a->ctot && (a->dtype == EUNET_F32 || a->dtype == EUNET_BF16);
}
int e16(int dt) { return dt == EUNET_BF16 ? 8 : 4; }
bool vec_ok(const eunet_act* a) {
  const int E = e16(a->dtype);
  return a->c % E == 0 && a->ctot % E == 0 && a->coff % E == 0;
}

// ---------------------------------------------------------------------------
// enc1.0 / fusion_head.0: direct 3x3 conv for Cin <= 8, 64 output channels per block.y
// ---------------------------------------------------------------------------
struct SmallArgs {
  const void* x; int N, H, W, xct, xco, cin;
  const float* w; const float* b;
  void* y; int yct, yco, cout;
  float* stats; int tx, ty, ntiles;
};

// 8 lanes per pixel (lane group g = lane & 7 owns output channels co0+8g..+7),
// 32 pixels per pass = one output row of the 16x32 tile; per-thread Welford over
// its 8 pixels, Chan-combined across lanes and waves (no transposes)
// C1: one input channel (enc1.0 of the 1-channel configurations) -- the lane's 9 x 8 weights
// live in registers instead of being re-read from LDS for every pixel.
template <typename T, bool C1>
__global__ __launch_bounds__(NT) void conv_small_fwd_kernel(SmallArgs a) {
  __shared__ float xs[(SFH + 2) * (STW + 2) * SCI];
  __shared__ __attribute__((aligned(16))) float wsm[SCI * 9 * 64];  // [ci*9+t][64 co]
  __shared__ float wn_s[4], wm_s[4][64], wq_s[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane & 7, ps = tid >> 3;
  const int tile = blockIdx.x, tpi = a.tx * a.ty;
  const int n = tile / tpi, trem = tile - n * tpi;
  const int y0 = (trem / a.tx) * SFH, x0 = (trem % a.tx) * STW;
  const int co0 = blockIdx.y * 64;
  const int cin = a.cin;
  for (int i = tid; i < (SFH + 2) * (STW + 2) * cin; i += NT) {
    const int hp = i / cin, ci = i - hp * cin;
    const int hy = hp / (STW + 2), hx = hp - hy * (STW + 2);
    const int yy = y0 + hy - 1, xx = x0 + hx - 1;
    float v = 0.f;
    if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
      v = Elem<T>::ld((const T*)a.x + ((long long)(n * a.H + yy) * a.W + xx) * a.xct + a.xco + ci);
    xs[hp * SCI + ci] = v;
  }
  for (int i = tid; i < 64 * cin * 9; i += NT) {
    const int co = i / (cin * 9), r = i - co * cin * 9;
    wsm[r * 64 + co] = (co0 + co < a.cout) ? a.w[(long long)(co0 + co) * cin * 9 + r] : 0.f;
  }
  __syncthreads();
  float wr[C1 ? 9 : 1][8];
  if constexpr (C1)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) wr[t][e] = wsm[t * 64 + 8 * g + e];
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = (a.b != nullptr && co0 + 8 * g + e < a.cout) ? a.b[co0 + 8 * g + e] : 0.f;
  float cnt = 0.f, mean[8], m2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { mean[e] = 0.f; m2[e] = 0.f; }
  constexpr int E = Vec16<T>::N;
  // whole 16-byte stores for every lane whose 8 channels exist (per lane: the 96-channel layers' second
  // co-block holds 32; element stores there ran enc1.0 at 2.1 TB/s at configs[4])
  const bool full = (co0 + 8 * g + 8 <= a.cout) && ((a.yct | a.yco) % E) == 0;
  for (int pass = 0; pass < SFH; ++pass) {
    const int px = pass * 32 + ps;
    const int r = px / STW, c = px - r * STW;
    const int yy = y0 + r, xx = x0 + c;
    if (yy >= a.H || xx >= a.W) continue;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = bias[e];
    if constexpr (C1) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t - ky * 3;
        const float v = xs[((r + ky) * (STW + 2) + c + kx) * SCI];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(wr[t][e], v, acc[e]);
      }
    }
    for (int ci = 0; ci < (C1 ? 0 : cin); ++ci) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t - ky * 3;
        const float v = xs[((r + ky) * (STW + 2) + c + kx) * SCI + ci];
        const float4 w0 = *(const float4*)(wsm + (ci * 9 + t) * 64 + 8 * g);
        const float4 w1 = *(const float4*)(wsm + (ci * 9 + t) * 64 + 8 * g + 4);
        acc[0] = fmaf(w0.x, v, acc[0]); acc[1] = fmaf(w0.y, v, acc[1]);
        acc[2] = fmaf(w0.z, v, acc[2]); acc[3] = fmaf(w0.w, v, acc[3]);
        acc[4] = fmaf(w1.x, v, acc[4]); acc[5] = fmaf(w1.y, v, acc[5]);
        acc[6] = fmaf(w1.z, v, acc[6]); acc[7] = fmaf(w1.w, v, acc[7]);
      }
    }
    T* yp = (T*)a.y + ((long long)(n * a.H + yy) * a.W + xx) * a.yct + a.yco + co0 + 8 * g;
    if (full) {  // (non-temporal: y is read back by the next conv well after it has left L2)
      __builtin_nontemporal_store(__builtin_bit_cast(u32x4, Vec16<T>::pack(acc)), (u32x4*)yp);
      if constexpr (E == 4) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, Vec16<T>::pack(acc + 4)), (u32x4*)(yp + 4));
    } else {
      for (int e = 0; e < 8; ++e)
        if (co0 + 8 * g + e < a.cout) Elem<T>::st(yp + e, acc[e]);
    }
    cnt += 1.f;
    const float inv = 1.f / cnt;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = acc[e] - mean[e];
      mean[e] = fmaf(d, inv, mean[e]);
      m2[e] = fmaf(d, acc[e] - mean[e], m2[e]);
    }
  }
  if (a.stats == nullptr) return;
#pragma unroll
  for (int off = 8; off <= 32; off <<= 1) {
    const float nb = __shfl_xor(cnt, off, 64);
    const float nt = cnt + nb;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float mb = __shfl_xor(mean[e], off, 64), qb = __shfl_xor(m2[e], off, 64);
      const float d = mb - mean[e];
      if (nt > 0.f) {
        mean[e] += d * nb / nt;
        m2[e] += qb + d * d * cnt * nb / nt;
      }
    }
    cnt = nt;
  }
  if (lane < 8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      wm_s[wv][8 * g + e] = mean[e];
      wq_s[wv][8 * g + e] = m2[e];
    }
    if (lane == 0) wn_s[wv] = cnt;
  }
  __syncthreads();
  if (tid < 64 && co0 + tid < a.cout) {
    double bn = 0.0, bm = 0.0, bq = 0.0;
    for (int w = 0; w < 4; ++w) {
      const double nb = wn_s[w];
      if (nb <= 0.0) continue;
      const double d = (double)wm_s[w][tid] - bm, nt = bn + nb;
      bm += d * nb / nt;
      bq += (double)wq_s[w][tid] + d * d * bn * nb / nt;
      bn = nt;
    }
    a.stats[((long long)tile * 2 + 0) * a.cout + co0 + tid] = (float)(bm * bn);
    a.stats[((long long)tile * 2 + 1) * a.cout + co0 + tid] = (float)bq;
    if (blockIdx.y == 0 && tid == 0) a.stats[(long long)2 * a.cout * a.ntiles + tile] = (float)bn;
  }
}

struct SmallWgArgs {
  const void* x; int N, H, W, xct, xco, cin;
  const void* dy; int dct, dco, cout;
  float* dw; float* db;
  int tx, ty, ntiles, per_split;
};

// direct-conv wgrad as MFMA: dW[co][ci*9+t] = sum_p dY[p][co] im2col(x)[p][ci*9+t];
// im2col (cin*9 columns padded to njt*16 <= 80) and the dY tile are staged in LDS per 8x32 tile
template <typename T, int CI>  // CI = max input channels of the instance (4: enc1.0, 8: fusion_head.0)
__global__ __launch_bounds__(NT) void conv_small_wgrad_kernel(SmallWgArgs a) {
  constexpr int SCI = CI, SJT = (CI * 9 + 15) / 16;  // LDS sized per instance (occupancy)
  constexpr int E = Vec16<T>::N;
  __shared__ __attribute__((aligned(16))) float xs[(STH + 2) * (STW + 2) * SCI];
  __shared__ __attribute__((aligned(16))) T gs[STH * STW * 64];         // dY tile [256 px][64 co]
  __shared__ __attribute__((aligned(16))) T cs[STH * STW * SJT * 16];  // im2col [256 px][icw]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int split = blockIdx.x, co0 = blockIdx.y * 64;
  const int t_begin = split * a.per_split, t_end = min(a.ntiles, t_begin + a.per_split);
  const int tpi = a.tx * a.ty, cin = a.cin;
  const int njt = (cin * 9 + 15) / 16, icw = njt * 16;  // im2col columns (LDS row stride)
  f32x4 acc[SJT];
#pragma unroll
  for (int j = 0; j < SJT; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbv[8];  // bias gradient: channels 8 (tid & 7) .. +7 over pixels (tid >> 3) + 32 i
#pragma unroll
  for (int e = 0; e < 8; ++e) dbv[e] = 0.f;
  // The next tile's x halo and dY tile are loaded into registers while this tile's MFMAs run
  // (one exposed global round trip per block instead of one per tile).
  constexpr int XI = ((STH + 2) * (STW + 2) * SCI + NT - 1) / NT, DI = STH * STW * 64 / E / NT;
  static_assert(STH * STW * 64 / E % NT == 0, "dY units per thread");
  T rx[XI];  // raw: a conversion inside the bounds branch would make each prefetch load wait there
  uint4 rd[DI];
  auto load_tile = [&](int tile) {
    const int n = tile / tpi, trem = tile - n * tpi;
    const int y0 = (trem / a.tx) * STH, x0 = (trem % a.tx) * STW;
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + k * NT;
      const int hp = i / cin, ci = i - hp * cin;
      const int hy = hp / (STW + 2), hx = hp - hy * (STW + 2);
      const int yy = y0 + hy - 1, xx = x0 + hx - 1;
      rx[k] = (i < (STH + 2) * (STW + 2) * cin && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
                  ? ((const T*)a.x)[((long long)(n * a.H + yy) * a.W + xx) * a.xct + a.xco + ci]
                  : T(0);
    }
#pragma unroll
    for (int k = 0; k < DI; ++k) {
      const int id = tid + k * NT;
      const int px = id / (64 / E), u = id - px * (64 / E);
      const int r = px / STW, c = px - r * STW;
      const int yy = y0 + r, xx = x0 + c, co = co0 + u * E;
      rd[k] = (yy < a.H && xx < a.W && co < a.cout)
                  ? *(const uint4*)((const T*)a.dy + ((long long)(n * a.H + yy) * a.W + xx) * a.dct + a.dco + co)
                  : make_uint4(0, 0, 0, 0);
    }
  };
  if (t_begin < t_end) load_tile(t_begin);
  for (int tile = t_begin; tile < t_end; ++tile) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + k * NT;
      if (i < (STH + 2) * (STW + 2) * cin) {
        const int hp = i / cin, ci = i - hp * cin;
        xs[hp * SCI + ci] = Elem<T>::ld(&rx[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < DI; ++k) {
      const int id = tid + k * NT;
      const int px = id / (64 / E), u = id - px * (64 / E);
      *(uint4*)(gs + px * 64 + u * E) = rd[k];
      if constexpr (E == 8) {  // bf16: the bias gradient from the staged registers -- unit id holds channels
                               // 8 (tid & 7) .. + 7 of pixel (tid >> 3) + 32 k, the dbv mapping below
        float f[E];
        Vec16<T>::unpack(rd[k], f);
#pragma unroll
        for (int e = 0; e < E; ++e) dbv[e] += f[e];
      }
    }
    if (tile + 1 < t_end) load_tile(tile + 1);
    __syncthreads();
    if constexpr (E != 8) {  // fp32: the thread's 8 channels span two units -- from the staged tile
#pragma unroll
      for (int i = 0; i < STH * STW / 32; ++i) {  // independent 16-B reads, no wait per element
        const T* src = gs + ((tid >> 3) + 32 * i) * 64 + (tid & 7) * 8;
#pragma unroll
        for (int h = 0; h < 8 / E; ++h) {
          float f[E];
          Vec16<T>::unpack(*(const uint4*)(src + h * E), f);
#pragma unroll
          for (int e = 0; e < E; ++e) dbv[h * E + e] += f[e];
        }
      }
    }
    {  // the im2col row of pixel px = tid: column j = ci * 9 + t, zero past cin * 9 (to icw).  Nine 16-byte
       // reads of the halo (a tap's SCI channels at once) and icw / E 16-byte writes per thread (one element
       // per read / write with per-element index arithmetic before: VALU-bound)
      static_assert(STH * STW == NT, "one im2col row per thread");
      const int px = tid, r = px / STW, c = px % STW;
      float v[CI * 9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t - ky * 3;
        const float* src = xs + ((r + ky) * (STW + 2) + c + kx) * SCI;
#pragma unroll
        for (int qq = 0; qq < CI / 4; ++qq) {
          const f32x4 f = *(const f32x4*)(src + 4 * qq);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[(4 * qq + e) * 9 + t] = 4 * qq + e < cin ? f[e] : 0.f;  // (past cin: unstaged)
        }
      }
      T* const dst = cs + px * icw;
#pragma unroll
      for (int u = 0; u < SJT * 16 / E; ++u) {
        if (u * E >= icw) break;
        float f[E];
#pragma unroll
        for (int e = 0; e < E; ++e) f[e] = u * E + e < CI * 9 ? v[u * E + e] : 0.f;
        *(uint4*)(dst + u * E) = Vec16<T>::pack(f);
      }
    }
    __syncthreads();
    const int cw = wv * 16;
    if constexpr (sizeof(T) == 2) {
      const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
      for (int ks = 0; ks < STH * STW / 32; ++ks) {
        const int pxa = ks * 32 + 8 * g + q4;
        const s16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, (char*)gs + (pxa * 64 + cw + 4 * p4) * 2));
        const s16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, (char*)gs + ((pxa + 4) * 64 + cw + 4 * p4) * 2));
        const bf16x8 af = cat_bf16x4(alo, ahi);
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt) {
          if (jt >= njt) break;
          const s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, (char*)cs + (pxa * icw + jt * 16 + 4 * p4) * 2));
          const s16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, (char*)cs + ((pxa + 4) * icw + jt * 16 + 4 * p4) * 2));
          acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, cat_bf16x4(blo, bhi), acc[jt], 0, 0, 0);
        }
      }
    } else {
      const int kq = lane >> 4, i = lane & 15;
      for (int ks = 0; ks < STH * STW / 4; ++ks) {
        const int px = ks * 4 + kq;
        const float av = ((const float*)gs)[px * 64 + cw + i];
#pragma unroll
        for (int jt = 0; jt < SJT; ++jt) {
          if (jt >= njt) break;
          acc[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, ((const float*)cs)[px * icw + jt * 16 + i], acc[jt], 0, 0, 0);
        }
      }
    }
  }
  float* out = a.dw + (long long)split * a.cout * 9 * cin;
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int jt = 0; jt < SJT; ++jt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co0 + wv * 16 + g * 4 + e, j = jt * 16 + li;
      if (co < a.cout && j < cin * 9) {
        const int ci = j / 9, t = j - ci * 9;
        out[((long long)co * 9 + t) * cin + ci] = acc[jt][e];
      }
    }
  __syncthreads();
  float(*dbs)[64] = (float(*)[64])gs;  // [32 pixel groups][64 co] over the finished dY tile
#pragma unroll
  for (int e = 0; e < 8; ++e) dbs[tid >> 3][(tid & 7) * 8 + e] = dbv[e];
  __syncthreads();
  if (a.db != nullptr && tid < 64 && co0 + tid < a.cout) {
    float t = 0.f;
    for (int r = 0; r < 32; ++r) t += dbs[r][tid];
    a.db[(long long)split * a.cout + co0 + tid] = t;
  }
}

// ---------------------------------------------------------------------------
// BatchNorm statistics: Chan-combine per-tile (sum, M2, count) in fp64
// ---------------------------------------------------------------------------
constexpr int FNT = 1024;  // threads per channel block of bn_finalize (8 tiles per thread at 1024^2)
__global__ __launch_bounds__(FNT) void bn_finalize_kernel(const float* st, int tiles, int C, const float* gamma,
                                                         const float* beta, float eps, float mom, float* rm,
                                                         float* rv, float* mean_o, float* invstd_o, float* scale_o,
                                                         float* shift_o, long long* nbt, const double* guard) {
  __shared__ double shn[FNT], shm[FNT], shq[FNT];
  const int c = blockIdx.x, tid = threadIdx.x;
  const float* cnt = st + (long long)2 * C * tiles;
  // one pass: each thread Chan-merges its tiles (count, mean, M2) online, then a fixed-order tree
  double n = 0.0, mean = 0.0, m2 = 0.0;
  auto merge = [](double& n, double& mean, double& m2, double nb, double mb, double qb) {
    const double nt = n + nb;
    if (nb <= 0.0) return;
    const double d = mb - mean;
    mean += d * (nb / nt);
    m2 += qb + d * d * (n * nb / nt);
    n = nt;
  };
  // the loads of FB tiles are issued before their merges (same merge order, bit-identical).  At 64
  // channels x 16k tiles the launch (~21 us) is bound by its strided reads on 64 CUs (each wave
  // load touches 64 lines); a two-launch form over channel-coalesced tile slices measured no faster
  // per step (the extra launch costs what it saves, profiles/r04_ab.txt)
  constexpr int FB = 8;
  for (int t0 = tid; t0 < tiles; t0 += FB * FNT) {
    float vn[FB], vs[FB], vq[FB];
#pragma unroll
    for (int i = 0; i < FB; ++i) {
      const bool in = t0 + i * FNT < tiles;
      const long long ti = min(t0 + i * FNT, tiles - 1);  // unconditional loads, then the select
      const float a = cnt[ti], b = st[(ti * 2) * C + c], q = st[(ti * 2 + 1) * C + c];
      vn[i] = in ? a : 0.f;
      vs[i] = in ? b : 0.f;
      vq[i] = in ? q : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FB; ++i) {
      const double nb = (double)vn[i];
      if (nb > 0.0) merge(n, mean, m2, nb, (double)vs[i] / nb, (double)vq[i]);
    }
  }
  shn[tid] = n; shm[tid] = mean; shq[tid] = m2;
  __syncthreads();
  for (int o = FNT / 2; o > 0; o >>= 1) {
    if (tid < o) {
      double a_n = shn[tid], a_m = shm[tid], a_q = shq[tid];
      merge(a_n, a_m, a_q, shn[tid + o], shm[tid + o], shq[tid + o]);
      shn[tid] = a_n; shm[tid] = a_m; shq[tid] = a_q;
    }
    __syncthreads();
  }
  n = shn[0]; mean = shm[0]; m2 = shq[0];
  // the running statistics stay as they are while the update guard is raised (eunet_set_update_guard)
  const bool keep = guard != nullptr && *guard != 0.0;
  if (keep) { rm = nullptr; rv = nullptr; nbt = nullptr; }
  if (tid == 0 && c == 0 && nbt != nullptr) *nbt += 1;  // BatchNorm2d.num_batches_tracked
  if (tid == 0) {
    const double var_b = m2 / n;
    const double var_u = n > 1.0 ? m2 / (n - 1.0) : var_b;
    const double istd = 1.0 / sqrt(var_b + (double)eps);
    const double sc = (double)gamma[c] * istd;
    if (mean_o) mean_o[c] = (float)mean;
    if (invstd_o) invstd_o[c] = (float)istd;
    if (scale_o) scale_o[c] = (float)sc;
    if (shift_o) shift_o[c] = (float)((double)beta[c] - mean * sc);
    if (rm) rm[c] = (float)((1.0 - mom) * (double)rm[c] + mom * mean);
    if (rv) rv[c] = (float)((1.0 - mom) * (double)rv[c] + mom * var_u);
  }
}

__global__ void bn_eval_affine_kernel(int C, const float* g, const float* b, const float* rm, const float* rv,
                                      float eps, float* sc, float* sh) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float s = g[c] / sqrtf(rv[c] + eps);
  sc[c] = s;
  sh[c] = b[c] - rm[c] * s;
}

// ---------------------------------------------------------------------------
// BN+ReLU -> (skip activation) + MaxPool2d(2)
// ---------------------------------------------------------------------------
template <typename T>
__global__ void bnrelu_pool_kernel(const T* y, int N, int H, int W, int C, int yct, int yco, const float* sc,
                                   const float* sh, T* act, int act_ct, int act_co, T* pool, int pct, int pco) {
  constexpr int E = Vec16<T>::N;
  const int U = C / E, Ho = H / 2, Wo = W / 2;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * Ho * Wo * U;
  if (id >= total) return;
  const int u = (int)(id % U);
  long long p = id / U;
  const int xo = (int)(p % Wo); p /= Wo;
  const int yo = (int)(p % Ho);
  const int n = (int)(p / Ho);
  const int c = u * E;
  float s[E], t[E], m[E];
#pragma unroll
  for (int j = 0; j < E; ++j) { s[j] = sc[c + j]; t[j] = sh[c + j]; m[j] = -INFINITY; }
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const long long pix = (long long)(n * H + 2 * yo + dy) * W + 2 * xo + dx;
      float f[E];
      // y is read once here (disjoint windows) and the skip activation is next read by the decoder, long
      // after: both non-temporal; the pooled output, read by the next encoder conv, is cached normally
      Vec16<T>::unpack(__builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4*)(y + pix * yct + yco + c))), f);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        f[j] = fmaxf(fmaf(f[j], s[j], t[j]), 0.f);
        m[j] = fmaxf(m[j], f[j]);
      }
      if (act != nullptr)
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, Vec16<T>::pack(f)), (u32x4*)(act + pix * act_ct + act_co + c));
    }
  const long long po = (long long)(n * Ho + yo) * Wo + xo;
  *(uint4*)(pool + po * pct + pco + c) = Vec16<T>::pack(m);
}

// z = relu(y * scale + shift), one 16-byte channel unit per thread and step: the activation of a
// DoubleConv's first BN+ReLU (models.py:219-222), materialised once so the second conv's forward
// and weight gradient read it without re-applying the transform per halo pixel
template <typename T>
__global__ __launch_bounds__(256) void bnrelu_kernel(const T* y, long long P, int C, int yct, int yco, const float* sc,
                                                     const float* sh, T* out, int oct, int oco) {
  constexpr int E = Vec16<T>::N;
  const int U = C / E;
  const long long total = P * U;
  for (long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x; id < total;
       id += (long long)gridDim.x * blockDim.x) {
    const long long p = id / U;
    const int c = (int)(id - p * U) * E;
    float f[E];
    Vec16<T>::unpack(*(const uint4*)(y + p * yct + yco + c), f);
#pragma unroll
    for (int j = 0; j < E; ++j) f[j] = fmaxf(fmaf(f[j], sc[c + j], sh[c + j]), 0.f);
    *(uint4*)(out + p * oct + oco + c) = Vec16<T>::pack(f);
  }
}

// BN+ReLU -> bilinear x2 upsample (align_corners=False), PyTorch's weights (0.25 / 0.75, edge rows and columns
// weighted 1 / 0 exactly as upsample_bilinear2d's clamped source index), as a row sweep: a thread owns two
// adjacent low-res columns (j0, j0 + 1) x one 16-byte channel unit over rpt low-res rows (8, or 4 for small grids)
// and keeps the x-interpolated rows i-1, i, i+1 in registers, so each low-res row is loaded and transformed once
// per sweep (4 loads per row; the per-pixel-pair form loaded a 3 x 4 neighbourhood, 12, for every pair: 534 vs
// 459 us over the bench's three launches, bit-identical, profiles/r05_ab.txt), with the next row's loads in
// flight while the current outputs are formed.
template <typename T>
__global__ __launch_bounds__(256) void bnrelu_up_rows_kernel(const T* y, int N, int h, int w, int C, int yct, int yco,
                                                             const float* sc, const float* sh, T* out, int oct,
                                                             int oco, int rpt) {
  constexpr int E = Vec16<T>::N, E2 = E / 2;
  const int U = C / E, H2 = 2 * h, W2 = 2 * w, wb = (w + 1) / 2, hb = (h + rpt - 1) / rpt;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)N * hb * wb * U;
  if (id >= total) return;
  const int u = (int)(id % U);
  long long p = id / U;
  const int jb = (int)(p % wb); p /= wb;
  const int ib = (int)(p % hb);
  const int n = (int)(p / hb);
  const int c = u * E, j0 = 2 * jb, i0 = ib * rpt, i1 = min(i0 + rpt, h);
  const bool two = j0 + 1 < w;
  f32x2 s2[E2], t2[E2];
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    s2[e] = (f32x2){sc[c + 2 * e], sc[c + 2 * e + 1]};
    t2[e] = (f32x2){sh[c + 2 * e], sh[c + 2 * e + 1]};
  }
  const int cs[4] = {max(j0 - 1, 0), j0, min(j0 + 1, w - 1), min(j0 + 2, w - 1)};
  const f32x2 q1 = {0.25f, 0.25f}, q3 = {0.75f, 0.75f};
  const float wxa = j0 > 0 ? 0.25f : 1.f, wxb = j0 > 0 ? 0.75f : 0.f;
  const f32x2 wxa2 = {wxa, wxa}, wxb2 = {wxb, wxb};
  const T* yb = y + (long long)n * h * w * yct + yco + c;
  auto load = [&](int r, uint4 (&raw)[4]) {
#pragma unroll
    for (int b = 0; b < 4; ++b) raw[b] = *(const uint4*)(yb + ((long long)r * w + cs[b]) * yct);
  };
  // BN + ReLU of the four loaded columns, then the x interpolation: output columns 2 j0 .. 2 j0 + 3
  auto xrow = [&](const uint4 (&raw)[4], f32x2 (&xr)[4][E2]) {
    f32x2 v[4][E2];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      float f[E];
      Vec16<T>::unpack(raw[b], f);
#pragma unroll
      for (int e = 0; e < E2; ++e) {
        const f32x2 r = __builtin_elementwise_fma((f32x2){f[2 * e], f[2 * e + 1]}, s2[e], t2[e]);
        v[b][e] = (f32x2){fmaxf(r.x, 0.f), fmaxf(r.y, 0.f)};
      }
    }
#pragma unroll
    for (int e = 0; e < E2; ++e) {
      xr[0][e] = __builtin_elementwise_fma(wxb2, v[1][e], wxa2 * (j0 > 0 ? v[0][e] : v[1][e]));
      xr[1][e] = __builtin_elementwise_fma(q1, v[2][e], q3 * v[1][e]);
      xr[2][e] = __builtin_elementwise_fma(q3, v[2][e], q1 * v[1][e]);
      xr[3][e] = __builtin_elementwise_fma(q1, v[3][e], q3 * v[2][e]);
    }
  };
  auto store = [&](int orow, const f32x2 (&o)[4][E2]) {
    const long long po = (long long)(n * H2 + orow) * W2 + 2 * j0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (b >= 2 && !two) break;
      float f[E];
#pragma unroll
      for (int e = 0; e < E2; ++e) { f[2 * e] = o[b][e].x; f[2 * e + 1] = o[b][e].y; }
      __builtin_nontemporal_store(__builtin_bit_cast(u32x4, Vec16<T>::pack(f)), (u32x4*)(out + (po + b) * oct + oco + c));
    }
  };
  f32x2 xp[4][E2], xc[4][E2], xn[4][E2];
  uint4 raw[4];
  load(max(i0 - 1, 0), raw);
  xrow(raw, xp);
  load(i0, raw);
  xrow(raw, xc);
  load(min(i0 + 1, h - 1), raw);
#pragma unroll 1
  for (int i = i0; i < i1; ++i) {
    // output row 2i: rows (i-1, i) weights (0.25, 0.75), or row i with weights (1, 0) at i = 0
    const float wya = i > 0 ? 0.25f : 1.f, wyb = i > 0 ? 0.75f : 0.f;
    const f32x2 wya2 = {wya, wya}, wyb2 = {wyb, wyb};
    f32x2 o[4][E2];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < E2; ++e)
        o[b][e] = __builtin_elementwise_fma(wyb2, xc[b][e], wya2 * (i > 0 ? xp[b][e] : xc[b][e]));
    store(2 * i, o);
    xrow(raw, xn);  // row min(i + 1, h - 1)
    if (i + 1 < i1) load(min(i + 2, h - 1), raw);
    // output row 2i + 1: rows (i, i+1) weights (0.75, 0.25), i+1 clamped
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < E2; ++e) o[b][e] = __builtin_elementwise_fma(q1, xn[b][e], q3 * xc[b][e]);
    store(2 * i + 1, o);
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < E2; ++e) { xp[b][e] = xc[b][e]; xc[b][e] = xn[b][e]; }
  }
}

// BN+ReLU -> 1x1 conv (C -> K <= 3), fp32 NHWC output
// 8 lanes per pixel: lane g reads the 16-byte channel groups 8g (+64) of its pixel, so a
// wave reads 8 whole pixel rows (coalesced); BN scale/shift and W live in registers.  A block
// step covers C1X_PX x 32 pixels with all C1X_PX loads issued before any use (memory-level
// parallelism: one dependent load per step ran this HBM-bound kernel at 2.2 TB/s); the 8-lane
// sums are DPP (quad butterflies + half-row mirror), not LDS shuffles.  C <= 128, C % 8 == 0.
constexpr int C1X_PX = 4;
__device__ __forceinline__ float oct8_sum(float v) {  // sum over the 8 lanes of an aligned octet
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // quad [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // quad [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)); // row_half_mirror
  return v;
}

template <typename T>
__global__ __launch_bounds__(256) void bnrelu_conv1x1_kernel(const T* y, long long P, int C, int yct, int yco,
                                                             const float* sc, const float* sh, const float* w,
                                                             const float* b, int K, float* z) {
  constexpr int E = Vec16<T>::N;
  const int g = threadIdx.x & 7;
  const bool two = C > 64;
  float s8[2][8], t8[2][8], w8[2][3][8];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 64 * j + 8 * g + e;
      const bool ok = c < C;
      s8[j][e] = ok ? sc[c] : 0.f;
      t8[j][e] = ok ? sh[c] : 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) w8[j][k][e] = (ok && k < K) ? w[k * C + c] : 0.f;
    }
  const float b0 = b[0], b1 = K > 1 ? b[1] : 0.f, b2 = K > 2 ? b[2] : 0.f;
  const bool cg0 = 8 * g < C, cg1 = two && 64 + 8 * g < C;
  const long long step = (long long)gridDim.x * 32 * C1X_PX;
  for (long long p0 = (long long)blockIdx.x * 32 * C1X_PX + (threadIdx.x >> 3); p0 < P; p0 += step) {
    uint4 raw[C1X_PX][2][E == 4 ? 2 : 1];
#pragma unroll
    for (int u = 0; u < C1X_PX; ++u) {
      const long long p = p0 + 32 * u;
      const bool pok = p < P;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = pok && (j == 0 ? cg0 : cg1);
        const T* src = y + (ok ? p * yct + yco + 64 * j + 8 * g : 0);
        raw[u][j][0] = ok ? *(const uint4*)src : make_uint4(0, 0, 0, 0);
        if constexpr (E == 4) raw[u][j][1] = ok ? *(const uint4*)(src + 4) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < C1X_PX; ++u) {
      float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (j == 1 && !two) break;
        float f[8];
        Vec16<T>::unpack(raw[u][j][0], f);
        if constexpr (E == 4) Vec16<T>::unpack(raw[u][j][E == 4 ? 1 : 0], f + 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = fmaxf(fmaf(f[e], s8[j][e], t8[j][e]), 0.f);
#pragma unroll
          for (int k = 0; k < 3; ++k) acc[k] = fmaf(w8[j][k][e], a, acc[k]);
        }
      }
      const long long p = p0 + 32 * u;
      const float z0 = oct8_sum(acc[0]) + b0;
      if (K == 1) {
        if (g == 0 && p < P) z[p] = z0;
      } else {
        const float z1 = oct8_sum(acc[1]) + b1;
        if (K == 2) {
          if (g == 0 && p < P) *(float2*)(z + p * 2) = make_float2(z0, z1);
        } else {
          const float z2 = oct8_sum(acc[2]) + b2;
          if (g == 0 && p < P) {
            z[p * 3] = z0;
            z[p * 3 + 1] = z1;
            z[p * 3 + 2] = z2;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------
// pixels per reduction tile: ~2048 tiles (whole-chip parallelism even for the 128^2 x 512-ch
// levels), 64..1024 pixels each
long long bwd_pix(long long P) {
  long long pix = ((P / 2048 + 63) / 64) * 64;
  return pix < 64 ? 64 : (pix > 1024 ? 1024 : pix);
}

template <typename T>
__global__ __launch_bounds__(NT) void bn_bwd_reduce_kernel(const T* g, int gct, int gco, const T* y, int yct, int yco,
                                                           long long P, int C, const float* mean, const float* istd,
                                                           const float* scale, const float* shift, float* part,
                                                           int tpix) {
  constexpr int E = Vec16<T>::N;
  __shared__ float red[2][NT][E];
  const int U = C / E;
  const int tid = threadIdx.x;
  const int slots = NT / U;  // U <= NT required (C <= 2048 bf16)
  const int u = tid % U, sl = tid / U;
  const int c = u * E;
  float s1[E], s2[E], mu[E], is[E], ga[E], be[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    s1[j] = 0.f; s2[j] = 0.f;
    if (sl < slots) { mu[j] = mean[c + j]; is[j] = istd[c + j]; ga[j] = scale[c + j]; be[j] = shift[c + j]; }
  }
  const long long p0 = (long long)blockIdx.x * tpix;
  const long long p1 = min(P, p0 + tpix);
  if (sl < slots) {
    for (long long p = p0 + sl; p < p1; p += slots) {
      float gf[E], yf[E];
      Vec16<T>::unpack(*(const uint4*)(g + p * gct + gco + c), gf);
      Vec16<T>::unpack(*(const uint4*)(y + p * yct + yco + c), yf);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        const float xh = (yf[j] - mu[j]) * is[j];
        const float gg = (fmaf(yf[j], ga[j], be[j]) > 0.f) ? gf[j] : 0.f;  // the forward's ReLU mask
        s1[j] += gg;
        s2[j] = fmaf(gg, xh, s2[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < E; ++j) { red[0][tid][j] = s1[j]; red[1][tid][j] = s2[j]; }
  __syncthreads();
  if (sl == 0) {
    for (int k = 1; k < slots; ++k) {
#pragma unroll
      for (int j = 0; j < E; ++j) { s1[j] += red[0][k * U + u][j]; s2[j] += red[1][k * U + u][j]; }
    }
#pragma unroll
    for (int j = 0; j < E; ++j) {
      part[((long long)blockIdx.x * 2 + 0) * C + c + j] = s1[j];
      part[((long long)blockIdx.x * 2 + 1) * C + c + j] = s2[j];
    }
  }
}

// deterministic two-stage column sum of a [rows][ld] fp32 partial matrix:
// stage 1 -> fp64 partials [RB][cols] (fixed row chunks), stage 2 -> out[cols]
constexpr int COLSUM_RB_MAX = 256;
__global__ __launch_bounds__(NT) void colsum_stage1(const float* part, int rows, int cols, int ld, int chunk,
                                                    double* ws) {
  __shared__ double sh[4][64];
  const int tid = threadIdx.x, cl = tid & 63, rg = tid >> 6;
  const int col = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  double s = 0.0;
  if (col < cols) {
    // 8 loads in flight per thread, added in the same row order as one at a time
    // (+0.0 for the rows past the chunk: s starts at +0.0 and never becomes -0.0, so adding it is exact)
    for (int r = r0 + rg; r < r1; r += 32) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // unconditional loads (clamped row), then the select
        const float x = part[(long long)min(r + 4 * i, r1 - 1) * ld + col];
        v[i] = r + 4 * i < r1 ? x : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += (double)v[i];
    }
  }
  sh[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && col < cols) ws[(long long)blockIdx.y * cols + col] = sh[0][cl] + sh[1][cl] + sh[2][cl] + sh[3][cl];
}

__global__ __launch_bounds__(NT) void colsum_stage2(const double* ws, int rb, int cols, ColSegs segs) {
  __shared__ double sh[4][64];
  const int tid = threadIdx.x, cl = tid & 63, rg = tid >> 6;
  const int col = blockIdx.x * 64 + cl;
  double s = 0.0;
  if (col < cols) {
    for (int r = rg; r < rb; r += 32) {
      double v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const double x = ws[(long long)min(r + 4 * i, rb - 1) * cols + col];
        v[i] = r + 4 * i < rb ? x : 0.0;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[i];
    }
  }
  sh[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && col < cols) {
    const float v = (float)(sh[0][cl] + sh[1][cl] + sh[2][cl] + sh[3][cl]);
    int i = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j) i = (j < segs.n && col >= segs.start[j]) ? j : i;
    segs.out[i][col - segs.start[i]] = v;
  }
}

// gy = gamma istd (g' - dbeta/n - xhat dgamma/n), g' = g [y scale + shift > 0] (the forward's ReLU
// mask: every BN-backward reduction and this apply use the forward affine, so the sums the apply
// subtracts are over exactly the g' it applies), folded per channel into gy = K1 g' + y K2 + K3
// with K1 = scale = gamma istd.  A thread keeps one 16-byte channel
// unit with its coefficients in registers and strides over pixels; the block holds
// floor(256 / U) pixels x U units (base_ch 96 -> U = 12, 21 pixels per step).
// The per-channel constants of the BN-backward apply, gy = k1 g' + k2 y + k3 (k1 = scale = gamma
// istd, also the forward-mask slope; kq = shift).  One function for the standalone apply below and
// the coefficient table the fused consumers read (eunet_bn_bwd_coef -> conv3x3 dgrad staging), so
// both round identically.
struct BnBwdCoef { float k1, kq, k2, k3; };
__device__ __forceinline__ BnBwdCoef bn_bwd_coef(float mean, float istd, float scale, float shift, float dbeta,
                                                 float dgamma, float inv_n) {
  const float off = -mean * istd;
  const float dg = dgamma * inv_n;
  BnBwdCoef c;
  c.k1 = scale;
  c.kq = shift;
  c.k2 = -scale * istd * dg;
  c.k3 = -scale * fmaf(off, dg, dbeta * inv_n);
  return c;
}

__global__ void bn_bwd_coef_kernel(const float* mean, const float* istd, const float* scale, const float* shift,
                                   const float* dbeta, const float* dgamma, float inv_n, int C, float* coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const BnBwdCoef k = bn_bwd_coef(mean[c], istd[c], scale[c], shift[c], dbeta[c], dgamma[c], inv_n);
  coef[c] = k.k1;
  coef[C + c] = k.kq;
  coef[2 * C + c] = k.k2;
  coef[3 * C + c] = k.k3;
}

template <typename T, typename TO, bool COEF = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* g, int gct, int gco, const T* y, int yct, int yco,
                                                           long long P, int C, const float* mean, const float* istd,
                                                           const float* scale, const float* shift, const float* dbeta,
                                                           const float* dgamma, TO* gy, int oct, int oco,
                                                           const float* coef) {
  constexpr int E = Vec16<T>::N;
  const int U = C / E;
  const int u = threadIdx.x % U, c = u * E;
  const float inv_n = 1.f / (float)P;
  float kP[E], kQ[E], k1[E], k2[E], k3[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    // COEF: the table eunet_bn_bwd_coef wrote (the same bn_bwd_coef values).  A compile-time choice:
    // with a runtime one the kernel held both paths' registers and ran 35 % slower (2.61 vs
    // 1.93 ms/step over its 14 launches, same-box rocprofv3)
    BnBwdCoef k;
    if constexpr (COEF)
      k = BnBwdCoef{coef[c + j], coef[C + c + j], coef[2 * C + c + j], coef[3 * C + c + j]};
    else
      k = bn_bwd_coef(mean[c + j], istd[c + j], scale[c + j], shift[c + j], dbeta[c + j], dgamma[c + j], inv_n);
    kP[j] = k.k1;
    kQ[j] = k.kq;
    k1[j] = k.k1;
    k2[j] = k.k2;
    k3[j] = k.k3;
  }
  const int ppb = blockDim.x / U;  // pixels per block per step (blockDim.x = ppb * U)
  for (long long p = (long long)blockIdx.x * ppb + threadIdx.x / U; p < P; p += (long long)gridDim.x * ppb) {
    float gf[E], yf[E], o[E];
    // g and y are read once here: non-temporal loads, so they do not displace the L2 lines the
    // concurrent weight-gradient kernels re-read (their X halo / dY tiles)
    Vec16<T>::unpack(__builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4*)(g + p * gct + gco + c))), gf);
    Vec16<T>::unpack(__builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4*)(y + p * yct + yco + c))), yf);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const float gg = fmaf(yf[j], kP[j], kQ[j]) > 0.f ? gf[j] : 0.f;
      o[j] = fmaf(k1[j], gg, fmaf(yf[j], k2[j], k3[j]));
    }
    EUNET_DASSERT(p < P && oco + c + E <= oct && u < U);
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, Vec16<TO>::pack(o)), (u32x4*)(gy + p * oct + oco + c));
  }
}

// bn_bwd_apply for dec1's input gradient without it in memory: g = W^T gz recomputed per pixel exactly as
// conv1x1_bwd_kernel forms it (the same fmaf chain over k < 3 with zero weights / gz past K, then its rounding
// to T), then the apply above.  conv1x1_bwd_bnr reduced the same rounded g' and no longer stores g: at the
// bench shape a 64-channel bf16 tensor at 1024^2 x 4, 537 MB written there and read here (the gz read that
// replaces it: 33 MB).
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_1x1_kernel(const T* y, int yct, int yco, long long P, int C,
                                                               const float* w, int K, const float* gz,
                                                               const float* mean, const float* istd,
                                                               const float* scale, const float* shift,
                                                               const float* dbeta, const float* dgamma, T* gy, int oct,
                                                               int oco) {
  constexpr int E = Vec16<T>::N;
  const int U = C / E;
  const int u = threadIdx.x % U, c = u * E;
  const float inv_n = 1.f / (float)P;
  float kP[E], kQ[E], k1[E], k2[E], k3[E], wk[3][E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const BnBwdCoef k = bn_bwd_coef(mean[c + j], istd[c + j], scale[c + j], shift[c + j], dbeta[c + j],
                                    dgamma[c + j], inv_n);
    kP[j] = k.k1;
    kQ[j] = k.kq;
    k1[j] = k.k1;
    k2[j] = k.k2;
    k3[j] = k.k3;
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) wk[kk][j] = kk < K ? w[kk * C + c + j] : 0.f;
  }
  const int ppb = blockDim.x / U;
  for (long long p = (long long)blockIdx.x * ppb + threadIdx.x / U; p < P; p += (long long)gridDim.x * ppb) {
    float gk[3];
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) gk[kk] = kk < K ? gz[p * K + kk] : 0.f;
    float yf[E], go[E], gf[E], o[E];
    Vec16<T>::unpack(__builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4*)(y + p * yct + yco + c))), yf);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      float sv = 0.f;
#pragma unroll
      for (int kk = 0; kk < 3; ++kk) sv = fmaf(wk[kk][j], gk[kk], sv);
      go[j] = sv;
    }
    Vec16<T>::unpack(Vec16<T>::pack(go), gf);  // the rounding of conv1x1_bwd's store
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const float gg = fmaf(yf[j], kP[j], kQ[j]) > 0.f ? gf[j] : 0.f;
      o[j] = fmaf(k1[j], gg, fmaf(yf[j], k2[j], k3[j]));
    }
    EUNET_DASSERT(p < P && oco + c + E <= oct && u < U);
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, Vec16<T>::pack(o)), (u32x4*)(gy + p * oct + oco + c));
  }
}

// Fused BN-backward reduction in a gradient producer (the reduction half of bn_bwd_reduce for
// the block whose output gradient g the kernel writes): each thread accumulates, for its 16-byte
// channel unit, s1 += g', s2 += g' xhat over the pixels it writes (g' = stored g where
// y scale + shift > 0, xhat = (y - mean) istd); the block then sums its threads of equal unit
// in fixed order into part[block][2][C].  Requires blockDim.x % U == 0 (U = C / E channel units).
struct BnRed {
  const void* y; int yct, yco;
  const float* mean; const float* istd; const float* scale; const float* shift;  // scale / shift: the forward affine
  float* part;
};

template <typename T>
__device__ __forceinline__ void bnred_block(const BnRed& r, int C, const float* s1, const float* s2) {
  constexpr int E = Vec16<T>::N;
  __shared__ float red[2][NT][E];
  const int tid = threadIdx.x, U = C / E;
#pragma unroll
  for (int j = 0; j < E; ++j) { red[0][tid][j] = s1[j]; red[1][tid][j] = s2[j]; }
  __syncthreads();
  if (tid < U) {
    float t1[E], t2[E];
#pragma unroll
    for (int j = 0; j < E; ++j) { t1[j] = 0.f; t2[j] = 0.f; }
    for (int k = tid; k < (int)blockDim.x; k += U)
#pragma unroll
      for (int j = 0; j < E; ++j) { t1[j] += red[0][k][j]; t2[j] += red[1][k][j]; }
#pragma unroll
    for (int j = 0; j < E; ++j) {
      r.part[((long long)blockIdx.x * 2 + 0) * C + tid * E + j] = t1[j];
      r.part[((long long)blockIdx.x * 2 + 1) * C + tid * E + j] = t2[j];
    }
  }
}

// Per-thread BN-backward constants of one 16-byte channel unit (the thread's unit is fixed across
// the grid-stride loops below: the stride is a multiple of U).
template <int E>
struct BnUnit {
  float mu[E], is[E], sc[E], sh[E];
  __device__ __forceinline__ void load(const BnRed& r, int c) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      mu[j] = r.mean[c + j];
      is[j] = r.istd[c + j];
      sc[j] = r.scale[c + j];
      sh[j] = r.shift[c + j];
    }
  }
  // s1 += g', s2 += g' xhat with g' = g [y scale + shift > 0], xhat = (y - mean) istd
  __device__ __forceinline__ void acc(const float* g, const float* y, float* s1, float* s2) const {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const float gp = fmaf(y[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
      s1[j] += gp;
      s2[j] = fmaf(gp, (y[j] - mu[j]) * is[j], s2[j]);
    }
  }
};

// MaxPool2d(2) adjoint (+ the skip gradient gs): every load of a unit is issued before its first
// store (the stores may alias the loads for the compiler, so loads placed after a store would wait
// for it).  RED: the pooled activation is not read -- bnrelu_pool stored it as
// round(relu(y scale + shift)), recomputed here bit for bit from the y the BN-backward reduction
// reads anyway, so the argmax (first maximum, NaN wins, as max_pool2d) is the same.
template <typename T, bool RED = false>
// amdgpu_waves_per_eu(1): its own ~165 registers, 3 waves per SIMD (4 spills 80 B: 699 -> 832 us per step)
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1))) void pool_bwd_add_kernel(const T* act, int act_ct, int act_co, const T* gp, int gpct,
                                                          int gpco, const T* gs, int gsct, int gsco, T* go, int goct,
                                                          int goco, int N, int H, int W, int C, BnRed br) {
  constexpr int E = Vec16<T>::N;
  const int U = C / E, Ho = H / 2, Wo = W / 2;
  float s1[E], s2[E];
#pragma unroll
  for (int j = 0; j < E; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  BnUnit<E> bu;
  const long long id0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (RED) bu.load(br, (int)(id0 % U) * E);
  const T* src = RED ? (const T*)br.y : act;
  const int sct = RED ? br.yct : act_ct, sco = RED ? br.yco : act_co;
  for (long long id = id0; id < (long long)N * Ho * Wo * U; id += (long long)gridDim.x * blockDim.x) {
    const int u = (int)(id % U);
    long long p = id / U;
    const int xo = (int)(p % Wo); p /= Wo;
    const int yo = (int)(p % Ho);
    const int n = (int)(p / Ho);
    const int c = u * E;
    long long pix[4];
    uint4 ra[4], rs[4];
    // every input element is read once (disjoint 2x2 windows): non-temporal loads, so they do not
    // displace the L2 lines the concurrent weight-gradient kernels re-read
    auto ldnt = [](const T* q) { return __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4*)q)); };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pix[k] = (long long)(n * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1);
      ra[k] = ldnt(src + pix[k] * sct + sco + c);
    }
    const uint4 rg = ldnt(gp + ((long long)(n * Ho + yo) * Wo + xo) * gpct + gpco + c);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      rs[k] = gs != nullptr ? ldnt(gs + pix[k] * gsct + gsco + c) : make_uint4(0, 0, 0, 0);
    float best[E], gpv[E];
    int arg[E];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // argmax over the activation, unpacked from the loads on the fly
      float a[E];
      Vec16<T>::unpack(ra[k], a);
      if constexpr (RED) {
#pragma unroll
        for (int j = 0; j < E; ++j) a[j] = fmaxf(fmaf(a[j], bu.sc[j], bu.sh[j]), 0.f);
        Vec16<T>::unpack(Vec16<T>::pack(a), a);  // the stored (rounded) activation
      }
#pragma unroll
      for (int j = 0; j < E; ++j)
        if (k == 0 || a[j] > best[j] || (a[j] != a[j])) { best[j] = a[j]; arg[j] = k; }
    }
    Vec16<T>::unpack(rg, gpv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float o[E];
      Vec16<T>::unpack(rs[k], o);
#pragma unroll
      for (int j = 0; j < E; ++j) o[j] += (arg[j] == k) ? gpv[j] : 0.f;
      const uint4 packed = Vec16<T>::pack(o);
      if (go)  // (go null: reduced only, bn_bwd_apply_pool)
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, packed), (u32x4*)(go + pix[k] * goct + goco + c));
      if constexpr (RED) {
        float gr[E], yv[E];
        Vec16<T>::unpack(packed, gr);
        Vec16<T>::unpack(ra[k], yv);
        bu.acc(gr, yv, s1, s2);
      }
    }
  }
  if constexpr (RED) bnred_block<T>(br, C, s1, s2);
}

// bn_bwd_apply for the max-pool adjoint's gradient without it in memory: per 2x2 window and channel unit the
// gradient gout = gs + scatter(gp) is recomputed exactly as pool_bwd_add_kernel<T, true> forms and rounds it
// (argmax over round(relu(y scale + shift)), first maximum, NaN wins), then the BN-backward apply of the block's
// second BatchNorm.  pool_bwd_add_bnr reduced the same g' and no longer stores gout: the apply reads gs and the
// quarter-size gp instead of gout -- 0.75 C per pixel less traffic (gout's write and read, gp's re-read).  The
// block size is a multiple of the channel units (bnr_block), so a thread keeps one unit's constants.
template <typename T>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1))) void bn_bwd_apply_pool_kernel(
    const T* gp, int gpct, int gpco, const T* gs, int gsct, int gsco, const T* y, int yct, int yco, const float* mean,
    const float* istd, const float* scale, const float* shift, const float* dbeta, const float* dgamma, T* gy, int oct,
    int oco, int N, int H, int W, int C) {
  constexpr int E = Vec16<T>::N;
  const int U = C / E, Ho = H / 2, Wo = W / 2;
  const float inv_n = 1.f / (float)((long long)N * H * W);
  const long long id0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c = (int)(id0 % U) * E;
  float kP[E], kQ[E], k1[E], k2[E], k3[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const BnBwdCoef k = bn_bwd_coef(mean[c + j], istd[c + j], scale[c + j], shift[c + j], dbeta[c + j],
                                    dgamma[c + j], inv_n);
    kP[j] = k.k1;
    kQ[j] = k.kq;
    k1[j] = k.k1;
    k2[j] = k.k2;
    k3[j] = k.k3;
  }
  auto ldnt = [](const T* q) { return __builtin_bit_cast(uint4, __builtin_nontemporal_load((const u32x4*)q)); };
  for (long long id = id0; id < (long long)N * Ho * Wo * U; id += (long long)gridDim.x * blockDim.x) {
    long long p = id / U;
    const int xo = (int)(p % Wo); p /= Wo;
    const int yo = (int)(p % Ho);
    const int n = (int)(p / Ho);
    long long pix[4];
    uint4 ra[4], rs[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pix[k] = (long long)(n * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1);
      ra[k] = ldnt(y + pix[k] * yct + yco + c);
    }
    const uint4 rg = ldnt(gp + ((long long)(n * Ho + yo) * Wo + xo) * gpct + gpco + c);
#pragma unroll
    for (int k = 0; k < 4; ++k) rs[k] = gs != nullptr ? ldnt(gs + pix[k] * gsct + gsco + c) : make_uint4(0, 0, 0, 0);
    float best[E], gpv[E];
    int arg[E];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float a[E];
      Vec16<T>::unpack(ra[k], a);
#pragma unroll
      for (int j = 0; j < E; ++j) a[j] = fmaxf(fmaf(a[j], kP[j], kQ[j]), 0.f);
      Vec16<T>::unpack(Vec16<T>::pack(a), a);
#pragma unroll
      for (int j = 0; j < E; ++j)
        if (k == 0 || a[j] > best[j] || (a[j] != a[j])) { best[j] = a[j]; arg[j] = k; }
    }
    Vec16<T>::unpack(rg, gpv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float o[E], gr[E], yv[E], out[E];
      Vec16<T>::unpack(rs[k], o);
#pragma unroll
      for (int j = 0; j < E; ++j) o[j] += (arg[j] == k) ? gpv[j] : 0.f;
      Vec16<T>::unpack(Vec16<T>::pack(o), gr);  // the rounding of pool_bwd_add's store
      Vec16<T>::unpack(ra[k], yv);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        const float gg = fmaf(yv[j], kP[j], kQ[j]) > 0.f ? gr[j] : 0.f;
        out[j] = fmaf(k1[j], gg, fmaf(yv[j], k2[j], k3[j]));
      }
      __builtin_nontemporal_store(__builtin_bit_cast(u32x4, Vec16<T>::pack(out)), (u32x4*)(gy + pix[k] * oct + oco + c));
    }
  }
}


template <typename T, typename TO>
__global__ void up_bwd_kernel(const T* g, int gct, int gco, TO* o, int oct, int oco, int N, int h, int w, int C) {
  constexpr int E = Vec16<T>::N;
  const int U = C / E, H2 = 2 * h, W2 = 2 * w;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long long)N * h * w * U) return;
  const int u = (int)(id % U);
  long long p = id / U;
  const int x = (int)(p % w); p /= w;
  const int y = (int)(p % h);
  const int n = (int)(p / h);
  const int c = u * E;
  float acc[E];
#pragma unroll
  for (int j = 0; j < E; ++j) acc[j] = 0.f;
  for (int oy = 2 * y - 1; oy <= 2 * y + 2; ++oy) {
    if (oy < 0 || oy >= H2) continue;
    const float wy = up2_adj_w(oy, h, y);
    if (wy == 0.f) continue;
    for (int ox = 2 * x - 1; ox <= 2 * x + 2; ++ox) {
      if (ox < 0 || ox >= W2) continue;
      const float wx = up2_adj_w(ox, w, x);
      if (wx == 0.f) continue;
      float f[E];
      Vec16<T>::unpack(*(const uint4*)(g + ((long long)(n * H2 + oy) * W2 + ox) * gct + gco + c), f);
      const float ww = wy * wx;
#pragma unroll
      for (int j = 0; j < E; ++j) acc[j] = fmaf(ww, f[j], acc[j]);
    }
  }
  *(uint4*)(o + ((long long)(n * h + y) * w + x) * oct + oco + c) = Vec16<TO>::pack(acc);
}

// Upsample x2 adjoint, separable, as a row sweep: a thread owns low-res columns x0, x0+1 of one
// 16-byte channel unit over UP_R low-res rows.  Each high-res row r of its 6-column window is
// reduced horizontally once (H_b[r] = sum_dx wx_b(dx) g[r][2 x0 - 1 + dx]) and weighted into the
// (at most two) output rows it feeds (rows 2y-1 .. 2y+2 feed y): per output row two new high-res
// rows are read (6 loads per output instead of 9 for a 2x2 block).  RED: the BN-backward sums of
// the produced gradient, with the outputs' y loaded with the window rows (a load placed after a
// store that may alias it would wait for the store).
constexpr int UP_R = 8;
// amdgpu_waves_per_eu(2): left alone the fused-reduction bf16 instance took 258 registers (1 wave / SIMD); at 2
// it fits 256 and ran 959 -> 796 us per step
template <typename T, typename TO, bool RED = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void up_bwd_rows_kernel(const T* g, int gct, int gco, TO* o, int oct, int oco, int N,
                                                          int h, int w, int C, BnRed br) {
  constexpr int E = Vec16<T>::N;
  const int U = C / E, H2 = 2 * h, W2 = 2 * w, hr = (h + UP_R - 1) / UP_R, wb = (w + 1) / 2;
  float s1[E], s2[E];
#pragma unroll
  for (int j = 0; j < E; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  for (long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x; id < (long long)N * hr * wb * U;
       id += (long long)gridDim.x * blockDim.x) {
    const int u = (int)(id % U);
    long long p = id / U;
    const int xb = (int)(p % wb); p /= wb;
    const int yr = (int)(p % hr);
    const int n = (int)(p / hr);
    const int c = u * E, x0 = 2 * xb, ys = yr * UP_R, ye = min(h, ys + UP_R);
    float wxs[6][2];
#pragma unroll
    for (int dx = 0; dx < 6; ++dx) {
      const int ox = 2 * x0 - 1 + dx;
      const bool ok = ox >= 0 && ox < W2;
      wxs[dx][0] = ok ? up2_adj_w(ox, w, x0) : 0.f;
      wxs[dx][1] = ok && x0 + 1 < w ? up2_adj_w(ox, w, x0 + 1) : 0.f;
    }
    const T* gn = g + (long long)n * H2 * W2 * gct + gco + c;
    // horizontal partials of high-res row r (zero outside the image); packed fp32 (v_pk_fma_f32: two
    // channels per instruction, each element rounded as the scalar fma rounds it)
    constexpr int E2 = E / 2;
    auto hrow = [&](int r, f32x2 (*hv)[E2]) {
      uint4 v[6];
#pragma unroll
      for (int dx = 0; dx < 6; ++dx) {
        const int ox = 2 * x0 - 1 + dx;
        v[dx] = (r >= 0 && r < H2 && ox >= 0 && ox < W2) ? *(const uint4*)(gn + ((long long)r * W2 + ox) * gct)
                                                          : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < E2; ++j) hv[b][j] = (f32x2){0.f, 0.f};
#pragma unroll
      for (int dx = 0; dx < 6; ++dx) {
        float f[E];
        Vec16<T>::unpack(v[dx], f);
        const f32x2 w0 = {wxs[dx][0], wxs[dx][0]}, w1 = {wxs[dx][1], wxs[dx][1]};
#pragma unroll
        for (int j = 0; j < E2; ++j) {
          const f32x2 fv = {f[2 * j], f[2 * j + 1]};
          hv[0][j] = __builtin_elementwise_fma(w0, fv, hv[0][j]);
          hv[1][j] = __builtin_elementwise_fma(w1, fv, hv[1][j]);
        }
      }
    };
    // row r feeds the outputs y with 2y-1 <= r <= 2y+2: carry the next output row's partial sums
    auto wrow = [&](int r, int y) { return (r >= 0 && r < H2 && y < h) ? up2_adj_w(r, h, y) : 0.f; };
    f32x2 acur[2][E2], anext[2][E2], hv[2][E2];
    hrow(2 * ys - 1, hv);
    {
      const float wa = wrow(2 * ys - 1, ys);
      const f32x2 wa2 = {wa, wa};
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < E2; ++j) acur[b][j] = wa2 * hv[b][j];
    }
    hrow(2 * ys, hv);
    {
      const float wa = wrow(2 * ys, ys);
      const f32x2 wa2 = {wa, wa};
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < E2; ++j) acur[b][j] = __builtin_elementwise_fma(wa2, hv[b][j], acur[b][j]);
    }
#pragma unroll 1
    for (int y = ys; y < ye; ++y) {
      uint4 ryv[2];
#pragma unroll
      for (int b = 0; b < 2; ++b)
        ryv[b] = (RED && x0 + b < w)
                     ? *(const uint4*)((const TO*)br.y + ((long long)(n * h + y) * w + x0 + b) * br.yct + br.yco + c)
                     : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int k = 1; k <= 2; ++k) {
        hrow(2 * y + k, hv);
        const float wc = wrow(2 * y + k, y), wn = wrow(2 * y + k, y + 1);
        const f32x2 wc2 = {wc, wc}, wn2 = {wn, wn};
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int j = 0; j < E2; ++j) {
            acur[b][j] = __builtin_elementwise_fma(wc2, hv[b][j], acur[b][j]);
            anext[b][j] = k == 1 ? wn2 * hv[b][j] : __builtin_elementwise_fma(wn2, hv[b][j], anext[b][j]);
          }
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (x0 + b >= w) continue;
        const long long pix = (long long)(n * h + y) * w + x0 + b;
        float ac[E];
#pragma unroll
        for (int j = 0; j < E2; ++j) { ac[2 * j] = acur[b][j].x; ac[2 * j + 1] = acur[b][j].y; }
        const uint4 packed = Vec16<TO>::pack(ac);
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, packed), (u32x4*)(o + pix * oct + oco + c));
        if constexpr (RED) {
          float gr[E], yv[E];
          Vec16<TO>::unpack(packed, gr);
          Vec16<TO>::unpack(ryv[b], yv);
#pragma unroll
          for (int j = 0; j < E; ++j) {  // (the BN constants from L1: registers would cost occupancy)
            const float gp = fmaf(yv[j], br.scale[c + j], br.shift[c + j]) > 0.f ? gr[j] : 0.f;
            s1[j] += gp;
            s2[j] = fmaf(gp, (yv[j] - br.mean[c + j]) * br.istd[c + j], s2[j]);
          }
        }
      }
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < E2; ++j) acur[b][j] = anext[b][j];
    }
  }
  if constexpr (RED) bnred_block<TO>(br, C, s1, s2);
}

// fp32 K-channel (K <= 4) upsample backward for the head: g [N,2h,2w,K] -> o [N,h,w,K]
__global__ void up_bwd_small_kernel(const float* g, float* o, int N, int h, int w, int K) {
  const int H2 = 2 * h, W2 = 2 * w;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long long)N * h * w) return;
  const int x = (int)(id % w);
  const int y = (int)((id / w) % h);
  const int n = (int)(id / ((long long)w * h));
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int oy = 2 * y - 1; oy <= 2 * y + 2; ++oy) {
    if (oy < 0 || oy >= H2) continue;
    const float wy = up2_adj_w(oy, h, y);
    if (wy == 0.f) continue;
    for (int ox = 2 * x - 1; ox <= 2 * x + 2; ++ox) {
      if (ox < 0 || ox >= W2) continue;
      const float wx = up2_adj_w(ox, w, x);
      if (wx == 0.f) continue;
      const float* gp = g + ((long long)(n * H2 + oy) * W2 + ox) * K;
      for (int k = 0; k < K; ++k) acc[k] = fmaf(wy * wx, gp[k], acc[k]);
    }
  }
  for (int k = 0; k < K; ++k) o[id * K + k] = acc[k];
}

// K = 2 specialisation: separable row / column adjoint weights computed once per thread, one
// 8-byte load per contributing high-res pixel
__global__ __launch_bounds__(256) void up_bwd_k2_kernel(const float2* g, float2* o, int N, int h, int w) {
  const int H2 = 2 * h, W2 = 2 * w;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long long)N * h * w) return;
  const int x = (int)(id % w);
  const int y = (int)((id / w) % h);
  const int n = (int)(id / ((long long)w * h));
  float wy[4], wx[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int oy = 2 * y - 1 + d, ox = 2 * x - 1 + d;
    wy[d] = (oy >= 0 && oy < H2) ? up2_adj_w(oy, h, y) : 0.f;
    wx[d] = (ox >= 0 && ox < W2) ? up2_adj_w(ox, w, x) : 0.f;
  }
  float2 acc = make_float2(0.f, 0.f);
#pragma unroll
  for (int dy = 0; dy < 4; ++dy) {
    if (wy[dy] == 0.f) continue;
    const float2* row = g + (long long)(n * H2 + 2 * y - 1 + dy) * W2;
#pragma unroll
    for (int dx = 0; dx < 4; ++dx) {
      if (wx[dx] == 0.f) continue;
      const float2 v = row[2 * x - 1 + dx];
      const float ww = wy[dy] * wx[dx];
      acc.x = fmaf(ww, v.x, acc.x);
      acc.y = fmaf(ww, v.y, acc.y);
    }
  }
  o[id] = acc;
}

// dec1 backward: gact = W^T gz; per-block partials of gW [K][C] and gb [K].
// 8 lanes per pixel, lane group g owns channels 8g+64j (C <= 128); partial
// sums stay in registers over the block's C1X_PIX pixels.
constexpr int C1X_PIX = 1024;
// J = 1 (C <= 64) or 2 (C <= 128): the per-lane state (BN constants, 1x1 weights, partial sums)
// is sized by it, so the 64-channel dec2 output runs at twice the occupancy
#define C1X_LAUNCH(kern, T, BNR, ARGS)                                                       \
  do {                                                                                       \
    if (y->c <= 64) kern<T, 1, BNR><<<tiles, NT, 0, (hipStream_t)stream>>> ARGS;             \
    else kern<T, 2, BNR><<<tiles, NT, 0, (hipStream_t)stream>>> ARGS;                        \
  } while (0)
// sum over the 8 pixel slots of a wave (lanes l, l^8, l^16, l^32, ...): DPP row rotate by 8 within
// each 16-lane row, then the gfx950 permlane16 / permlane32 swaps (no ds_bpermute round trips)
__device__ __forceinline__ float sum_slots8(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));  // row_ror 8
  return xor32_sum(xor16_sum(v));
}

// BNR: also the BN-backward reduction (sum g', sum g' xhat) of y's BatchNorm over the produced
// gradient (g' = the stored gradient where relu(bn(y)) > 0), per block into bpart[block][2][C]
template <typename T, int J, bool BNR>  // J = ceil(C / 64) channel halves per lane group
__global__ __launch_bounds__(NT) void conv1x1_bwd_kernel(const T* y, long long P, int C, int yct, int yco,
                                                         const float* sc, const float* sh, const float* w, int K,
                                                         const float* gz, T* ga, int gct, int gco, float* part,
                                                         const float* bmean, const float* bistd, float* bpart) {
  constexpr int E = Vec16<T>::N;
  __shared__ float red[4][3 * 128 + 3 + (BNR ? 2 * 128 : 0)];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane & 7, ps = tid >> 3;
  const int stride = K * C + K;
  float aw[J][3][8], ab[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) aw[j][k][e] = 0.f;
  float s8[J][8], t8[J][8], w8[J][3][8];  // this lane's channels 64j + 8g + e
  float mu8[J][8], is8[J][8], bs1[J][8], bs2[J][8];
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 64 * j + 8 * g + e;
      const bool ok = c < C;
      s8[j][e] = ok ? sc[c] : 0.f;
      t8[j][e] = ok ? sh[c] : 0.f;
      if constexpr (BNR) {
        mu8[j][e] = ok ? bmean[c] : 0.f;
        is8[j][e] = ok ? bistd[c] : 0.f;
        bs1[j][e] = 0.f;
        bs2[j][e] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) w8[j][k][e] = (ok && k < K) ? w[k * C + c] : 0.f;
    }
  const long long p0 = (long long)blockIdx.x * C1X_PIX;
  const long long p1 = min(P, p0 + C1X_PIX);
  // PPI pixels per iteration (2 when the state fits), every load issued before the first store
  // (a load placed after a store that may alias it waits for the store)
  constexpr int PPI = J == 1 ? 2 : 1;
  for (long long pa = p0 + ps; pa < p1; pa += 32 * PPI) {
    float gk[PPI][3];
    uint4 ry[PPI][J][2];  // [pixel][j][half]
#pragma unroll
    for (int i = 0; i < PPI; ++i) {
      const long long p = pa + 32 * i;
      const bool pv = p < p1;
#pragma unroll
      for (int k = 0; k < 3; ++k) gk[i][k] = (pv && k < K) ? gz[p * K + k] : 0.f;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = 64 * j + 8 * g;
        const bool ok = pv && c < C;
        ry[i][j][0] = ok ? *(const uint4*)(y + p * yct + yco + c) : make_uint4(0, 0, 0, 0);
        ry[i][j][1] = (ok && E == 4) ? *(const uint4*)(y + p * yct + yco + c + 4) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < PPI; ++i) {
      const long long p = pa + 32 * i;
      if (p >= p1) continue;
      if (g == 0)
#pragma unroll
        for (int k = 0; k < 3; ++k) ab[k] += gk[i][k];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c = 64 * j + 8 * g;
        if (c >= C) continue;
        float f[8], go[8];
        Vec16<T>::unpack(ry[i][j][0], f);
        if constexpr (E == 4) Vec16<T>::unpack(ry[i][j][1], f + 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float act = fmaxf(fmaf(f[e], s8[j][e], t8[j][e]), 0.f);
          float sv = 0.f;
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            sv = fmaf(w8[j][k][e], gk[i][k], sv);
            aw[j][k][e] = fmaf(gk[i][k], act, aw[j][k][e]);
          }
          go[e] = sv;
        }
        const uint4 pk0 = Vec16<T>::pack(go);
        if (ga) *(uint4*)(ga + p * gct + gco + c) = pk0;  // (ga null: reduced only, eunet_bn_bwd_apply_1x1)
        uint4 pk1 = pk0;
        if constexpr (E == 4) {
          pk1 = Vec16<T>::pack(go + 4);
          if (ga) *(uint4*)(ga + p * gct + gco + c + 4) = pk1;
        }
        if constexpr (BNR) {  // the stored (rounded) gradient, as bn_bwd_reduce would read it
          float gr[8];
          Vec16<T>::unpack(pk0, gr);
          if constexpr (E == 4) Vec16<T>::unpack(pk1, gr + 4);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float xh = (f[e] - mu8[j][e]) * is8[j][e];
            const float gp = fmaf(f[e], s8[j][e], t8[j][e]) > 0.f ? gr[e] : 0.f;
            bs1[j][e] += gp;
            bs2[j][e] = fmaf(gp, xh, bs2[j][e]);
          }
        }
      }
    }
  }
  // reduce over the 8 pixel slots of each wave (xor 8, 16, 32), then across waves
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) aw[j][k][e] = k < K ? sum_slots8(aw[j][k][e]) : 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) ab[k] = k < K ? sum_slots8(ab[k]) : 0.f;
  if constexpr (BNR)
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bs1[j][e] = sum_slots8(bs1[j][e]);
        bs2[j][e] = sum_slots8(bs2[j][e]);
      }
  if (lane < 8) {
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = 64 * j + 8 * g + e;
          if (k < K && c < C) red[wv][k * C + c] = aw[j][k][e];
        }
    if (lane == 0)
      for (int k = 0; k < K; ++k) red[wv][K * C + k] = ab[k];
    if constexpr (BNR)
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int c = 64 * j + 8 * g + e;
          if (c < C) {
            red[wv][stride + c] = bs1[j][e];
            red[wv][stride + C + c] = bs2[j][e];
          }
        }
  }
  __syncthreads();
  for (int i = tid; i < stride; i += NT)
    part[(long long)blockIdx.x * stride + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  if constexpr (BNR)
    for (int i = tid; i < 2 * C; i += NT)
      bpart[(long long)blockIdx.x * 2 * C + i] =
          red[0][stride + i] + red[1][stride + i] + red[2][stride + i] + red[3][stride + i];
}

}  // namespace

// ===========================================================================
static int colsum_rb(int rows) {
  int rb = (rows + 63) / 64;
  return rb < 1 ? 1 : (rb > COLSUM_RB_MAX ? COLSUM_RB_MAX : rb);
}

size_t eunet_colsum_ws(int rows, int cols) { return (size_t)colsum_rb(rows) * cols * sizeof(double); }

int eunet_colsum_segs(const float* part, int rows, int cols, int ld, const ColSegs& segs, void* ws, hipStream_t s) {
  EUNET_REQUIRE(part && ws && rows > 0 && cols > 0 && ld >= cols && segs.n >= 1 && segs.n <= 4 && segs.start[0] == 0,
                "colsum: bad args");
  for (int i = 0; i < segs.n; ++i)
    EUNET_REQUIRE(segs.out[i] && (i == 0 || (segs.start[i] > segs.start[i - 1] && segs.start[i] < cols)),
                  "colsum: bad segments");
  const int rb = colsum_rb(rows);
  const int chunk = cdiv(rows, rb);
  colsum_stage1<<<dim3(cdiv(cols, 64), rb), NT, 0, s>>>(part, rows, cols, ld, chunk, (double*)ws);
  colsum_stage2<<<cdiv(cols, 64), NT, 0, s>>>((const double*)ws, rb, cols, segs);
  EUNET_LAUNCH_CHECK("colsum");
  return EUNET_OK;
}

int eunet_colsum_ld(const float* part, int rows, int cols, int ld, float* out, void* ws, hipStream_t s, int split,
                    float* out_hi) {
  ColSegs g = {{out, out_hi, nullptr, nullptr}, {0, split, 0, 0}, out_hi != nullptr ? 2 : 1};
  return eunet_colsum_segs(part, rows, cols, ld, g, ws, s);
}

extern "C" {

int eunet_nchw_to_nhwc(const float* x, const eunet_act* out, void* stream);

int eunet_conv_small_fwd(const eunet_act* x, const float* w, const float* bias, const eunet_act* y, float* stats,
                         void* stream) {
  EUNET_REQUIRE(act_ok(x) && act_ok(y) && w, "conv_small_fwd: bad args");
  EUNET_REQUIRE(x->c <= SCI && x->dtype == y->dtype, "conv_small_fwd: Cin <= 8 and equal dtypes required");
  EUNET_REQUIRE(x->n == y->n && x->h == y->h && x->w == y->w, "conv_small_fwd: spatial mismatch");
  SmallArgs a;
  a.x = x->ptr; a.N = x->n; a.H = x->h; a.W = x->w; a.xct = x->ctot; a.xco = x->coff; a.cin = x->c;
  a.w = w; a.b = bias;
  a.y = y->ptr; a.yct = y->ctot; a.yco = y->coff; a.cout = y->c;
  a.stats = stats; a.tx = cdiv(x->w, STW); a.ty = cdiv(x->h, SFH); a.ntiles = x->n * a.tx * a.ty;
  dim3 grid(a.ntiles, cdiv(y->c, 64));
  const bool c1 = x->c == 1;
  if (x->dtype == EUNET_BF16) {
    if (c1) conv_small_fwd_kernel<bf16_t, true><<<grid, NT, 0, (hipStream_t)stream>>>(a);
    else conv_small_fwd_kernel<bf16_t, false><<<grid, NT, 0, (hipStream_t)stream>>>(a);
  } else {
    if (c1) conv_small_fwd_kernel<float, true><<<grid, NT, 0, (hipStream_t)stream>>>(a);
    else conv_small_fwd_kernel<float, false><<<grid, NT, 0, (hipStream_t)stream>>>(a);
  }
  EUNET_LAUNCH_CHECK("conv_small_fwd");
  return EUNET_OK;
}

int eunet_conv_small_wgrad_splits(const eunet_act* dy, int* nsplit) {
  EUNET_REQUIRE(act_ok(dy) && nsplit, "conv_small_wgrad_splits: bad args");
  const int ntiles = dy->n * cdiv(dy->h, STH) * cdiv(dy->w, STW);
  constexpr int SMALL_WG_BLOCKS = 512;  // 768 / 1024 measured slower (enc1.0: 213 -> 283 / 309 us)
  int s = cdiv(SMALL_WG_BLOCKS, cdiv(dy->c, 64));
  s = s > ntiles ? ntiles : (s < 1 ? 1 : s);
  const int per = cdiv(ntiles, s);
  *nsplit = cdiv(ntiles, per);
  return EUNET_OK;
}

int eunet_conv_small_wgrad(const eunet_act* x, const eunet_act* dy, float* dw_part, float* db_part, int nsplit,
                           void* stream) {
  EUNET_REQUIRE(act_ok(x) && act_ok(dy) && dw_part && nsplit > 0, "conv_small_wgrad: bad args");
  EUNET_REQUIRE(x->c <= SCI && x->dtype == dy->dtype, "conv_small_wgrad: Cin <= 8, equal dtypes");
  SmallWgArgs a;
  a.x = x->ptr; a.N = x->n; a.H = x->h; a.W = x->w; a.xct = x->ctot; a.xco = x->coff; a.cin = x->c;
  a.dy = dy->ptr; a.dct = dy->ctot; a.dco = dy->coff; a.cout = dy->c;
  a.dw = dw_part; a.db = db_part;
  a.tx = cdiv(x->w, STW); a.ty = cdiv(x->h, STH); a.ntiles = x->n * a.tx * a.ty;
  a.per_split = cdiv(a.ntiles, nsplit);
  EUNET_REQUIRE(cdiv(a.ntiles, a.per_split) == nsplit, "conv_small_wgrad: nsplit mismatch");
  dim3 grid(nsplit, cdiv(dy->c, 64));
  if (x->dtype == EUNET_BF16)
    if (x->c <= 4)
      conv_small_wgrad_kernel<bf16_t, 4><<<grid, NT, 0, (hipStream_t)stream>>>(a);
    else
      conv_small_wgrad_kernel<bf16_t, 8><<<grid, NT, 0, (hipStream_t)stream>>>(a);
  else
    if (x->c <= 4)
      conv_small_wgrad_kernel<float, 4><<<grid, NT, 0, (hipStream_t)stream>>>(a);
    else
      conv_small_wgrad_kernel<float, 8><<<grid, NT, 0, (hipStream_t)stream>>>(a);
  EUNET_LAUNCH_CHECK("conv_small_wgrad");
  return EUNET_OK;
}

int eunet_bn_finalize(const float* stats, int tiles, int c, const float* gamma, const float* beta, float eps,
                      float momentum, float* run_mean, float* run_var, float* mean, float* invstd, float* scale,
                      float* shift, int64_t* num_batches_tracked, void* stream) {
  EUNET_REQUIRE(stats && tiles > 0 && c > 0 && gamma && beta, "bn_finalize: bad args");
  bn_finalize_kernel<<<c, FNT, 0, (hipStream_t)stream>>>(stats, tiles, c, gamma, beta, eps, momentum, run_mean,
                                                        run_var, mean, invstd, scale, shift,
                                                        (long long*)num_batches_tracked, eunet::update_guard());
  EUNET_LAUNCH_CHECK("bn_finalize");
  return EUNET_OK;
}

int eunet_bn_eval_affine(int c, const float* gamma, const float* beta, const float* run_mean, const float* run_var,
                         float eps, float* scale, float* shift, void* stream) {
  EUNET_REQUIRE(c > 0 && gamma && beta && run_mean && run_var && scale && shift, "bn_eval_affine: bad args");
  bn_eval_affine_kernel<<<cdiv(c, 256), 256, 0, (hipStream_t)stream>>>(c, gamma, beta, run_mean, run_var, eps,
                                                                        scale, shift);
  EUNET_LAUNCH_CHECK("bn_eval_affine");
  return EUNET_OK;
}

int eunet_bnrelu(const eunet_act* y, const float* scale, const float* shift, const eunet_act* out, void* stream) {
  EUNET_REQUIRE(act_ok(y) && act_ok(out) && scale && shift && vec_ok(y) && vec_ok(out), "bnrelu: bad args");
  EUNET_REQUIRE(out->n == y->n && out->h == y->h && out->w == y->w && out->c == y->c && out->dtype == y->dtype,
                "bnrelu: shape mismatch");
  const long long P = (long long)y->n * y->h * y->w, total = P * (y->c / e16(y->dtype));
  const unsigned g = (unsigned)std::min<long long>((total + 255) / 256, 16384);
  if (y->dtype == EUNET_BF16)
    bnrelu_kernel<bf16_t><<<g, 256, 0, (hipStream_t)stream>>>((const bf16_t*)y->ptr, P, y->c, y->ctot, y->coff,
                                                            scale, shift, (bf16_t*)out->ptr, out->ctot, out->coff);
  else
    bnrelu_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>((const float*)y->ptr, P, y->c, y->ctot, y->coff,
                                                           scale, shift, (float*)out->ptr, out->ctot, out->coff);
  EUNET_LAUNCH_CHECK("bnrelu");
  return EUNET_OK;
}

int eunet_bnrelu_pool(const eunet_act* y, const float* scale, const float* shift, const eunet_act* act,
                      const eunet_act* pooled, void* stream) {
  EUNET_REQUIRE(act_ok(y) && act_ok(pooled) && scale && shift && vec_ok(y) && vec_ok(pooled),
                "bnrelu_pool: bad args");
  EUNET_REQUIRE(y->h % 2 == 0 && y->w % 2 == 0, "bnrelu_pool: H and W must be even");
  EUNET_REQUIRE(pooled->h == y->h / 2 && pooled->w == y->w / 2 && pooled->c == y->c && pooled->n == y->n,
                "bnrelu_pool: pooled shape");
  if (act) EUNET_REQUIRE(act_ok(act) && vec_ok(act) && act->h == y->h && act->w == y->w && act->c == y->c,
                         "bnrelu_pool: act shape");
  const int E = e16(y->dtype);
  const long long total = (long long)y->n * (y->h / 2) * (y->w / 2) * (y->c / E);
  const unsigned g = (unsigned)((total + 255) / 256);
  if (y->dtype == EUNET_BF16)
    bnrelu_pool_kernel<bf16_t><<<g, 256, 0, (hipStream_t)stream>>>(
        (const bf16_t*)y->ptr, y->n, y->h, y->w, y->c, y->ctot, y->coff, scale, shift,
        act ? (bf16_t*)act->ptr : nullptr, act ? act->ctot : 0, act ? act->coff : 0, (bf16_t*)pooled->ptr,
        pooled->ctot, pooled->coff);
  else
    bnrelu_pool_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>(
        (const float*)y->ptr, y->n, y->h, y->w, y->c, y->ctot, y->coff, scale, shift,
        act ? (float*)act->ptr : nullptr, act ? act->ctot : 0, act ? act->coff : 0, (float*)pooled->ptr,
        pooled->ctot, pooled->coff);
  EUNET_LAUNCH_CHECK("bnrelu_pool");
  return EUNET_OK;
}

int eunet_bnrelu_upsample(const eunet_act* y, const float* scale, const float* shift, const eunet_act* out,
                          void* stream) {
  EUNET_REQUIRE(act_ok(y) && act_ok(out) && scale && shift && vec_ok(y) && vec_ok(out), "bnrelu_upsample: bad args");
  EUNET_REQUIRE(out->h == 2 * y->h && out->w == 2 * y->w && out->c == y->c && out->n == y->n &&
                    out->dtype == y->dtype,
                "bnrelu_upsample: shape");
  const int E = e16(y->dtype);
  // rows per thread: 8, or 4 when the grid would have fewer than 4096 blocks (measured: 2 rows per thread is slower)
  int rpt = 8;
  auto blocks = [&](int r) { return ((long long)y->n * cdiv(y->h, r) * ((y->w + 1) / 2) * (y->c / E) + 255) / 256; };
  if (blocks(rpt) < 4096) rpt = 4;
  const unsigned g = (unsigned)blocks(rpt);
  if (y->dtype == EUNET_BF16)
    bnrelu_up_rows_kernel<bf16_t><<<g, 256, 0, (hipStream_t)stream>>>(
        (const bf16_t*)y->ptr, y->n, y->h, y->w, y->c, y->ctot, y->coff, scale, shift, (bf16_t*)out->ptr,
        out->ctot, out->coff, rpt);
  else
    bnrelu_up_rows_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>(
        (const float*)y->ptr, y->n, y->h, y->w, y->c, y->ctot, y->coff, scale, shift, (float*)out->ptr,
        out->ctot, out->coff, rpt);
  EUNET_LAUNCH_CHECK("bnrelu_upsample");
  return EUNET_OK;
}

int eunet_bnrelu_conv1x1(const eunet_act* y, const float* scale, const float* shift, const float* w, const float* b,
                         int k, float* z, void* stream) {
  EUNET_REQUIRE(act_ok(y) && vec_ok(y) && scale && shift && w && b && z && k >= 1 && k <= 3,
                "bnrelu_conv1x1: bad args");
  EUNET_REQUIRE(y->c <= 128 && y->c % 8 == 0, "bnrelu_conv1x1: needs C <= 128, C %% 8 == 0");
  const long long P = (long long)y->n * y->h * y->w;
  const long long nb = (P + 32 * C1X_PX - 1) / (32 * C1X_PX);
  const unsigned g = (unsigned)(nb < 8192 ? nb : 8192);
  if (y->dtype == EUNET_BF16)
    bnrelu_conv1x1_kernel<bf16_t><<<g, 256, 0, (hipStream_t)stream>>>((const bf16_t*)y->ptr, P, y->c, y->ctot,
                                                                        y->coff, scale, shift, w, b, k, z);
  else
    bnrelu_conv1x1_kernel<float><<<g, 256, 0, (hipStream_t)stream>>>((const float*)y->ptr, P, y->c, y->ctot,
                                                                       y->coff, scale, shift, w, b, k, z);
  EUNET_LAUNCH_CHECK("bnrelu_conv1x1");
  return EUNET_OK;
}

int eunet_bn_bwd_tiles(const eunet_act* y, int* tiles) {
  EUNET_REQUIRE(act_ok(y) && tiles, "bn_bwd_tiles: bad args");
  const long long P = (long long)y->n * y->h * y->w;
  *tiles = (int)((P + bwd_pix(P) - 1) / bwd_pix(P));
  return EUNET_OK;
}

int eunet_bn_bwd_reduce(const eunet_act* g, const eunet_act* y, const float* mean, const float* invstd,
                        const float* scale, const float* shift, float* part, void* stream) {
  EUNET_REQUIRE(act_ok(g) && act_ok(y) && vec_ok(g) && vec_ok(y) && mean && invstd && scale && shift && part,
                "bn_bwd_reduce: bad args");
  EUNET_REQUIRE(g->dtype == y->dtype && g->c == y->c && g->n == y->n && g->h == y->h && g->w == y->w,
                "bn_bwd_reduce: shape mismatch");
  EUNET_REQUIRE(y->c / e16(y->dtype) <= NT, "bn_bwd_reduce: too many channels");
  const long long P = (long long)y->n * y->h * y->w;
  const int tpix = (int)bwd_pix(P);
  const unsigned tiles = (unsigned)((P + tpix - 1) / tpix);
  if (y->dtype == EUNET_BF16)
    bn_bwd_reduce_kernel<bf16_t><<<tiles, NT, 0, (hipStream_t)stream>>>(
        (const bf16_t*)g->ptr, g->ctot, g->coff, (const bf16_t*)y->ptr, y->ctot, y->coff, P, y->c, mean, invstd,
        scale, shift, part, tpix);
  else
    bn_bwd_reduce_kernel<float><<<tiles, NT, 0, (hipStream_t)stream>>>(
        (const float*)g->ptr, g->ctot, g->coff, (const float*)y->ptr, y->ctot, y->coff, P, y->c, mean, invstd,
        scale, shift, part, tpix);
  EUNET_LAUNCH_CHECK("bn_bwd_reduce");
  return EUNET_OK;
}

int eunet_colsum_ws_bytes(int rows, int cols, size_t* bytes) {
  EUNET_REQUIRE(bytes && rows > 0 && cols > 0, "colsum_ws_bytes: bad args");
  *bytes = eunet_colsum_ws(rows, cols);
  return EUNET_OK;
}

int eunet_colsum(const float* part, int rows, int cols, float* out, void* ws, void* stream) {
  return eunet_colsum_ld(part, rows, cols, cols, out, ws, (hipStream_t)stream);
}

int eunet_colsum_split(const float* part, int rows, int cols, int split, float* out_lo, float* out_hi, void* ws,
                       void* stream) {
  EUNET_REQUIRE(out_hi && split > 0 && split < cols, "colsum_split: bad split");
  return eunet_colsum_ld(part, rows, cols, cols, out_lo, ws, (hipStream_t)stream, split, out_hi);
}

static int bn_bwd_apply_launch(const eunet_act* g, const eunet_act* y, const float* mean, const float* invstd,
                               const float* scale, const float* shift, const float* dbeta, const float* dgamma,
                               const float* coef, const eunet_act* gy, void* stream) {
  EUNET_REQUIRE(act_ok(g) && act_ok(y) && act_ok(gy) && vec_ok(g) && vec_ok(y) && vec_ok(gy),
                "bn_bwd_apply: bad tensors");
  EUNET_REQUIRE(coef || (mean && invstd && scale && shift && dbeta && dgamma), "bn_bwd_apply: null stats");
  EUNET_REQUIRE(g->dtype == y->dtype && gy->dtype == y->dtype && g->c == y->c && gy->c == y->c,
                "bn_bwd_apply: mismatch");
  const long long P = (long long)y->n * y->h * y->w;
  const int U = y->c / e16(y->dtype);
  EUNET_REQUIRE(U <= 256, "bn_bwd_apply: at most 256 channel units (C <= 256 x %d)", e16(y->dtype));
  const int bs = (256 / U) * U;
  const long long nb = (P * U + bs - 1) / bs;
  const unsigned gr = (unsigned)(nb < 4096 ? nb : 4096);
#define EUNET_APPLY_LAUNCH(TT, CF)                                                                              \
  bn_bwd_apply_kernel<TT, TT, CF><<<gr, bs, 0, (hipStream_t)stream>>>(                                        \
      (const TT*)g->ptr, g->ctot, g->coff, (const TT*)y->ptr, y->ctot, y->coff, P, y->c, mean, invstd, scale, \
      shift, dbeta, dgamma, (TT*)gy->ptr, gy->ctot, gy->coff, coef)
  if (y->dtype == EUNET_BF16) {
    if (coef) EUNET_APPLY_LAUNCH(bf16_t, true);
    else EUNET_APPLY_LAUNCH(bf16_t, false);
  } else {
    if (coef) EUNET_APPLY_LAUNCH(float, true);
    else EUNET_APPLY_LAUNCH(float, false);
  }
#undef EUNET_APPLY_LAUNCH
  EUNET_LAUNCH_CHECK("bn_bwd_apply");
  return EUNET_OK;
}

int eunet_bn_bwd_apply(const eunet_act* g, const eunet_act* y, const float* mean, const float* invstd,
                       const float* scale, const float* shift, const float* dbeta, const float* dgamma,
                       const eunet_act* gy, void* stream) {
  EUNET_REQUIRE(mean && invstd && scale && shift && dbeta && dgamma, "bn_bwd_apply: null stats");
  return bn_bwd_apply_launch(g, y, mean, invstd, scale, shift, dbeta, dgamma, nullptr, gy, stream);
}

int eunet_bn_bwd_apply_1x1(const eunet_act* y, const float* w, int k, const float* gz, const float* mean,
                           const float* invstd, const float* scale, const float* shift, const float* dbeta,
                           const float* dgamma, const eunet_act* gy, void* stream) {
  EUNET_REQUIRE(act_ok(y) && act_ok(gy) && vec_ok(y) && vec_ok(gy) && w && gz && mean && invstd && scale && shift &&
                    dbeta && dgamma,
                "bn_bwd_apply_1x1: bad args");
  EUNET_REQUIRE(k >= 1 && k <= 3 && gy->dtype == y->dtype && gy->c == y->c && gy->n == y->n && gy->h == y->h &&
                    gy->w == y->w,
                "bn_bwd_apply_1x1: K <= 3, gy like y");
  const long long P = (long long)y->n * y->h * y->w;
  const int U = y->c / e16(y->dtype);
  EUNET_REQUIRE(U <= 256, "bn_bwd_apply_1x1: at most 256 channel units");
  const int bs = (256 / U) * U;
  const long long nb = (P * U + bs - 1) / bs;
  const unsigned gr = (unsigned)(nb < 4096 ? nb : 4096);
  if (y->dtype == EUNET_BF16)
    bn_bwd_apply_1x1_kernel<bf16_t><<<gr, bs, 0, (hipStream_t)stream>>>(
        (const bf16_t*)y->ptr, y->ctot, y->coff, P, y->c, w, k, gz, mean, invstd, scale, shift, dbeta, dgamma,
        (bf16_t*)gy->ptr, gy->ctot, gy->coff);
  else
    bn_bwd_apply_1x1_kernel<float><<<gr, bs, 0, (hipStream_t)stream>>>(
        (const float*)y->ptr, y->ctot, y->coff, P, y->c, w, k, gz, mean, invstd, scale, shift, dbeta, dgamma,
        (float*)gy->ptr, gy->ctot, gy->coff);
  EUNET_LAUNCH_CHECK("bn_bwd_apply_1x1");
  return EUNET_OK;
}

int eunet_bn_bwd_apply_coef(const eunet_act* g, const eunet_act* y, const float* coef, const eunet_act* gy,
                            void* stream) {
  EUNET_REQUIRE(coef, "bn_bwd_apply_coef: null coef");
  return bn_bwd_apply_launch(g, y, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, coef, gy, stream);
}

int eunet_bn_bwd_coef(const float* mean, const float* invstd, const float* scale, const float* shift,
                      const float* dbeta, const float* dgamma, long long count, int C, float* coef, void* stream) {
  EUNET_REQUIRE(mean && invstd && scale && shift && dbeta && dgamma && coef && count > 0 && C > 0,
                "bn_bwd_coef: bad args");
  bn_bwd_coef_kernel<<<(C + 255) / 256, 256, 0, (hipStream_t)stream>>>(mean, invstd, scale, shift, dbeta, dgamma,
                                                                       1.f / (float)count, C, coef);
  EUNET_LAUNCH_CHECK("bn_bwd_coef");
  return EUNET_OK;
}

int eunet_pool_bwd_add(const eunet_act* act, const eunet_act* gpool, const eunet_act* gskip, const eunet_act* gout,
                       void* stream) {
  EUNET_REQUIRE(act_ok(act) && act_ok(gpool) && act_ok(gout) && vec_ok(act) && vec_ok(gpool) && vec_ok(gout),
                "pool_bwd_add: bad tensors");
  if (gskip) EUNET_REQUIRE(act_ok(gskip) && vec_ok(gskip) && gskip->c == act->c, "pool_bwd_add: gskip");
  EUNET_REQUIRE(gpool->h * 2 == act->h && gpool->w * 2 == act->w && gout->h == act->h && gout->w == act->w &&
                    gpool->c == act->c && gout->c == act->c,
                "pool_bwd_add: shapes");
  const int E = e16(act->dtype);
  const long long total = (long long)act->n * (act->h / 2) * (act->w / 2) * (act->c / E);
  const unsigned gr = (unsigned)((total + 255) / 256);
#define PBA(T)                                                                                                  \
  pool_bwd_add_kernel<T><<<gr, 256, 0, (hipStream_t)stream>>>(                                                  \
      (const T*)act->ptr, act->ctot, act->coff, (const T*)gpool->ptr, gpool->ctot, gpool->coff,                 \
      gskip ? (const T*)gskip->ptr : nullptr, gskip ? gskip->ctot : 0, gskip ? gskip->coff : 0, (T*)gout->ptr, \
      gout->ctot, gout->coff, act->n, act->h, act->w, act->c, BnRed{})
  if (act->dtype == EUNET_BF16) PBA(bf16_t);
  else PBA(float);
#undef PBA
  EUNET_LAUNCH_CHECK("pool_bwd_add");
  return EUNET_OK;
}

int eunet_upsample_bwd(const eunet_act* ghi, const eunet_act* glo, void* stream) {
  EUNET_REQUIRE(act_ok(ghi) && act_ok(glo), "upsample_bwd: bad tensors");
  EUNET_REQUIRE(ghi->h == 2 * glo->h && ghi->w == 2 * glo->w && ghi->c == glo->c && ghi->n == glo->n,
                "upsample_bwd: shapes");
  if (ghi->dtype == EUNET_F32 && glo->dtype == EUNET_F32 && ghi->ctot == ghi->c && glo->ctot == glo->c &&
      ghi->c <= 4 && ghi->coff == 0 && glo->coff == 0) {
    const long long total = (long long)glo->n * glo->h * glo->w;
    if (ghi->c == 2)
      up_bwd_k2_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
          (const float2*)ghi->ptr, (float2*)glo->ptr, glo->n, glo->h, glo->w);
    else
      up_bwd_small_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
          (const float*)ghi->ptr, (float*)glo->ptr, glo->n, glo->h, glo->w, glo->c);
    EUNET_LAUNCH_CHECK("upsample_bwd_small");
    return EUNET_OK;
  }
  EUNET_REQUIRE(vec_ok(ghi) && vec_ok(glo) && ghi->dtype == glo->dtype, "upsample_bwd: vector layout");
  const int E = e16(ghi->dtype);
  const long long total = (long long)glo->n * ((glo->h + UP_R - 1) / UP_R) * ((glo->w + 1) / 2) * (glo->c / E);
  const unsigned gr = (unsigned)((total + 255) / 256);
  if (ghi->dtype == EUNET_BF16)
    up_bwd_rows_kernel<bf16_t, bf16_t><<<gr, 256, 0, (hipStream_t)stream>>>(
        (const bf16_t*)ghi->ptr, ghi->ctot, ghi->coff, (bf16_t*)glo->ptr, glo->ctot, glo->coff, glo->n, glo->h,
        glo->w, glo->c, BnRed{});
  else
    up_bwd_rows_kernel<float, float><<<gr, 256, 0, (hipStream_t)stream>>>(
        (const float*)ghi->ptr, ghi->ctot, ghi->coff, (float*)glo->ptr, glo->ctot, glo->coff, glo->n, glo->h,
        glo->w, glo->c, BnRed{});
  EUNET_LAUNCH_CHECK("upsample_bwd");
  return EUNET_OK;
}

// ---- gradient producers with the BN-backward reduction of the block they feed fused in ----
namespace {
// block size of the fused BN-backward reductions: the block's threads must cover whole channel units
// (a thread's unit is fixed across the grid-stride loop) -- 256 threads, or 192 for the channel counts
// of base 96 (96 / 192 / 384 / 768 channels: 12 / 24 / 48 / 96 bf16 units); 0: not fusable
int bnr_block(const eunet_act* g) {
  const int U = g->c / e16(g->dtype);
  return U > 0 && NT % U == 0 ? NT : (U > 0 && 192 % U == 0 ? 192 : 0);
}
bool bnr_ok(const eunet_act* g, const eunet_act* y) {
  return act_ok(y) && vec_ok(y) && y->dtype == g->dtype && y->n == g->n && y->h == g->h && y->w == g->w &&
         y->c == g->c && bnr_block(g) > 0;
}
long long pool_threads(const eunet_act* gout) {
  return (long long)gout->n * (gout->h / 2) * (gout->w / 2) * (gout->c / e16(gout->dtype));
}
// fused-reduction grid, which is also the number of partial rows: at most cap blocks (each thread
// then covers several outputs).  Measured: the max-pool adjoint prefers 2048 (fewer rows to write
// and sum), the upsample adjoint, with more work per output, 8192 (more loads in flight).
int bnr_grid(long long threads, int cap, int block) { return (int)std::min<long long>((threads + block - 1) / block, cap); }
long long up_threads(const eunet_act* glo) {
  return (long long)glo->n * ((glo->h + UP_R - 1) / UP_R) * ((glo->w + 1) / 2) * (glo->c / e16(glo->dtype));
}
}  // namespace

int eunet_pool_bwd_add_bnr_rows(const eunet_act* gout, int* rows) {
  EUNET_REQUIRE(act_ok(gout) && rows, "pool_bwd_add_bnr_rows: bad args");
  const int bs = bnr_block(gout);
  *rows = bs > 0 ? bnr_grid(pool_threads(gout), 2048, bs) : 0;
  return EUNET_OK;
}

int eunet_pool_bwd_add_bnr(const eunet_act* act, const eunet_act* gpool, const eunet_act* gskip,
                           const eunet_act* gout, const eunet_act* y, const float* mean, const float* invstd,
                           const float* scale, const float* shift, float* part, void* stream) {
  EUNET_REQUIRE(act_ok(act) && vec_ok(act), "pool_bwd_add_bnr: bad act");
  eunet_act none;
  if (!gout) {  // reduce only (the apply recomputes gout: eunet_bn_bwd_apply_pool)
    none = *act;
    none.ptr = nullptr;
    none.ctot = act->c;
    none.coff = 0;
    gout = &none;
  }
  EUNET_REQUIRE(act_ok(gpool) && vec_ok(gpool) && (!gout->ptr || (act_ok(gout) && vec_ok(gout))),
                "pool_bwd_add_bnr: bad tensors");
  if (gskip) EUNET_REQUIRE(act_ok(gskip) && vec_ok(gskip) && gskip->c == act->c, "pool_bwd_add_bnr: gskip");
  EUNET_REQUIRE(gpool->h * 2 == act->h && gpool->w * 2 == act->w && gout->h == act->h && gout->w == act->w &&
                    gpool->c == act->c && gout->c == act->c,
                "pool_bwd_add_bnr: shapes");
  EUNET_REQUIRE(bnr_ok(gout, y) && mean && invstd && scale && shift && part,
                "pool_bwd_add_bnr: y / BN args (and 256 or 192 %% channel units == 0)");
  const BnRed br{y->ptr, y->ctot, y->coff, mean, invstd, scale, shift, part};
  const int bs = bnr_block(gout);
  const unsigned gr = (unsigned)bnr_grid(pool_threads(gout), 2048, bs);
#define PBA(T)                                                                                                  \
  pool_bwd_add_kernel<T, true><<<gr, bs, 0, (hipStream_t)stream>>>(                                             \
      (const T*)act->ptr, act->ctot, act->coff, (const T*)gpool->ptr, gpool->ctot, gpool->coff,                 \
      gskip ? (const T*)gskip->ptr : nullptr, gskip ? gskip->ctot : 0, gskip ? gskip->coff : 0, (T*)gout->ptr, \
      gout->ctot, gout->coff, act->n, act->h, act->w, act->c, br)
  if (act->dtype == EUNET_BF16) PBA(bf16_t);
  else PBA(float);
#undef PBA
  EUNET_LAUNCH_CHECK("pool_bwd_add_bnr");
  return EUNET_OK;
}

int eunet_bn_bwd_apply_pool(const eunet_act* gpool, const eunet_act* gskip, const eunet_act* y, const float* mean,
                            const float* invstd, const float* scale, const float* shift, const float* dbeta,
                            const float* dgamma, const eunet_act* gy, void* stream) {
  EUNET_REQUIRE(act_ok(gpool) && vec_ok(gpool) && act_ok(y) && vec_ok(y) && act_ok(gy) && vec_ok(gy) && mean &&
                    invstd && scale && shift && dbeta && dgamma,
                "bn_bwd_apply_pool: bad args");
  if (gskip) EUNET_REQUIRE(act_ok(gskip) && vec_ok(gskip) && gskip->c == y->c && gskip->n == y->n &&
                               gskip->h == y->h && gskip->w == y->w && gskip->dtype == y->dtype,
                           "bn_bwd_apply_pool: gskip");
  EUNET_REQUIRE(gpool->h * 2 == y->h && gpool->w * 2 == y->w && gpool->n == y->n && gpool->c == y->c &&
                    gpool->dtype == y->dtype && gy->n == y->n && gy->h == y->h && gy->w == y->w && gy->c == y->c &&
                    gy->dtype == y->dtype,
                "bn_bwd_apply_pool: shapes (even H and W: every pixel in a 2x2 window)");
  const int bs = bnr_block(y);
  EUNET_REQUIRE(bs > 0, "bn_bwd_apply_pool: 256 or 192 %% channel units == 0");
  const long long th = pool_threads(y);
  const unsigned gr = (unsigned)std::min<long long>((th + bs - 1) / bs, 8192);
#define BAP(T)                                                                                                       \
  bn_bwd_apply_pool_kernel<T><<<gr, bs, 0, (hipStream_t)stream>>>(                                                   \
      (const T*)gpool->ptr, gpool->ctot, gpool->coff, gskip ? (const T*)gskip->ptr : nullptr, gskip ? gskip->ctot : 0, \
      gskip ? gskip->coff : 0, (const T*)y->ptr, y->ctot, y->coff, mean, invstd, scale, shift, dbeta, dgamma,          \
      (T*)gy->ptr, gy->ctot, gy->coff, y->n, y->h, y->w, y->c)
  if (y->dtype == EUNET_BF16) BAP(bf16_t);
  else BAP(float);
#undef BAP
  EUNET_LAUNCH_CHECK("bn_bwd_apply_pool");
  return EUNET_OK;
}

int eunet_upsample_bwd_bnr_rows(const eunet_act* glo, int* rows) {
  EUNET_REQUIRE(act_ok(glo) && rows, "upsample_bwd_bnr_rows: bad args");
  const int bs = vec_ok(glo) ? bnr_block(glo) : 0;
  *rows = bs > 0 ? bnr_grid(up_threads(glo), 8192, bs) : 0;
  return EUNET_OK;
}

int eunet_upsample_bwd_bnr(const eunet_act* ghi, const eunet_act* glo, const eunet_act* y, const float* mean,
                           const float* invstd, const float* scale, const float* shift, float* part, void* stream) {
  EUNET_REQUIRE(act_ok(ghi) && act_ok(glo) && vec_ok(ghi) && vec_ok(glo) && ghi->dtype == glo->dtype,
                "upsample_bwd_bnr: bad tensors");
  EUNET_REQUIRE(ghi->h == 2 * glo->h && ghi->w == 2 * glo->w && ghi->c == glo->c && ghi->n == glo->n,
                "upsample_bwd_bnr: shapes");
  EUNET_REQUIRE(bnr_ok(glo, y) && mean && invstd && scale && shift && part,
                "upsample_bwd_bnr: y / BN args (and 256 or 192 %% channel units == 0)");
  const BnRed br{y->ptr, y->ctot, y->coff, mean, invstd, scale, shift, part};
  const int bs = bnr_block(glo);
  const unsigned gr = (unsigned)bnr_grid(up_threads(glo), 8192, bs);
  if (ghi->dtype == EUNET_BF16)
    up_bwd_rows_kernel<bf16_t, bf16_t, true><<<gr, bs, 0, (hipStream_t)stream>>>(
        (const bf16_t*)ghi->ptr, ghi->ctot, ghi->coff, (bf16_t*)glo->ptr, glo->ctot, glo->coff, glo->n, glo->h,
        glo->w, glo->c, br);
  else
    up_bwd_rows_kernel<float, float, true><<<gr, bs, 0, (hipStream_t)stream>>>(
        (const float*)ghi->ptr, ghi->ctot, ghi->coff, (float*)glo->ptr, glo->ctot, glo->coff, glo->n, glo->h,
        glo->w, glo->c, br);
  EUNET_LAUNCH_CHECK("upsample_bwd_bnr");
  return EUNET_OK;
}

int eunet_conv1x1_bwd_tiles(const eunet_act* y, int* tiles) {
  EUNET_REQUIRE(act_ok(y) && tiles, "conv1x1_bwd_tiles: bad args");
  *tiles = (int)(((long long)y->n * y->h * y->w + C1X_PIX - 1) / C1X_PIX);
  return EUNET_OK;
}

int eunet_conv1x1_bwd(const eunet_act* y, const float* scale, const float* shift, const float* w, int k,
                      const float* gz, const eunet_act* gact, float* part, void* stream) {
  EUNET_REQUIRE(act_ok(y) && act_ok(gact) && vec_ok(y) && vec_ok(gact) && scale && shift && w && gz && part,
                "conv1x1_bwd: bad args");
  EUNET_REQUIRE(k >= 1 && k <= 3 && y->c <= 128 && y->c % 8 == 0 && gact->c == y->c && gact->dtype == y->dtype,
                "conv1x1_bwd: K<=3, C<=128, C%8==0");
  const long long P = (long long)y->n * y->h * y->w;
  const unsigned tiles = (unsigned)((P + C1X_PIX - 1) / C1X_PIX);
  if (y->dtype == EUNET_BF16)
    C1X_LAUNCH(conv1x1_bwd_kernel, bf16_t, false, ((const bf16_t*)y->ptr, P, y->c, y->ctot,
                                                                        y->coff, scale, shift, w, k, gz,
                                                                        (bf16_t*)gact->ptr, gact->ctot, gact->coff,
                                                                        part, nullptr, nullptr, nullptr));
  else
    C1X_LAUNCH(conv1x1_bwd_kernel, float, false, ((const float*)y->ptr, P, y->c, y->ctot,
                                                                       y->coff, scale, shift, w, k, gz,
                                                                       (float*)gact->ptr, gact->ctot, gact->coff,
                                                                       part, nullptr, nullptr, nullptr));
  EUNET_LAUNCH_CHECK("conv1x1_bwd");
  return EUNET_OK;
}

int eunet_conv1x1_bwd_bnr(const eunet_act* y, const float* scale, const float* shift, const float* w, int k,
                          const float* gz, const eunet_act* gact, float* part, const float* mean, const float* invstd,
                          float* bn_part, void* stream) {
  EUNET_REQUIRE(act_ok(y) && vec_ok(y) && (!gact || (act_ok(gact) && vec_ok(gact))) && scale && shift && w && gz &&
                    part,
                "conv1x1_bwd: bad args");
  EUNET_REQUIRE(k >= 1 && k <= 3 && y->c <= 128 && y->c % 8 == 0 &&
                    (!gact || (gact->c == y->c && gact->dtype == y->dtype)),
                "conv1x1_bwd: K<=3, C<=128, C%8==0");
  const eunet_act none{};
  if (!gact) gact = &none;  // (a null ptr: the kernel reduces without storing)
  EUNET_REQUIRE(mean && invstd && bn_part, "conv1x1_bwd_bnr: BN args");
  const long long P = (long long)y->n * y->h * y->w;
  const unsigned tiles = (unsigned)((P + C1X_PIX - 1) / C1X_PIX);
  if (y->dtype == EUNET_BF16)
    C1X_LAUNCH(conv1x1_bwd_kernel, bf16_t, true, ((const bf16_t*)y->ptr, P, y->c, y->ctot,
                                                                        y->coff, scale, shift, w, k, gz,
                                                                        (bf16_t*)gact->ptr, gact->ctot, gact->coff,
                                                                        part, mean, invstd, bn_part));
  else
    C1X_LAUNCH(conv1x1_bwd_kernel, float, true, ((const float*)y->ptr, P, y->c, y->ctot,
                                                                       y->coff, scale, shift, w, k, gz,
                                                                       (float*)gact->ptr, gact->ctot, gact->coff,
                                                                       part, mean, invstd, bn_part));
  EUNET_LAUNCH_CHECK("conv1x1_bwd_bnr");
  return EUNET_OK;
}

}  // extern "C"
