// Conv2d 3x3 / stride 1 / padding 1 on NHWC activations, MFMA implicit GEMM.
//
// Reference call sites: models.py:219,222 (_conv_block, every DoubleConv of
// BasicUNet models.py:203-211) and their autograd (dgrad / wgrad).
//
// Forward (and dgrad, which is the same kernel on W'[ci][co][8-t]):
//   GEMM  M = output pixels (8x32 tile per block), N = Cout (64 per block),
//         K = 9 taps x Cin, consumed one Cin chunk (KC channels) at a time.
//   The chunk's input halo tile [(8+2) x (32+2) px][KC] is staged once in LDS
//   and re-read by all 9 taps (no im2col, 1.4x halo over-read instead of 9x),
//   together with the chunk's weights [64 co][9 taps][KC].
//   bf16: v_mfma_f32_16x16x32_bf16 (fp32 accumulate), KC = 32.
//   f32 : v_mfma_f32_16x16x4_f32 (exact fp32 fma chain), KC = 16.
//   Both read 16-B fragments: lane l takes pixel (l&15) / channel quarter (l>>4);
//   LDS images are [quarter][pixel|co*9+tap][16 B] (conflict-free fragment reads).
//   Optional operand transform relu(x*scale+shift) = the preceding BN+ReLU,
//   applied when the staged registers are written to LDS (zero padding after).
//   Epilogue: + bias, store, and per-tile BatchNorm partials (sum, M2) from the
//   fp32 accumulators (two-pass in registers -> Chan-combinable).
//
// Wgrad: dW[co][t][ci] = sum_p dY[p][co] * X~[p+d_t][ci], pixels are the GEMM K.
//   Block = (pixel-tile split, 64 co, KC ci); dY tile and X halo staged in LDS;
//   bf16 fragments (8 consecutive pixels) come from ds_read_b64_tr_b16.
#include "common.h"

namespace {

constexpr int TH = 8, TW = 32;            // output tile (pixels)
constexpr int HW_ = TW + 2, HH_ = TH + 2;  // halo tile
constexpr int HPX = HH_ * HW_;            // 340 halo pixels
constexpr int HPXP = 352;                 // padded plane (multiple of 16)
constexpr int BN = 64;                    // output channels per block
constexpr int NTHR = 256;
constexpr int A_UNITS = 4 * HPX;          // 16-B units in one halo chunk
constexpr int A_ITERS = (A_UNITS + NTHR - 1) / NTHR;  // 6
constexpr int B_UNITS = 4 * BN * 9;       // 2304
constexpr int B_ITERS = B_UNITS / NTHR;   // 9
constexpr int A_LDS_BYTES = 4 * HPXP * 16;  // 22528
constexpr int B_LDS_BYTES = B_UNITS * 16;   // 36864

template <typename T> struct KCh { static constexpr int v = 4 * Vec16<T>::N; };  // 16 (f32) / 32 (bf16)

struct FwdArgs {
  const void* x; int N, H, W, xct, xco, cin;
  const float* isc; const float* ish;
  const void* wp; int cout_pad, nkc;
  const float* bias;
  void* y; int yct, yco, cout;
  float* stats; int tx, ty, ntiles;
};

// stage one halo unit (pixel hp, quarter q) of chunk kc into registers
template <typename T>
__device__ __forceinline__ uint4 load_halo_unit(const FwdArgs& a, int n, int y0, int x0, int id, int kc,
                                                bool& ok) {
  constexpr int E = Vec16<T>::N, KC = KCh<T>::v;
  const int hp = id >> 2, q = id & 3;
  const int hy = hp / HW_, hx = hp - hy * HW_;
  const int yy = y0 + hy - 1, xx = x0 + hx - 1;
  const int c = kc * KC + q * E;
  ok = (id < A_UNITS) && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W && c < a.cin;
  if (!ok) return make_uint4(0, 0, 0, 0);
  const T* p = (const T*)a.x + (((long long)(n * a.H + yy) * a.W + xx) * a.xct + a.xco + c);
  return *(const uint4*)p;
}

template <typename T>
__device__ __forceinline__ void store_halo_unit(const FwdArgs& a, char* lds, int id, int kc, uint4 v, bool ok) {
  constexpr int E = Vec16<T>::N, KC = KCh<T>::v;
  if (id >= A_UNITS) return;
  const int hp = id >> 2, q = id & 3;
  if (ok && a.isc != nullptr) {
    const int c = kc * KC + q * E;
    float f[E];
    Vec16<T>::unpack(v, f);
#pragma unroll
    for (int j = 0; j < E; ++j) f[j] = fmaxf(fmaf(f[j], a.isc[c + j], a.ish[c + j]), 0.f);
    v = Vec16<T>::pack(f);
  }
  *(uint4*)(lds + (q * HPXP + hp) * 16) = v;
}

// v2: 512 threads = 8 waves (2 per SIMD); wave w computes output row w of the
// 8x32 tile (32 px x 64 co = 2x4 MFMA tiles).  LDS is double-buffered: the next
// chunk's global loads go to registers before the MFMAs of the current chunk
// and are written (with the BN+ReLU transform) into the other buffer right
// after them, so there is ONE barrier per K-chunk.  The epilogue stages the
// tile through LDS and stores whole 16-byte vectors.
constexpr int FT = 512;
constexpr int FA_ITERS = (A_UNITS + FT - 1) / FT;  // 3
constexpr int FB_ITERS = B_UNITS / FT;             // 4 full rounds ...
constexpr int FB_TAIL = B_UNITS - FB_ITERS * FT;   // ... + 256 units for threads 0..255
constexpr int STAGE_BYTES = A_LDS_BYTES + B_LDS_BYTES;  // 59392
constexpr int OUT_LD = 68;                              // fp32 row stride of the output staging tile
constexpr int FWD_LDS = 2 * STAGE_BYTES;                // 118784 (>= 256*68*4 + 2*8*64*4)

template <typename T>
__global__ __launch_bounds__(FT, 1) void conv3x3_fwd_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tile = blockIdx.x;
  const int tpi = a.tx * a.ty;
  const int n = tile / tpi, trem = tile - n * tpi;
  const int y0 = (trem / a.tx) * TH, x0 = (trem % a.tx) * TW;
  const int co0 = blockIdx.y * BN;
  const int q = lane >> 4, li = lane & 15;

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  uint4 ra[FA_ITERS];
  bool rok[FA_ITERS];
  u32x4 rb[FB_ITERS];
  u32x4 rbt = (u32x4){0u, 0u, 0u, 0u};
  const u32x4* wp = (const u32x4*)a.wp;
  const bool tail = tid < FB_TAIL;

#define CONV_BUNIT(ID_, KC_) \
  wp[((long long)((KC_) * 4 + (ID_) / (BN * 9)) * a.cout_pad + co0) * 9 + (ID_) % (BN * 9)]
#define CONV_GLOAD(KC_)                                                                       \
  do {                                                                                        \
    _Pragma("unroll") for (int i = 0; i < FA_ITERS; ++i)                                      \
        ra[i] = load_halo_unit<T>(a, n, y0, x0, tid + i * FT, (KC_), rok[i]);                 \
    _Pragma("unroll") for (int i = 0; i < FB_ITERS; ++i) rb[i] = CONV_BUNIT(tid + i * FT, KC_); \
    if (tail) rbt = CONV_BUNIT(tid + FB_ITERS * FT, KC_);                                     \
  } while (0)
#define CONV_LWRITE(KC_, BUF_)                                                                \
  do {                                                                                        \
    char* As_ = smem + (BUF_) * STAGE_BYTES;                                                  \
    char* Bs_ = As_ + A_LDS_BYTES;                                                            \
    _Pragma("unroll") for (int i = 0; i < FA_ITERS; ++i)                                      \
        store_halo_unit<T>(a, As_, tid + i * FT, (KC_), ra[i], rok[i]);                       \
    _Pragma("unroll") for (int i = 0; i < FB_ITERS; ++i) *(u32x4*)(Bs_ + (tid + i * FT) * 16) = rb[i]; \
    if (tail) *(u32x4*)(Bs_ + (tid + FB_ITERS * FT) * 16) = rbt;                              \
  } while (0)

  CONV_GLOAD(0);
  CONV_LWRITE(0, 0);
  __syncthreads();
  for (int kc = 0; kc < a.nkc; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < a.nkc) CONV_GLOAD(kc + 1);
    const char* As = smem + cur * STAGE_BYTES;
    const char* Bs = As + A_LDS_BYTES;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - ky * 3;
      uint4 fa[2], fb[4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int hp = (wv + ky) * HW_ + mt * 16 + li + kx;
        fa[mt] = *(const uint4*)(As + (q * HPXP + hp) * 16);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) fb[nt] = *(const uint4*)(Bs + (q * (BN * 9) + (nt * 16 + li) * 9 + t) * 16);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          if constexpr (sizeof(T) == 2) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, fa[mt]), __builtin_bit_cast(bf16x8, fb[nt]), acc[mt][nt], 0, 0, 0);
          } else {
            const uint4 A_ = fa[mt], B_ = fb[nt];
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(A_.x), __uint_as_float(B_.x), acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(A_.y), __uint_as_float(B_.y), acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(A_.z), __uint_as_float(B_.z), acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(A_.w), __uint_as_float(B_.w), acc[mt][nt], 0, 0, 0);
          }
        }
    }
    if (kc + 1 < a.nkc) CONV_LWRITE(kc + 1, cur ^ 1);
    __syncthreads();
  }
#undef CONV_GLOAD
#undef CONV_LWRITE
#undef CONV_BUNIT

  // ---- epilogue: bias, BN partials, LDS-staged vector stores ---------------
  const int vh = min(TH, a.H - y0), vw = min(TW, a.W - x0);
  const bool rv = wv < vh;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int co = co0 + nt * 16 + li;
    const float bv = (a.bias != nullptr && co < a.cout) ? a.bias[co] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[mt][nt][i] += bv;
  }
  float* stage = (float*)smem;                              // [256 px][OUT_LD]
  float* red = (float*)(smem + TH * TW * OUT_LD * 4);       // [8][64] x 2
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int px = wv * TW + mt * 16 + q * 4 + i;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) stage[px * OUT_LD + nt * 16 + li] = acc[mt][nt][i];
    }
  if (a.stats != nullptr) {
    float s[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float v = 0.f;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) v += (rv && mt * 16 + q * 4 + i < vw) ? acc[mt][nt][i] : 0.f;
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      s[nt] = v;
    }
    if (q == 0)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) red[wv * 64 + nt * 16 + li] = s[nt];
    __syncthreads();
    const float cnt = (float)(vh * vw);
    float mb[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) t += red[w * 64 + nt * 16 + li];
      mb[nt] = t / cnt;
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float v = 0.f;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float d = acc[mt][nt][i] - mb[nt];
          v += (rv && mt * 16 + q * 4 + i < vw) ? d * d : 0.f;
        }
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      s[nt] = v;
    }
    if (q == 0)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) red[512 + wv * 64 + nt * 16 + li] = s[nt];
    __syncthreads();
    if (tid < 64 && co0 + tid < a.cout) {
      float sum = 0.f, m2 = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        sum += red[w * 64 + tid];
        m2 += red[512 + w * 64 + tid];
      }
      a.stats[((long long)tile * 2 + 0) * a.cout + co0 + tid] = sum;
      a.stats[((long long)tile * 2 + 1) * a.cout + co0 + tid] = m2;
    }
    if (blockIdx.y == 0 && tid == 0) a.stats[(long long)2 * a.cout * a.ntiles + tile] = cnt;
  } else {
    __syncthreads();
  }
  constexpr int E = Vec16<T>::N;
  constexpr int UPX = 64 / E;  // 16-byte units per pixel row of the tile
  T* yp = (T*)a.y;
#pragma unroll
  for (int j = 0; j < TH * TW * UPX / FT; ++j) {
    const int id = tid + j * FT;
    const int px = id / UPX, u = id - px * UPX;
    const int r = px / TW, c = px - r * TW;
    const int co = co0 + u * E;
    if (r < vh && c < vw && co < a.cout) {
      const float* sp = stage + px * OUT_LD + u * E;
      float f[E];
#pragma unroll
      for (int e = 0; e < E; ++e) f[e] = sp[e];
      const long long pix = (long long)(n * a.H + y0 + r) * a.W + x0 + c;
      *(uint4*)(yp + pix * a.yct + a.yco + co) = Vec16<T>::pack(f);
    }
  }
}

// ---------------------------------------------------------------------------
// weight packing: torch [Cout][Cin][3][3] fp32 -> [Cin_p/KC][4][Cout_p][9][E]
// transpose_flip: pack W'[o=ci][i=co][t] = W[co][ci][8-t] (dgrad operand)
// ---------------------------------------------------------------------------
template <typename T>
__global__ void pack_kernel(const float* w, int cout, int cin, int flip, T* wp, int cout_p, int cin_p) {
  constexpr int E = Vec16<T>::N, KC = KCh<T>::v;
  const long long total = (long long)cin_p * cout_p * 9;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= total) return;
  // id enumerates output elements in packed order
  const int e = (int)(id % E);
  long long r = id / E;
  const int t = (int)(r % 9); r /= 9;
  const int o = (int)(r % cout_p); r /= cout_p;
  const int qq = (int)(r % 4);
  const int kc = (int)(r / 4);
  const int i = kc * KC + qq * E + e;  // "input" channel of the GEMM
  // GEMM channels: o (output), i (input); torch roles depend on flip
  float v = 0.f;
  if (!flip) {
    if (o < cout && i < cin) v = w[((long long)o * cin + i) * 9 + t];
  } else {
    // o = torch ci, i = torch co
    if (o < cin && i < cout) v = w[((long long)i * cin + o) * 9 + (8 - t)];
  }
  Elem<T>::st(wp + id, v);
}

// ---------------------------------------------------------------------------
// wgrad
// ---------------------------------------------------------------------------
struct WgArgs {
  const void* x; int N, H, W, xct, xco, cin;
  const float* isc; const float* ish;
  const void* dy; int dct, dco, cout;
  float* dw; float* db;
  int tx, ty, ntiles, per_split;
};

template <typename T>
__global__ __launch_bounds__(NTHR, 1) void conv3x3_wgrad_kernel(WgArgs a) {
  constexpr int E = Vec16<T>::N, KC = KCh<T>::v;
  constexpr int DY_UNITS_PX = 64 / E;                 // 16-B units per pixel row of dY tile
  constexpr int DY_UNITS = TH * TW * DY_UNITS_PX;     // 2048 (bf16) / 4096 (f32)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* As = smem;                      // X halo [4][HPXP][16B]
  char* Ds = smem + A_LDS_BYTES;        // dY tile [256 px][64 co] T
  float* dbred = (float*)(Ds + TH * TW * 64 * sizeof(T));  // [4][64]

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int split = blockIdx.x, co0 = blockIdx.y * 64, kc = blockIdx.z;
  const int t_begin = split * a.per_split;
  const int t_end = min(a.ntiles, t_begin + a.per_split);
  const int tpi = a.tx * a.ty;

  FwdArgs fa;
  fa.x = a.x; fa.N = a.N; fa.H = a.H; fa.W = a.W; fa.xct = a.xct; fa.xco = a.xco; fa.cin = a.cin;
  fa.isc = a.isc; fa.ish = a.ish;

  constexpr int NACC = (sizeof(T) == 2) ? 18 : 9;
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int n = tile / tpi, trem = tile - n * tpi;
    const int y0 = (trem / a.tx) * TH, x0 = (trem % a.tx) * TW;
    __syncthreads();
    // stage X halo
#pragma unroll
    for (int i = 0; i < A_ITERS; ++i) {
      bool ok;
      const int id = tid + i * NTHR;
      uint4 v = load_halo_unit<T>(fa, n, y0, x0, id, kc, ok);
      store_halo_unit<T>(fa, As, id, kc, v, ok);
    }
    // stage dY tile
    for (int id = tid; id < DY_UNITS; id += NTHR) {
      const int px = id / DY_UNITS_PX, u = id - px * DY_UNITS_PX;
      const int r = px / TW, c = px - r * TW;
      const int yy = y0 + r, xx = x0 + c, co = co0 + u * E;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (yy < a.H && xx < a.W && co < a.cout)
        v = *(const uint4*)((const T*)a.dy + ((long long)(n * a.H + yy) * a.W + xx) * a.dct + a.dco + co);
      *(uint4*)(Ds + id * 16) = v;
    }
    __syncthreads();
    if (a.db != nullptr && kc == 0) {
      const T* d = (const T*)Ds;
      for (int px = wv; px < TH * TW; px += 4) dbacc += Elem<T>::ld(d + px * 64 + lane);
    }
    if constexpr (sizeof(T) == 2) {
      const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
      const int cw = wv * 16;
      for (int ks = 0; ks < TH; ++ks) {  // one output row = 32 pixels per k-step
        const int pxa = ks * TW + 8 * g + q4;
        const s16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, Ds + (pxa * 64 + cw + 4 * p4) * 2));
        const s16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, Ds + ((pxa + 4) * 64 + cw + 4 * p4) * 2));
        const bf16x8 af = cat_bf16x4(alo, ahi);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int ky = t / 3, kx = t - ky * 3;
          const int hp = (ks + ky) * HW_ + 8 * g + q4 + kx;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int qq = 2 * j + (p4 >> 1);
            const char* base = As + (qq * HPXP + hp) * 16 + (p4 & 1) * 8;
            const s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base));
            const s16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base + 4 * 16));
            const bf16x8 bf = cat_bf16x4(blo, bhi);
            acc[t * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[t * 2 + j], 0, 0, 0);
          }
        }
      }
    } else {
      const int kq = lane >> 4, i = lane & 15;
      const int cw = wv * 16;
      const float* d = (const float*)Ds;
      for (int ks = 0; ks < TH * TW / 4; ++ks) {
        const int px = ks * 4 + kq;
        const int r = px / TW, c = px - r * TW;
        const float av = d[px * 64 + cw + i];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int ky = t / 3, kx = t - ky * 3;
          const int hp = (r + ky) * HW_ + c + kx;
          const float bv = *(const float*)(As + ((i >> 2) * HPXP + hp) * 16 + (i & 3) * 4);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t], 0, 0, 0);
        }
      }
    }
  }

  // ---- write partials: dw[split][co][t][ci] -------------------------------
  const int g = lane >> 4, li = lane & 15;
  float* out = a.dw + (long long)split * a.cout * 9 * a.cin;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
#pragma unroll
    for (int j = 0; j < NACC / 9; ++j) {
      const int ci = kc * KC + j * 16 + li;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wv * 16 + g * 4 + e;
        if (co < a.cout && ci < a.cin) out[((long long)co * 9 + t) * a.cin + ci] = acc[t * (NACC / 9) + j][e];
      }
    }
  }
  if (a.db != nullptr && kc == 0) {
    __syncthreads();
    dbred[wv * 64 + lane] = dbacc;
    __syncthreads();
    if (tid < 64 && co0 + tid < a.cout)
      a.db[(long long)split * a.cout + co0 + tid] = dbred[tid] + dbred[64 + tid] + dbred[128 + tid] + dbred[192 + tid];
  }
}

// bf16 wgrad v2: block = (pixel-tile split, 64 co, 64 ci).  Wave w owns ci tile
// w (16 channels) for all 9 taps x 4 co tiles (36 accumulators), so one
// 32-pixel k-step costs 8 + 18 transposed fragment reads for 36 MFMAs.
constexpr int KCW = 64;                       // ci channels per wgrad block (bf16)
constexpr int WX_LDS = 8 * HPXP * 16;         // X halo [8 octants][HPXP][16 B]
constexpr int WD_LDS = TH * TW * 64 * 2;      // dY tile [256 px][64 co] bf16
constexpr int WG_LDS = WX_LDS + WD_LDS + 4 * 64 * 4;

__global__ __launch_bounds__(NTHR, 2) void conv3x3_wgrad_bf16_kernel(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Xs = smem;
  char* Ds = smem + WX_LDS;
  float* dbred = (float*)(Ds + WD_LDS);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int split = blockIdx.x, co0 = blockIdx.y * 64, kc = blockIdx.z;
  const int t_begin = split * a.per_split;
  const int t_end = min(a.ntiles, t_begin + a.per_split);
  const int tpi = a.tx * a.ty;
  const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;

  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[t][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;

  for (int tile = t_begin; tile < t_end; ++tile) {
    const int n = tile / tpi, trem = tile - n * tpi;
    const int y0 = (trem / a.tx) * TH, x0 = (trem % a.tx) * TW;
    __syncthreads();
    // X halo, 64 channels: unit id -> (pixel id>>3, octant id&7), BN+ReLU applied here
    for (int id = tid; id < 8 * HPX; id += NTHR) {
      const int hp = id >> 3, oc = id & 7;
      const int hy = hp / HW_, hx = hp - hy * HW_;
      const int yy = y0 + hy - 1, xx = x0 + hx - 1;
      const int c = kc * KCW + oc * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W && c < a.cin) {
        v = *(const uint4*)((const bf16_t*)a.x + ((long long)(n * a.H + yy) * a.W + xx) * a.xct + a.xco + c);
        if (a.isc != nullptr) {
          float f[8];
          Vec16<bf16_t>::unpack(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], a.isc[c + j], a.ish[c + j]), 0.f);
          v = Vec16<bf16_t>::pack(f);
        }
      }
      *(uint4*)(Xs + (oc * HPXP + hp) * 16) = v;
    }
    // dY tile
    for (int id = tid; id < TH * TW * 8; id += NTHR) {
      const int px = id >> 3, u = id & 7;
      const int r = px / TW, c = px - r * TW;
      const int yy = y0 + r, xx = x0 + c, co = co0 + u * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (yy < a.H && xx < a.W && co < a.cout)
        v = *(const uint4*)((const bf16_t*)a.dy + ((long long)(n * a.H + yy) * a.W + xx) * a.dct + a.dco + co);
      *(uint4*)(Ds + id * 16) = v;
    }
    __syncthreads();
    if (a.db != nullptr && kc == 0) {
      const bf16_t* d = (const bf16_t*)Ds;
      for (int px = wv; px < TH * TW; px += 4) dbacc += bf2f(d[px * 64 + lane]);
    }
    for (int ks = 0; ks < TH; ++ks) {
      const int pxa = ks * TW + 8 * g + q4;
      bf16x8 af[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + (pxa * 64 + ct * 16 + 4 * p4) * 2));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, Ds + ((pxa + 4) * 64 + ct * 16 + 4 * p4) * 2));
        af[ct] = cat_bf16x4(lo, hi);
      }
      const int oc = 2 * wv + (p4 >> 1);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t - ky * 3;
        const int hp = (ks + ky) * HW_ + 8 * g + q4 + kx;
        const char* base = Xs + (oc * HPXP + hp) * 16 + (p4 & 1) * 8;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base + 4 * 16));
        const bf16x8 bfr = cat_bf16x4(lo, hi);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ct], bfr, acc[t][ct], 0, 0, 0);
      }
    }
  }
  float* out = a.dw + (long long)split * a.cout * 9 * a.cin;
  const int ci = kc * KCW + wv * 16 + i16;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + ct * 16 + g * 4 + e;
        if (co < a.cout && ci < a.cin) out[((long long)co * 9 + t) * a.cin + ci] = acc[t][ct][e];
      }
  if (a.db != nullptr && kc == 0) {
    __syncthreads();
    dbred[wv * 64 + lane] = dbacc;
    __syncthreads();
    if (tid < 64 && co0 + tid < a.cout)
      a.db[(long long)split * a.cout + co0 + tid] = dbred[tid] + dbred[64 + tid] + dbred[128 + tid] + dbred[192 + tid];
  }
}

__global__ void wgrad_reduce_kernel(const float* part, const float* dbp, int nsplit, int cout, int cin, int taps,
                                    float* dw, float* db) {
  const long long per = (long long)cout * taps * cin;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id < per) {
    double s = 0.0;
    for (int k = 0; k < nsplit; ++k) s += (double)part[(long long)k * per + id];
    const int ci = (int)(id % cin);
    const long long r = id / cin;
    const int t = (int)(r % taps);
    const int co = (int)(r / taps);
    dw[((long long)co * cin + ci) * taps + t] = (float)s;
  }
  if (db != nullptr && id < cout) {
    double s = 0.0;
    for (int k = 0; k < nsplit; ++k) s += (double)dbp[(long long)k * cout + id];
    db[id] = (float)s;
  }
}

bool act_ok(const eunet_act* a) {
  return a && a->ptr && a->n > 0 && a->h > 0 && a->w > 0 && a->c > 0 && a->coff >= 0 &&
         a->coff + a->c <= a->ctot && (a->dtype == EUNET_F32 || a->dtype == EUNET_BF16);
}

int elems16(int dtype) { return dtype == EUNET_BF16 ? 8 : 4; }
int kchunk(int dtype) { return 4 * elems16(dtype); }

}  // namespace

extern "C" {

int eunet_conv3x3_packed_bytes(int cout, int cin, int dtype, size_t* bytes) {
  EUNET_REQUIRE(bytes && cout > 0 && cin > 0, "conv3x3_packed_bytes: bad args");
  const int cp = cdiv(cout, BN) * BN, kp = cdiv(cin, kchunk(dtype)) * kchunk(dtype);
  *bytes = (size_t)cp * kp * 9 * (dtype == EUNET_BF16 ? 2 : 4);
  return EUNET_OK;
}

int eunet_conv3x3_pack(const float* w, int cout, int cin, int flip, void* wp, int dtype, void* stream) {
  EUNET_REQUIRE(w && wp && cout > 0 && cin > 0, "conv3x3_pack: bad args");
  const int go = flip ? cin : cout, gi = flip ? cout : cin;  // GEMM output / input channels
  const int cp = cdiv(go, BN) * BN, kp = cdiv(gi, kchunk(dtype)) * kchunk(dtype);
  const long long total = (long long)cp * kp * 9;
  dim3 grid((unsigned)((total + 255) / 256));
  if (dtype == EUNET_BF16)
    pack_kernel<bf16_t><<<grid, 256, 0, (hipStream_t)stream>>>(w, cout, cin, flip, (bf16_t*)wp, cp, kp);
  else
    pack_kernel<float><<<grid, 256, 0, (hipStream_t)stream>>>(w, cout, cin, flip, (float*)wp, cp, kp);
  EUNET_LAUNCH_CHECK("conv3x3_pack");
  return EUNET_OK;
}

int eunet_conv3x3_tiles(const eunet_act* y, int* tiles) {
  EUNET_REQUIRE(act_ok(y) && tiles, "conv3x3_tiles: bad args");
  *tiles = y->n * cdiv(y->h, TH) * cdiv(y->w, TW);
  return EUNET_OK;
}

int eunet_conv3x3_fwd(const eunet_act* x, const float* in_scale, const float* in_shift, const void* wp,
                      const float* bias, const eunet_act* y, float* stats, void* stream) {
  EUNET_REQUIRE(act_ok(x) && act_ok(y) && wp, "conv3x3_fwd: bad tensors");
  EUNET_REQUIRE(x->dtype == y->dtype, "conv3x3_fwd: dtype mismatch");
  EUNET_REQUIRE(x->n == y->n && x->h == y->h && x->w == y->w, "conv3x3_fwd: spatial mismatch");
  const int E = elems16(x->dtype);
  EUNET_REQUIRE(x->c % E == 0 && x->ctot % E == 0 && x->coff % E == 0,
                "conv3x3_fwd: input channels/stride/offset must be multiples of %d", E);
  EUNET_REQUIRE((in_scale == nullptr) == (in_shift == nullptr), "conv3x3_fwd: scale/shift pair");
  FwdArgs a;
  a.x = x->ptr; a.N = x->n; a.H = x->h; a.W = x->w; a.xct = x->ctot; a.xco = x->coff; a.cin = x->c;
  a.isc = in_scale; a.ish = in_shift;
  a.wp = wp; a.cout_pad = cdiv(y->c, BN) * BN; a.nkc = cdiv(x->c, kchunk(x->dtype));
  a.bias = bias;
  a.y = y->ptr; a.yct = y->ctot; a.yco = y->coff; a.cout = y->c;
  a.stats = stats; a.tx = cdiv(x->w, TW); a.ty = cdiv(x->h, TH); a.ntiles = x->n * a.tx * a.ty;
  EUNET_REQUIRE(y->c % E == 0 && y->ctot % E == 0 && y->coff % E == 0,
                "conv3x3_fwd: output channels/stride/offset must be multiples of %d", E);
  dim3 grid(a.ntiles, a.cout_pad / BN);
  if (x->dtype == EUNET_BF16) {
    allow_lds(conv3x3_fwd_kernel<bf16_t>, FWD_LDS);
    conv3x3_fwd_kernel<bf16_t><<<grid, FT, FWD_LDS, (hipStream_t)stream>>>(a);
  } else {
    allow_lds(conv3x3_fwd_kernel<float>, FWD_LDS);
    conv3x3_fwd_kernel<float><<<grid, FT, FWD_LDS, (hipStream_t)stream>>>(a);
  }
  EUNET_LAUNCH_CHECK("conv3x3_fwd");
  return EUNET_OK;
}

int eunet_conv3x3_wgrad_splits(const eunet_act* dy, int cin, int dtype, int* nsplit) {
  EUNET_REQUIRE(act_ok(dy) && nsplit && cin > 0, "conv3x3_wgrad_splits: bad args");
  const int ntiles = dy->n * cdiv(dy->h, TH) * cdiv(dy->w, TW);
  const int blocks = cdiv(dy->c, 64) * cdiv(cin, dtype == EUNET_BF16 ? KCW : kchunk(dtype));
  int s = cdiv(dtype == EUNET_BF16 ? 512 : 2048, blocks);
  s = s < 1 ? 1 : s;
  s = s > ntiles ? ntiles : s;
  // keep partials <= 256 MiB
  const long long per = (long long)dy->c * 9 * cin * 4;
  while (s > 1 && per * s > (256ll << 20)) --s;
  const int per_split = cdiv(ntiles, s);
  *nsplit = cdiv(ntiles, per_split);
  return EUNET_OK;
}

int eunet_conv3x3_wgrad(const eunet_act* x, const float* in_scale, const float* in_shift, const eunet_act* dy,
                        float* dw_part, float* db_part, int nsplit, void* stream) {
  EUNET_REQUIRE(act_ok(x) && act_ok(dy) && dw_part && nsplit > 0, "conv3x3_wgrad: bad args");
  EUNET_REQUIRE(x->dtype == dy->dtype, "conv3x3_wgrad: dtype mismatch");
  EUNET_REQUIRE(x->n == dy->n && x->h == dy->h && x->w == dy->w, "conv3x3_wgrad: spatial mismatch");
  const int E = elems16(x->dtype);
  EUNET_REQUIRE(x->c % E == 0 && x->ctot % E == 0 && x->coff % E == 0 && dy->c % E == 0 &&
                    dy->ctot % E == 0 && dy->coff % E == 0,
                "conv3x3_wgrad: channels/strides must be multiples of %d", E);
  WgArgs a;
  a.x = x->ptr; a.N = x->n; a.H = x->h; a.W = x->w; a.xct = x->ctot; a.xco = x->coff; a.cin = x->c;
  a.isc = in_scale; a.ish = in_shift;
  a.dy = dy->ptr; a.dct = dy->ctot; a.dco = dy->coff; a.cout = dy->c;
  a.dw = dw_part; a.db = db_part;
  a.tx = cdiv(x->w, TW); a.ty = cdiv(x->h, TH); a.ntiles = x->n * a.tx * a.ty;
  a.per_split = cdiv(a.ntiles, nsplit);
  EUNET_REQUIRE(cdiv(a.ntiles, a.per_split) == nsplit, "conv3x3_wgrad: nsplit not from wgrad_splits");
  if (x->dtype == EUNET_BF16) {
    dim3 grid(nsplit, cdiv(dy->c, 64), cdiv(x->c, KCW));
    allow_lds(conv3x3_wgrad_bf16_kernel, WG_LDS);
    conv3x3_wgrad_bf16_kernel<<<grid, NTHR, WG_LDS, (hipStream_t)stream>>>(a);
  } else {
    dim3 grid(nsplit, cdiv(dy->c, 64), cdiv(x->c, kchunk(x->dtype)));
    const size_t lds = A_LDS_BYTES + TH * TW * 64 * 4 + 4 * 64 * 4;
    allow_lds(conv3x3_wgrad_kernel<float>, lds);
    conv3x3_wgrad_kernel<float><<<grid, NTHR, lds, (hipStream_t)stream>>>(a);
  }
  EUNET_LAUNCH_CHECK("conv3x3_wgrad");
  return EUNET_OK;
}

int eunet_wgrad_reduce(const float* dw_part, const float* db_part, int nsplit, int cout, int cin, int taps,
                       float* dw, float* db, void* stream) {
  EUNET_REQUIRE(dw_part && dw && nsplit > 0 && cout > 0 && cin > 0 && taps > 0, "wgrad_reduce: bad args");
  EUNET_REQUIRE((db_part == nullptr) == (db == nullptr), "wgrad_reduce: db pair");
  long long per = (long long)cout * taps * cin;
  if (per < cout) per = cout;
  wgrad_reduce_kernel<<<(unsigned)((per + 255) / 256), 256, 0, (hipStream_t)stream>>>(dw_part, db_part, nsplit,
                                                                                      cout, cin, taps, dw, db);
  EUNET_LAUNCH_CHECK("wgrad_reduce");
  return EUNET_OK;
}

}  // extern "C"
