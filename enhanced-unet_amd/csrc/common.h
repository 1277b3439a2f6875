// Shared device/host helpers for libeunet_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <utility>
#include <vector>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/eunet.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef uint16_t bf16_t;  // storage type for bf16 activations

__device__ __forceinline__ bf16x8 cat_bf16x4(s16x4 lo, s16x4 hi) {
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// ---------------------------------------------------------------------------
// host-side error plumbing (C-ABI returns int codes; message via eunet_last_error)
// ---------------------------------------------------------------------------
namespace eunet {
void set_error(const char* fmt, ...);
int check_launch(const char* what);

// The update guard of the current device (eunet_set_update_guard): a device fp64 word; while it is
// nonzero the persistent-state writes of eunet_bn_finalize and eunet_clip_adamw are skipped.  Read
// on the host at launch, so a captured graph keeps the pointer it was captured with.
constexpr int GUARD_NDEV = 64;
inline const double*& update_guard_slot(int dev) {
  static const double* slots[GUARD_NDEV] = {};
  return slots[dev];
}
inline const double* update_guard() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= GUARD_NDEV) return nullptr;
  return update_guard_slot(d);
}
}  // namespace eunet

#define EUNET_REQUIRE(cond, ...)                    \
  do {                                              \
    if (!(cond)) {                                  \
      eunet::set_error(__VA_ARGS__);                \
      return EUNET_ERR_INVALID;                     \
    }                                               \
  } while (0)

#define EUNET_LAUNCH_CHECK(name) \
  do {                           \
    int _rc = eunet::check_launch(name); \
    if (_rc) return _rc;         \
  } while (0)

// ---------------------------------------------------------------------------
// bounds-checked debug build (make debug -> libeunet_hip_debug.so, -DEUNET_DEBUG).
// EUNET_DASSERT(cond) in device code records the first failing source line of its translation
// unit and counts failures in a per-TU device word (a vector atomic: no trap, the kernel runs on);
// eunet_debug_status() reads every unit's words after a device synchronisation.  Release builds
// compile the checks away.  Each .hip file that uses EUNET_DASSERT names itself once with
// EUNET_DEBUG_UNIT(tag) at namespace scope.
// ---------------------------------------------------------------------------
#ifdef EUNET_DEBUG
#define EUNET_DEBUG_UNIT(tag)                                                    \
  __device__ unsigned g_eunet_dbg[2];                                            \
  namespace eunet {                                                              \
  int debug_read_##tag(unsigned* line, unsigned* count, bool reset) {            \
    unsigned h[2] = {0u, 0u};                                                    \
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_eunet_dbg), sizeof(h)) != hipSuccess) \
      return EUNET_ERR_HIP;                                                      \
    *line = h[0];                                                                \
    *count = h[1];                                                               \
    if (reset) {                                                                 \
      const unsigned z[2] = {0u, 0u};                                            \
      if (hipMemcpyToSymbol(HIP_SYMBOL(g_eunet_dbg), z, sizeof(z)) != hipSuccess) \
        return EUNET_ERR_HIP;                                                    \
    }                                                                            \
    return EUNET_OK;                                                             \
  }                                                                              \
  }
#define EUNET_DASSERT(cond)                                   \
  do {                                                        \
    if (!(cond)) {                                            \
      atomicCAS(&g_eunet_dbg[0], 0u, (unsigned)__LINE__);     \
      atomicAdd(&g_eunet_dbg[1], 1u);                         \
    }                                                         \
  } while (0)
#else
#define EUNET_DEBUG_UNIT(tag)
#define EUNET_DASSERT(cond) \
  do {                      \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// element conversion
// ---------------------------------------------------------------------------
// x + x[lane ^ 16] / x + x[lane ^ 32] on every lane with the gfx950 permlane swaps (VALU, no
// LDS crossbar as __shfl_xor's ds_bpermute)
__device__ __forceinline__ float xor16_sum(float v) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// two floats -> one dword of two bf16 (lo, hi), rounded to nearest even: a single v_cvt_pk_bf16_f32
// (f2bf(lo) | f2bf(hi) << 16 compiles to two conversions and a permute)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2_t));
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
  static constexpr int per16 = 4;  // elements per 16-byte unit
};
template <> struct Elem<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
  static constexpr int per16 = 8;
};

// 16-byte unit <-> 8 (bf16) or 4 (f32) floats
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  static __device__ __forceinline__ void unpack(uint4 u, float* f) {
    f[0] = __uint_as_float(u.x); f[1] = __uint_as_float(u.y);
    f[2] = __uint_as_float(u.z); f[3] = __uint_as_float(u.w);
  }
  static __device__ __forceinline__ uint4 pack(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
};
template <> struct Vec16<bf16_t> {
  static constexpr int N = 8;
  static __device__ __forceinline__ void unpack(uint4 u, float* f) {
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
  }
  static __device__ __forceinline__ uint4 pack(const float* f) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pk_bf16(f[2 * i], f[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

// ---------------------------------------------------------------------------
// wave helpers (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Butterfly transpose-reduce: every lane holds v[0..63] (one value per channel);
// afterwards lane l holds sum over the 64 lanes of channel l.  63 shuffles/lane.
__device__ __forceinline__ float wave_transpose_reduce64(float (&v)[64]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const bool upper = (lane & s) != 0;
#pragma unroll
    for (int i = 0; i < s; ++i) {
      // keep half [upper ? s+i : i], send the other half to partner lane^s
      float keep = upper ? v[i + s] : v[i];
      float send = upper ? v[i] : v[i + s];
      float recv = __shfl_xor(send, s, 64);
      v[i] = keep + recv;
    }
  }
  return v[0];
}

// bilinear x2 (align_corners=False) source index/weight, PyTorch's
// area_pixel_compute_source_index for scale 1/2 (F.interpolate, nn.Upsample)
__device__ __forceinline__ void up2_src(int o, int in, int& i0, int& i1, float& l1) {
  float s = 0.5f * ((float)o + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = (int)s;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
}

// the same in integer arithmetic (value-equal for 0 <= o < 2 in): o = 0 -> (0, 0); odd o = 2m+1 -> (m, 1/4);
// even o = 2m >= 2 -> (m - 1, 3/4); i1 = min(i0 + 1, in - 1)
__device__ __forceinline__ void up2_src_i(int o, int in, int& i0, int& i1, float& l1) {
  const int m = o >> 1;
  const bool odd = (o & 1) != 0;
  i0 = odd ? m : max(m - 1, 0);
  i1 = min(i0 + 1, in - 1);
  l1 = odd ? 0.25f : (o == 0 ? 0.f : 0.75f);
}

// adjoint of the x2 bilinear taps: the weight of low-res index i in high-res output o; per
// low-res row y the contributing high-res rows are 2y-1 .. 2y+2
__device__ __forceinline__ float up2_adj_w(int o, int in, int i) {
  int i0, i1;
  float l1;
  up2_src(o, in, i0, i1, l1);
  return (i0 == i ? 1.f - l1 : 0.f) + (i1 == i ? l1 : 0.f);
}

// the same weights of low-res index i (0 <= i < in) for the four high-res positions 2i-1 .. 2i+2 that can reach it,
// in closed form: (1/4, 3/4, 3/4, 1/4) inside, (0, 1, 3/4, 1/4) at i = 0 and (1/4, 3/4, 1, 0) at i = in-1 (both
// edges at in = 1: (0, 1, 1, 0)); positions outside 0 .. 2in-1 weigh 0.  Equal to up2_adj_w value by value.
__device__ __forceinline__ f32x4 up2_adj_w4(int i, int in) {
  f32x4 w = {0.25f, 0.75f, 0.75f, 0.25f};
  if (i == 0) { w[0] = 0.f; w[1] = 1.f; }
  if (i == in - 1) { w[2] = 1.f; w[3] = 0.f; }
  return w;
}

// deterministic fp64 column sum of a [rows][ld] partial matrix (bn_pool_up.hip); columns
// >= split go to out_hi[col - split] when out_hi != nullptr
int eunet_colsum_ld(const float* part, int rows, int cols, int ld, float* out, void* ws, hipStream_t s,
                    int split = 0, float* out_hi = nullptr);
// the same over several outputs: column c goes to out[i][c - start[i]] for the last segment i with
// start[i] <= c (start[0] = 0; one launch pair for a partial row that packs several gradients)
struct ColSegs {
  float* out[4];
  int start[4];
  int n;
};
int eunet_colsum_segs(const float* part, int rows, int cols, int ld, const ColSegs& segs, void* ws, hipStream_t s);

// kernels with > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
template <typename K>
inline void allow_lds(K* kernel, size_t bytes) {
  if (bytes <= 65536) return;
  // once per kernel (the attribute persists): a table of the kernels already raised, under a lock (the
  // forward and autograd's backward thread both launch)
  static std::mutex mu;
  static std::vector<std::pair<const void*, size_t>> done;
  std::lock_guard<std::mutex> lock(mu);
  for (const auto& d : done)
    if (d.first == (const void*)kernel && d.second >= bytes) return;
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  done.emplace_back((const void*)kernel, bytes);
}

__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// activation view accessors
__host__ __device__ inline long long act_pix(const eunet_act& a, int n, int y, int x) {
  return ((long long)(n * a.h + y) * a.w + x);
}
