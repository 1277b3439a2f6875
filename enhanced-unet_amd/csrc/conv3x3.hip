// Conv2d 3x3 / stride 1 / padding 1 on NHWC activations, MFMA implicit GEMM.
//
// Reference call sites: models.py:219,222 (_conv_block, every DoubleConv of
// BasicUNet models.py:203-211) and their autograd (dgrad / wgrad).
//
// Forward (and dgrad, which is the same kernel on W'[ci][co][8-t]):
//   GEMM  M = output pixels (16x32 tile per block), N = Cout (64 per block),
//         K = 9 taps x Cin, consumed one Cin chunk (KC channels) at a time.
//   The chunk's input halo tile [(16+2) x (32+2) px][KC] is staged once in LDS
//   and re-read by all 9 taps (no im2col, 1.2x halo over-read instead of 9x),
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
//
// The library takes no configuration from the environment: the alternatives measured
// against these kernels (double buffering, 8 waves, producer/consumer waves, LDS-DMA
// staging, weight fragments from L2, tap pipelining, persistent Cin=64 kernels (round 1, and a
// wave-group-skewed one in round 2), other block orders) are recorded in DESIGN.md §4 and
// profiles/r0*_ab_*; their code lives in the git history, not in this file.
#include <algorithm>
#include <type_traits>

#include "common.h"

EUNET_DEBUG_UNIT(conv3x3)

namespace {

constexpr int BN = 64;                    // output channels per block
constexpr int NTHR = 256;
constexpr int B_UNITS = 4 * BN * 9;       // 2304
constexpr int B_LDS_BYTES = B_UNITS * 16;   // 36864

template <typename T> struct KCh { static constexpr int v = 4 * Vec16<T>::N; };  // 16 (f32) / 32 (bf16)

struct FwdArgs {
  const void* x; int N, H, W, xct, xco, cin;
  const float* isc; const float* ish; int iss;  // operand transform; iss = per-sample stride (0: shared)
  const void* wp; int cout_pad, nkc;
  const float* bias;
  void* y; int yct, yco, cout;
  float* stats; int tx, ty, ntiles;
  // optional fused BN-backward reduction over the produced gradient (dgrad only):
  // part[tile][2][cout] = (sum g', sum g' xhat), g' = g [by bsc + bsh > 0] (the forward's ReLU
  // mask, bsc / bsh = its BN affine), xhat = (by - mean) istd, g = the stored (rounded) output
  const void* by; int byct, byco;
  const float* bmean; const float* bistd; const float* bsc; const float* bsh;
  float* bpart;
  const float* gsc;  // dgrad only, nullable: output scaled by gsc[n][co] (Dropout2d keep mask / (1-p))
  // dgrad only, nullable: BatchNorm-backward transform of the operand (the "apply" half of BN
  // backward, fused into the halo staging).  x holds g (gradient w.r.t. the BN+ReLU output), ty the
  // BN's input y in tyin (same layout as x); the staged operand is gy = k1 g [y k1 + kq > 0] + k2 y + k3
  // with tcoef = [k1 | kq | k2 | k3][cin] (eunet_bn_bwd_coef).  Co-block 0 also stores the tile
  // interior of gy to tgo (same layout, nullable) for the weight gradient.
  const void* tyin; const float* tcoef; void* tgo;
  int pro1;          // 1 (always, set by the launcher): the first K-chunk is staged in one round trip.
                     // Kept a runtime flag: with the halved-staging prologue still compiled in, the
                     // register allocator fits the kernel in 256 VGPRs without spills (a compile-time
                     // constant here produces SGPR / VGPR spills).
};

// Forward: 256 threads = 4 waves (one per SIMD), output tile 16 x 32 px x 64 co;
// wave w computes rows 4w..4w+3 (128 px = 8 m-tiles) x 64 co = 32 accumulators,
// so each tap issues 8 A + 4 B 16-byte LDS reads for 32 MFMAs.  Two blocks per CU
// (75 KB of LDS each, one stage): a block's staging overlaps the other block's
// MFMAs.  The first K-chunk is staged in one global round trip (the accumulators
// are not live yet), later chunks in halves to bound the staging registers.  Halo
// units are loaded 8 pixels x 4 quarters per 32 lanes so the LDS writes are
// conflict-free; the plain data gradient stages its halo by LDS-DMA instead (fslot).  The epilogue stages the tile through LDS and stores whole
// 16-byte vectors.
constexpr int FTH = 16, FTW = 32;            // output tile
constexpr int FHW = FTW + 2;                 // 34
constexpr int FHPX = (FTH + 2) * FHW;        // 612 halo pixels
constexpr int FHPXP = 640;                   // halo pixel slots (612 used), 4 channel quarters each
// LDS slot (16 B) of halo pixel hp's channel quarter q.  Plane-major [q][hp] (PIX = false: the forward with
// the BN+ReLU operand transform and the fused-apply data gradient, register staging) or pixel-major [hp][q]
// (PIX = true: the plain data gradient and the untransformed forward, staged by LDS-DMA -- a wave-instruction then reads 16 pixels x 64 contiguous bytes from global;
// plane-major slots would read 64 pixels x 16 B and measured slower, profiles/r04_ab.txt).  Measured per
// layout (13 layers, tools/conv_bench.py): the forward loses 2 % pixel-major (4-way bank conflicts of the
// fragment reads) and 6 % with the quarter XOR-swizzle that removes them (its per-read address VALU), the
// DMA-staged data gradient gains 6 %, the DMA-staged untransformed forward 5-13 % -- so the layout follows the
// staging.
// The pixel-major fragment reads are 2-way bank conflicted: a ds_read_b128 lane group (lanes 0-3 / 12-15 at
// quarter q, 4-11 at q + 1 over 16 consecutive halo pixels) puts pixels 4 apart on one 16-byte slot of the
// 256-byte bank row (SQ_LDS_BANK_CONFLICT 0.35-0.39 of the LDS cycles of every DMA-staged forward / data
// gradient, profiles/r06_sq_layers.txt).  Round 6 measured the conflict-free alternative that keeps the DMA
// contiguous, channel halves [q >> 1][hp][q & 1] (a DMA wave-instruction then reads 32 pixels x 32 B): 13-layer
// data gradient 5.95 vs 5.77 ms, untransformed forwards +3 %, bench -1.2 % (profiles/r06_ab.txt r6hp) -- the
// halved DMA contiguity costs more than the conflicts, which the MFMA phase's LDS headroom absorbs.
template <bool PIX>
__device__ __forceinline__ int fslot(int hp, int q) {
  return PIX ? hp * 4 + q : q * FHPXP + hp;
}
// inverse for slot s: (halo pixel, quarter)
template <bool PIX>
__device__ __forceinline__ void fslot_inv(int s, int& hp, int& q) {
  if (PIX) {
    hp = s >> 2;
    q = s & 3;
  } else {
    q = s / FHPXP;
    hp = s - q * FHPXP;
  }
}
constexpr int FT = 256;                      // threads of the forward block
constexpr int FA_UNITS = 4 * FHPX;           // 2448
constexpr int FA_BYTES = 4 * FHPXP * 16;     // 40960
constexpr int STAGE_BYTES = FA_BYTES + B_LDS_BYTES;  // 77824
constexpr int OUT_LD = 68;                   // fp32 row stride of the output staging tile
constexpr int FWD_LDS = STAGE_BYTES;         // two blocks / CU

// XCD-aware block order: hardware block b runs on XCD b % 8.  Logical block L =
// (tile, co-block) with the co-block fastest; each XCD gets a contiguous range of L,
// so the co-blocks that re-read one input tile (and its halo neighbours) share
// that XCD's L2 and run at the same time.
__device__ __forceinline__ void xcd_map(int b, int ntiles, int ncob, int& tile, int& cob) {
  const int total = ntiles * ncob, full = total & ~7;
  const int L = b < full ? (b & 7) * (full >> 3) + (b >> 3) : b;
  tile = L / ncob;
  cob = L - tile * ncob;
}

// unit id -> (halo pixel, quarter): 32 consecutive ids = 8 pixels x 4 quarters
// (pixel-major: unit id IS LDS slot id, so 16 lanes write 256 contiguous bytes and read 4 pixels x 64 B;
// plane-major: 32 consecutive ids = 8 pixels x 4 quarters)
template <bool PIX>
__device__ __forceinline__ void fwd_unit(int id, int& hp, int& q) {
  if (PIX) {
    fslot_inv<true>(id, hp, q);
  } else {
    hp = (id >> 5) * 8 + (id & 7);
    q = (id >> 3) & 3;
  }
}

// Halo staging loads go through buffer descriptors (one per sample slice of x, one for the
// packed weights): 32-bit per-unit offsets instead of 64-bit addresses, and no branch per
// unit -- a unit outside the image gets offset FWD_OOB, which the descriptor's range check
// turns into zeros.  Offsets are unsigned 32-bit: the launcher requires each slice to be < 3 GiB
// (FWD_OOB plus a chunk's channel offset stays above any valid offset; a 2048^2 x 288-channel bf16
// slice, the dual-branch base-96 dec2.0 input of configs[4], is 2.4 GB).
constexpr uint32_t FWD_OOB = 0xC0000000u;

template <typename T, bool PIX>
__device__ __forceinline__ uint32_t fwd_unit_off(const FwdArgs& a, int y0, int x0, int id) {
  constexpr int E = Vec16<T>::N;
  int hp, q;
  fwd_unit<PIX>(id, hp, q);
  const int hy = hp / FHW, hx = hp - hy * FHW;
  const int yy = y0 + hy - 1, xx = x0 + hx - 1;
  const bool ok = hp < FHPX && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
  return ok ? (uint32_t)((yy * a.W + xx) * a.xct + a.xco + q * E) * (uint32_t)sizeof(T) : FWD_OOB;
}

// The halo quarter (16-byte channel group) of unit id depends only on tid: FT = 256 units per
// staging iteration shift id by 256 i, which leaves the quarter unchanged.  So each thread
// transforms one fixed group of E channels per chunk and loads that group's BN scale / shift
// once per chunk, with the halo loads (not per unit after its data arrived: a dependent
// global round trip per unit).

// Diagnostic build only (tools/conv_stamps.py builds it with -DCONV_STAMP=1): wave 0 of every block
// of conv3x3_fwd_kernel stamps s_memtime around its phases -- staging (+ its barriers), the MFMA
// chunks (issue), the epilogue -- and writes per-block sums to g_conv_stamps (read back by
// eunet_conv_stamps).  The product build has none of it.
#ifndef CONV_STAMP
#define CONV_STAMP 0
#endif
#if CONV_STAMP
constexpr int STAMP_BLOCKS = 1 << 16;
constexpr int STAMP_N = 11;  // [t_start, total, stage, mfma, epilogue | epilogue: pre-pass (bias, stats),
                             //  pass 0 LDS staging + barrier, pass 0 stores, pass 1 staging, pass 1 stores, reduction]
__device__ unsigned long long g_conv_stamps[STAMP_BLOCKS * STAMP_N];
__device__ __forceinline__ unsigned long long conv_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif
// DG: a tag only (the same code either way) so the dgrad launches carry their own symbol --
// rocprofv3 and the bench report forward and data-gradient launches separately.
// TO: the output element type -- T, or float for a bf16 data gradient whose consumer keeps fp32
// (the dual-branch gate backward reads the 2K-channel g_f2 in fp32; no fused BN reduction then)
// BT: the dgrad with the BN-backward transform in its staging (eunet_conv3x3_dgrad_fused; bf16) -- its
// own instantiation, so the plain data-gradient launches keep their register allocation.
// BNB: the fused BN-backward reduction of the dgrad epilogue (a.bpart set) -- a template parameter so the
// forward and the plain data-gradient launches carry none of its code.
// PF: a bf16 forward without an operand transform (a DoubleConv's conv .0: its input is stored post-BN+ReLU)
// stages its halo by LDS-DMA like the plain data gradient (pixel-major slots, no staging registers):
// bit-identical, 5-13 % faster per layer standalone, -7 % over the six .0 layers (profiles/r05_ab.txt r5o).
// CT: the layer has a tail co-block whose channels past co0 + 32 are all padding (cout mod 64 in 1..32: the
// 96 / 288-channel layers of base 96, configs[4]); that block runs a second copy of the K loop over co tiles
// 0-1 only (half the MFMAs).  Its own instantiation: the copy's registers cost the other layers 0.2-0.5 %
// (profiles/r05_ab.txt r5v), and a uniform branch inside the MFMA loop 2-10 % (r5u).
template <typename T, bool DG, typename TO = T, bool BT = false, bool BNB = false, bool PF = false, bool CT = false>
__global__ __launch_bounds__(FT, 2) void conv3x3_fwd_kernel(FwdArgs a) {
  constexpr int NW = 4;                       // waves
  constexpr int RPW = FTH / NW;               // output rows per wave
  constexpr int MT = 2 * RPW;                 // 16-px m-tiles per wave
  constexpr int A_IT = (FA_UNITS + FT - 1) / FT;
  constexpr int B_IT = (B_UNITS + FT - 1) / FT;
  constexpr bool B_TAIL = B_UNITS % FT != 0;
  constexpr int NPASS = 2;                    // epilogue staging passes (LDS budget)
  constexpr int PROWS = FTH / NPASS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int tile, cob;
  xcd_map(blockIdx.x, a.ntiles, a.cout_pad / BN, tile, cob);
  EUNET_DASSERT(tile < a.ntiles && cob * BN < a.cout_pad && a.cout <= a.cout_pad);
  const int tpi = a.tx * a.ty;
  const int n = tile / tpi, trem = tile - n * tpi;
  const int y0 = (trem / a.tx) * FTH, x0 = (trem % a.tx) * FTW;
  const int co0 = cob * BN;
  const int q = lane >> 4, li = lane & 15;

  f32x4 acc[MT][4];
  u32x4 ra[A_IT];
  uint32_t aoff[A_IT];  // byte offset of each halo unit in the sample slice (FWD_OOB: padding)
  char* const As = smem;
  char* const Bs = smem + FA_BYTES;
  constexpr int E = Vec16<T>::N, KC = KCh<T>::v;
  // this thread's halo quarter (fwd_unit), the same for every unit (ids tid + FT i)
  constexpr bool PIX = ((DG && !BT) || PF) && sizeof(T) == 2;  // halo layout / staging (fslot)
  // CTE: a bf16 data gradient with a bf16 output (the plain and the BN-reducing ones) accumulates C^T (the MFMA
  // operands swapped: a lane holds 4 consecutive channels of one pixel) and stages its tile as bf16 in one pass
  // (not the CT tail instantiation: already at 254 VGPRs, the C^T epilogue spills it).  The forwards keep the C
  // layout: with C^T and their BN partials summed by DPP over a lane row the 13 standalone forwards measured
  // 0.6 % faster but the step 0.9 % slower in three alternating pairs (profiles/r06_ab.txt r6n / r6p; code in git)
  constexpr bool CTE = DG && !BT && !CT && sizeof(T) == 2 && sizeof(TO) == 2;
  const int sq = PIX ? tid & 3 : (tid >> 3) & 3;
  const int ns = __builtin_amdgcn_readfirstlane(n);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const T*)a.x + (long long)ns * a.H * a.W * a.xct), 0,
      (int)((uint32_t)(a.H * a.W * a.xct) * (uint32_t)sizeof(T)), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.wp, 0, a.nkc * KC * a.cout_pad * 9 * (int)sizeof(T), 0x00020000);
  // dgrad: the BN-backward transform (k1 in asc, kq in ash, k2 / k3 below) and its y operand
  constexpr int BE = DG ? E / 4 : 1;
  f32x4 ak2[BE], ak3[BE];
  u32x4 ry[DG ? A_IT : 1];
  // bf16 only: the fp32 dgrad has no registers to spare (eunet_conv3x3_dgrad_fused applies the transform
  // in a separate pass for fp32)
  constexpr bool BTR = DG && BT && sizeof(T) == 2;
  const bool btr = BTR && a.tcoef != nullptr;
  const uint32_t slice_bytes = (uint32_t)(a.H * a.W * a.xct) * (uint32_t)sizeof(T);
  // the plain data gradient (no operand transform; the default schedule applies the BN backward in a
  // separate pass): its halo goes straight into LDS by buffer_load ... lds (wave-instruction i of wave w
  // fills slots i * FT + 64 w .. +63 = 16 pixels x 4 quarters), so a K-chunk's staging is one
  // asynchronous round trip with no staging registers
  static_assert(!PIX || A_IT * FT == 4 * FHPXP, "dma_a: whole wave-instructions over the halo slots");
  const bool adma = PIX && !btr;
#pragma unroll
  for (int i = 0; i < A_IT; ++i) aoff[i] = fwd_unit_off<T, PIX>(a, y0, x0, tid + i * FT);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(btr ? (const T*)a.tyin + (long long)ns * a.H * a.W * a.xct : nullptr), 0, btr ? (int)slice_bytes : 0,
      0x00020000);
  const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc((void*)(btr ? a.tcoef : nullptr), 0,
                                                                      btr ? 16 * a.cin : 0, 0x00020000);
  // co-block 0 stores the staged gy (tile interior only: every pixel belongs to one tile)
  const bool wgy = btr && a.tgo != nullptr && cob == 0;
  const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(wgy ? (T*)a.tgo + (long long)ns * a.H * a.W * a.xct : nullptr), 0, wgy ? (int)slice_bytes : 0,
      0x00020000);
  auto chunk_ok = [&](int kc) { return kc * KC + sq * E < a.cin; };
  auto gload_a = [&](int kc, int i0, int i1) {
    const bool cok = chunk_ok(kc);
    const uint32_t cadd = (uint32_t)(kc * KC * (int)sizeof(T));
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      // a staged unit lies inside its sample slice (or is padding, read as zeros)
      EUNET_DASSERT(!cok || aoff[i] == FWD_OOB || aoff[i] + cadd + 16u <= slice_bytes);
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, cok ? aoff[i] + cadd : FWD_OOB, 0, 0);
      if constexpr (BTR)
        if (btr) ry[i] = __builtin_amdgcn_raw_buffer_load_b128(yr, cok ? aoff[i] + cadd : FWD_OOB, 0, 0);
    }
  };
  // BN scale / shift of this thread's channel group, through descriptors too (no branch, so
  // the loads issue with the halo loads; past cin / without a transform they read zeros)
  const int nbytes_aff = a.isc != nullptr ? a.cin * 4 : 0;
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.isc != nullptr ? a.isc + (long long)ns * a.iss : nullptr), 0, nbytes_aff, 0x00020000);
  const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.ish != nullptr ? a.ish + (long long)ns * a.iss : nullptr), 0, nbytes_aff, 0x00020000);
  f32x4 asc[E / 4], ash[E / 4];
  auto gload_affine = [&](int kc) {
    const uint32_t off = (uint32_t)((kc * KC + sq * E) * 4);
    if constexpr (BTR) {
      const uint32_t row = (uint32_t)(4 * a.cin);
#pragma unroll
      for (int j = 0; j < E / 4; ++j) {
        asc[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(cr, off + 16 * j, 0, 0));
        ash[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(cr, row + off + 16 * j, 0, 0));
        ak2[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(cr, 2 * row + off + 16 * j, 0, 0));
        ak3[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(cr, 3 * row + off + 16 * j, 0, 0));
      }
    } else {
#pragma unroll
      for (int j = 0; j < E / 4; ++j) {
        asc[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(sr, off + 16 * j, 0, 0));
        ash[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(hr, off + 16 * j, 0, 0));
      }
    }
  };
  auto lwrite_a = [&](int kc, int i0, int i1) {
    const bool cok = chunk_ok(kc);
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      int hp, qq;
      fwd_unit<PIX>(tid + i * FT, hp, qq);
      if (hp >= FHPX) continue;
      u32x4 v = ra[i];
      if constexpr (DG) {
        if (BTR && btr) {  // BN backward of the layer whose input gradient this is; padding stays zero
          float f[E], yv[E];
          Vec16<T>::unpack(__builtin_bit_cast(uint4, v), f);
          Vec16<T>::unpack(__builtin_bit_cast(uint4, ry[i]), yv);
          const bool ok = cok && aoff[i] < FWD_OOB;
#pragma unroll
          for (int j = 0; j < E; ++j) {
            const float k1 = asc[j >> 2][j & 3];
            const float gg = fmaf(yv[j], k1, ash[j >> 2][j & 3]) > 0.f ? f[j] : 0.f;  // the forward's ReLU mask
            f[j] = ok ? fmaf(k1, gg, fmaf(yv[j], ak2[j >> 2][j & 3], ak3[j >> 2][j & 3])) : 0.f;
          }
          v = __builtin_bit_cast(u32x4, Vec16<T>::pack(f));
        }
      } else if (a.isc != nullptr) {  // BN + ReLU of the producing layer; padding stays zero
        const bool ok = cok && aoff[i] < FWD_OOB;
        if constexpr (sizeof(T) == 2) {
          // packed fp32 FMA per bf16 pair, rounded to bf16, ReLU on the rounded pair (sign bit:
          // round(max(x, 0)) == max(round(x), 0)) -- as the weight gradient's staging does
          u32x4 o;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const f32x2 x = {__uint_as_float(v[d] << 16), __uint_as_float(v[d] & 0xFFFF0000u)};
            const f32x2 r = __builtin_elementwise_fma(
                x, (f32x2){asc[d >> 1][2 * (d & 1)], asc[d >> 1][2 * (d & 1) + 1]},
                (f32x2){ash[d >> 1][2 * (d & 1)], ash[d >> 1][2 * (d & 1) + 1]});
            const s16x2 b = __builtin_bit_cast(s16x2, pk_bf16(r[0], r[1]));
            o[d] = ok ? __builtin_bit_cast(uint32_t, __builtin_elementwise_max(b, (s16x2){0, 0})) : 0u;
          }
          v = o;
        } else {
          float f[E];
          Vec16<T>::unpack(__builtin_bit_cast(uint4, v), f);
#pragma unroll
          for (int j = 0; j < E; ++j) f[j] = ok ? fmaxf(fmaf(f[j], asc[j >> 2][j & 3], ash[j >> 2][j & 3]), 0.f) : 0.f;
          v = __builtin_bit_cast(u32x4, Vec16<T>::pack(f));
        }
      }
      *(u32x4*)(As + fslot<PIX>(hp, qq) * 16) = v;
    }
  };
  // weights straight into LDS (buffer_load ... lds: no staging VGPRs, no LDS write instructions); unit id =
  // tid + i * FT is LDS unit id, so wave-instruction i of wave w fills units i * FT + 64 w .. +63
  const int wvs = __builtin_amdgcn_readfirstlane(wv);
  auto dma_b = [&](int kc) {
    static_assert(!B_TAIL, "dma_b: whole wave-instructions");
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int id = tid + i * FT;
      const uint32_t wo = (uint32_t)((((kc * 4 + id / (BN * 9)) * a.cout_pad + co0) * 9 + id % (BN * 9)) * 16);
      EUNET_DASSERT(wo + 16u <= (uint32_t)(a.nkc * KC * a.cout_pad * 9 * (int)sizeof(T)));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void*)(Bs + (i * FT + wvs * 64) * 16),
                                               16, wo, 0, 0, 0);
    }
  };
  auto dma_a = [&](int kc) {
    const uint32_t cadd = (uint32_t)(kc * KC * (int)sizeof(T));
    const bool full = (kc + 1) * KC <= a.cin;  // else: quarters past cin read as zeros
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      uint32_t off = aoff[i];
      if (!full && kc * KC + (tid & 3) * E >= a.cin) off = FWD_OOB;  // (quarter of slot tid + FT i)
      EUNET_DASSERT(off == FWD_OOB || off + cadd + 16u <= slice_bytes);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(As + (i * FT + wvs * 64) * 16),
                                               16, off, cadd, 0, 0);
    }
  };
  constexpr int AH = A_IT / 2;
  auto chunk = [&](auto ntc) {  // NTC output tiles of 16 channels
    constexpr int NTC = decltype(ntc)::value;
#pragma unroll 1
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int t = ky * 3 + kx;
        uint4 fb[NTC];
#pragma unroll
        for (int nt = 0; nt < NTC; ++nt) fb[nt] = *(const uint4*)(Bs + (q * (BN * 9) + (nt * 16 + li) * 9 + t) * 16);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int hp = (RPW * wv + (mt >> 1) + ky) * FHW + (mt & 1) * 16 + li + kx;
          const uint4 fa = *(const uint4*)(As + fslot<PIX>(hp, q) * 16);
#pragma unroll
          for (int nt = 0; nt < NTC; ++nt) {
            if constexpr (CTE) {
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  __builtin_bit_cast(bf16x8, fb[nt]), __builtin_bit_cast(bf16x8, fa), acc[mt][nt], 0, 0, 0);
            } else if constexpr (sizeof(T) == 2) {
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  __builtin_bit_cast(bf16x8, fa), __builtin_bit_cast(bf16x8, fb[nt]), acc[mt][nt], 0, 0, 0);
            } else {
              const uint4 B_ = fb[nt];
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(fa.x), __uint_as_float(B_.x), acc[mt][nt], 0, 0, 0);
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(fa.y), __uint_as_float(B_.y), acc[mt][nt], 0, 0, 0);
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(fa.z), __uint_as_float(B_.z), acc[mt][nt], 0, 0, 0);
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(fa.w), __uint_as_float(B_.w), acc[mt][nt], 0, 0, 0);
            }
          }
        }
      }
  };

  // Phase offset: the two blocks sharing a CU start (and, with equal work, keep running) in
  // lock-step, staging at the same time and leaving the MFMA pipes idle together.  Odd blocks
  // start ~2.5k clocks late so one block's staging overlaps the other's MFMAs (ablation:
  // +15-20 % on every layer shape, profiles/r01_ab_phase.txt).
  if (blockIdx.x & 1) __builtin_amdgcn_s_sleep(40);
  auto stage_halves = [&](int kc) {
    dma_b(kc);
    if (PIX && adma) {
      dma_a(kc);
      return;
    }
    gload_affine(kc);
    if (DG && btr) {  // two loads per halo unit (g and y): thirds bound the staging registers
      constexpr int A3 = (A_IT + 2) / 3;
      gload_a(kc, 0, A3);
      lwrite_a(kc, 0, A3);
      gload_a(kc, A3, 2 * A3);
      lwrite_a(kc, A3, 2 * A3);
      gload_a(kc, 2 * A3, A_IT);
      lwrite_a(kc, 2 * A3, A_IT);
    } else {
      gload_a(kc, 0, AH);
      lwrite_a(kc, 0, AH);
      gload_a(kc, AH, A_IT);
      lwrite_a(kc, AH, A_IT);
    }
  };
  // co-block 0 of the fused BN-backward dgrad stores the tile interior of the staged gy (for the
  // weight gradient) from LDS right before the chunk's MFMAs, so the stores drain under them instead
  // of holding the next staging loads' vmcnt waits: 2048 units = 16 x 32 px x 4 channel quarters
  auto store_gy = [&](int kc) {
    if constexpr (BTR) {
      constexpr int SU = FTH * FTW * 4 / FT;  // 8 units per thread
#pragma unroll 1
      for (int j = 0; j < SU; ++j) {
        const int u = tid + j * FT;            // (pixel row, quarter, pixel column): coalesced stores
        const int px = u & (FTW - 1), qq = (u >> 5) & 3, py = u >> 7;
        const int yy = y0 + py, xx = x0 + px;
        const bool ok = yy < a.H && xx < a.W && kc * KC + qq * E < a.cin;
        const u32x4 v = *(const u32x4*)(As + fslot<PIX>((py + 1) * FHW + px + 1, qq) * 16);
        const uint32_t off = ok ? (uint32_t)(((yy * a.W + xx) * a.xct + a.xco + kc * KC + qq * E) * (int)sizeof(T)) : FWD_OOB;
        EUNET_DASSERT(!ok || off + 16u <= slice_bytes);
        __builtin_amdgcn_raw_buffer_store_b128(v, gr, off, 0, 0);
      }
    }
  };
#if CONV_STAMP
  unsigned long long st_t0 = conv_stamp(), st_stage = 0, st_mfma = 0, st_a, st_b;
  st_a = st_t0;
#endif
  if (PIX && adma) {
    stage_halves(0);
  } else if (a.pro1) {  // first chunk in one round trip: the accumulators are not live yet
    dma_b(0);
    gload_affine(0);
    gload_a(0, 0, A_IT);
    lwrite_a(0, 0, A_IT);
  } else {
    stage_halves(0);
  }
  __syncthreads();
  if (wgy) store_gy(0);
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#if CONV_STAMP
  st_b = conv_stamp();
  st_stage += st_b - st_a;
#endif
  for (int kc = 0; kc < a.nkc; ++kc) {
    if (kc > 0) {
#if CONV_STAMP
      st_a = conv_stamp();
#endif
      __syncthreads();  // every wave is done reading the stage
      stage_halves(kc);
      __syncthreads();
      if (wgy) store_gy(kc);
#if CONV_STAMP
      st_b = conv_stamp();
      st_stage += st_b - st_a;
#endif
    }
    __builtin_amdgcn_s_setprio(1);  // the MFMA phase issues ahead of the other block's staging
    if (CT && co0 + BN / 2 >= a.cout)  // (block-uniform)
      chunk(std::integral_constant<int, 2>{});
    else
      chunk(std::integral_constant<int, 4>{});
    __builtin_amdgcn_s_setprio(0);
#if CONV_STAMP
    st_a = conv_stamp();
    st_mfma += st_a - st_b;
#endif
  }

  // ---- epilogue ----
  constexpr int NTH = FT;
  constexpr int UPX = 64 / E;  // 16-byte units per pixel row of the tile
  static_assert(NTH % UPX == 0, "a thread's channel unit must be fixed across store iterations");
  constexpr bool bnb = BNB;
  const int ucol = tid % UPX;
  f32x2 bp1[E / 2], bp2[E / 2];  // the fused BN-backward reduction's per-thread sums (dgrad)
#pragma unroll
  for (int e = 0; e < E / 2; ++e) { bp1[e] = (f32x2){0.f, 0.f}; bp2[e] = (f32x2){0.f, 0.f}; }
#if CONV_STAMP
  unsigned long long st_ep[6] = {conv_stamp(), 0, 0, 0, 0, 0};
#endif
  if constexpr (CTE) {
    EUNET_DASSERT(a.stats == nullptr);
    // C^T accumulators: lane (q, li) holds, per (mt, nt), channels co0 + 16 nt + 4 q .. + 3 of the pixel in
    // m-tile mt, column li.  The tile is staged as bf16 [512 px][CLD] in ONE pass (4 channels = one 8-byte
    // LDS store: 32 per thread, where the fp32 [px][OUT_LD] staging took 128 4-byte stores in two passes),
    // then each thread stores 16 whole 16-byte units (and, BNB, reduces them with y).  No forward BN
    // statistics in a data gradient.
    constexpr int CLD = 72;  // bf16 per staged pixel row (144 B: 16-byte aligned unit reads)
    constexpr int SJ1 = FTH * FTW * UPX / NTH;  // 16 units per thread
    static_assert(FTH * FTW * CLD * 2 + 4 * BN * 4 <= FWD_LDS, "C^T epilogue LDS");
    static_assert(NTH / UPX == FTW, "unit step j = tile row j");
    bf16_t* const stgb = (bf16_t*)smem;
    float* const bprm2 = (float*)(smem + FTH * FTW * CLD * 2);
    const int vh = min(FTH, a.H - y0), vw = min(FTW, a.W - x0);
    if (a.bias != nullptr || a.gsc != nullptr) {  // (uniform: most data gradients have neither)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        f32x4 b4, g4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = co0 + nt * 16 + 4 * q + i;
          b4[i] = (a.bias != nullptr && co < a.cout) ? a.bias[co] : 0.f;
          g4[i] = (a.gsc != nullptr && co < a.cout) ? a.gsc[(long long)n * a.cout + co] : 1.f;
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f32x2 lo = ((f32x2){acc[mt][nt][0], acc[mt][nt][1]} + (f32x2){b4[0], b4[1]}) * (f32x2){g4[0], g4[1]};
          const f32x2 hi = ((f32x2){acc[mt][nt][2], acc[mt][nt][3]} + (f32x2){b4[2], b4[3]}) * (f32x2){g4[2], g4[3]};
          acc[mt][nt] = (f32x4){lo.x, lo.y, hi.x, hi.y};
        }
      }
    }
    // (pixels outside the image are staged but never stored or reduced: no masking of the accumulators)
    const long long yrs = (long long)a.W * a.yct;
    const long long tile_px = (long long)(n * a.H + y0) * a.W + x0;
    T* const ybase = (T*)a.y + tile_px * a.yct + a.yco + co0;
    const long long brs = (long long)a.W * a.byct;
    const T* const bybase = BNB ? (const T*)a.by + tile_px * a.byct + a.byco + co0 : nullptr;
    const int c = tid / UPX, cu = co0 + ucol * E;
    uint4 ryb[BNB ? SJ1 : 1];
    auto load_y = [&](int j0, int j1) {  // y of this thread's units j0..j1-1 (BN-backward input)
      if constexpr (BNB) {
#pragma unroll
        for (int j = j0; j < j1; ++j) {
          ryb[j] = make_uint4(0, 0, 0, 0);
          if (j < vh && c < vw && cu < a.cout) ryb[j] = *(const uint4*)(bybase + (long long)j * brs + (c * a.byct + ucol * E));
        }
      }
    };
    load_y(0, SJ1 / 2);  // (the accumulators are still live: half now, half after they are staged)
    __syncthreads();  // all waves are done with the K loop's LDS
    if (bnb && tid < BN) {
      const bool ok = co0 + tid < a.cout;
      bprm2[tid] = ok ? a.bmean[co0 + tid] : 0.f;
      bprm2[BN + tid] = ok ? a.bistd[co0 + tid] : 0.f;
      bprm2[2 * BN + tid] = ok ? a.bsc[co0 + tid] : 0.f;
      bprm2[3 * BN + tid] = ok ? a.bsh[co0 + tid] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int px = (RPW * wv + (mt >> 1)) * FTW + (mt & 1) * 16 + li;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        *(uint2*)(stgb + px * CLD + nt * 16 + 4 * q) =
            make_uint2(pk_bf16(acc[mt][nt][0], acc[mt][nt][1]), pk_bf16(acc[mt][nt][2], acc[mt][nt][3]));
    }
    load_y(SJ1 / 2, SJ1);
    __syncthreads();
    f32x2 km[E / 2], ki[E / 2], ks[E / 2], kh[E / 2];  // BN-backward mean, istd, scale, shift of the unit
    if constexpr (BNB) {
#pragma unroll
      for (int e = 0; e < E / 2; ++e) {
        const int cc = ucol * E + 2 * e;
        km[e] = *(const f32x2*)(bprm2 + cc);
        ki[e] = *(const f32x2*)(bprm2 + BN + cc);
        ks[e] = *(const f32x2*)(bprm2 + 2 * BN + cc);
        kh[e] = *(const f32x2*)(bprm2 + 3 * BN + cc);
      }
    }
#pragma unroll
    for (int j = 0; j < SJ1; ++j) {  // unit (pixel row j, column c, channel unit ucol)
      if (j < vh && c < vw && cu < a.cout) {
        const uint4 packed = *(const uint4*)(stgb + (j * FTW + c) * CLD + ucol * E);
        const long long off = (long long)j * yrs + (c * a.yct + ucol * E);
        EUNET_DASSERT(tile_px + (long long)j * a.W + c < (long long)a.N * a.H * a.W && cu + E <= a.cout &&
                      a.yco + cu + E <= a.yct);
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, packed), (u32x4*)(ybase + off));
        if constexpr (BNB) {
          float gr[E], yv[E];
          Vec16<T>::unpack(packed, gr);
          Vec16<T>::unpack(ryb[j], yv);
#pragma unroll
          for (int e = 0; e < E; e += 2) {  // packed fp32: each element rounded as the scalar ops round it
            const f32x2 y2 = {yv[e], yv[e + 1]};
            const f32x2 xh = (y2 - km[e >> 1]) * ki[e >> 1];
            const f32x2 pre = __builtin_elementwise_fma(y2, ks[e >> 1], kh[e >> 1]);
            const f32x2 gp = {pre.x > 0.f ? gr[e] : 0.f, pre.y > 0.f ? gr[e + 1] : 0.f};
            bp1[e >> 1] += gp;
            bp2[e >> 1] = __builtin_elementwise_fma(gp, xh, bp2[e >> 1]);
          }
        }
      }
    }
  } else {
    // ---- epilogue: bias, BN partials, LDS-staged vector stores (NPASS row bands) ----
    constexpr int NCW = NW;
    const int vh = min(FTH, a.H - y0), vw = min(FTW, a.W - x0);
    // Bias (and, dgrad only, the Dropout2d scale) in packed fp32; on a partial tile the accumulators of
    // pixels outside the image are zeroed afterwards (a uniform branch), so the BN sums below need no
    // per-element masks: the sum over all 128 values of a wave's rows is the sum over its valid ones, and
    // its M2 about the valid mean is the all-element M2 less (invalid count) x mean^2.  Two packed ops per
    // pair of values instead of six scalar ops per value (SQ: 5.1 VALU instructions per MFMA on the
    // 64-channel layers, profiles/r04_sq_layers.txt).
  #pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int co = co0 + nt * 16 + li;
      const float bv = (a.bias != nullptr && co < a.cout) ? a.bias[co] : 0.f;
      const f32x2 b2 = {bv, bv};
      if constexpr (DG) {
        const float gv = (a.gsc != nullptr && co < a.cout) ? a.gsc[(long long)n * a.cout + co] : 1.f;
        const f32x2 g2 = {gv, gv};
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f32x2 lo = ((f32x2){acc[mt][nt][0], acc[mt][nt][1]} + b2) * g2;
          const f32x2 hi = ((f32x2){acc[mt][nt][2], acc[mt][nt][3]} + b2) * g2;
          acc[mt][nt] = (f32x4){lo.x, lo.y, hi.x, hi.y};
        }
      } else {
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f32x2 lo = (f32x2){acc[mt][nt][0], acc[mt][nt][1]} + b2;
          const f32x2 hi = (f32x2){acc[mt][nt][2], acc[mt][nt][3]} + b2;
          acc[mt][nt] = (f32x4){lo.x, lo.y, hi.x, hi.y};
        }
      }
    }
    if (vh < FTH || vw < FTW) {  // partial tile (image edge): zero the pixels outside the image
  #pragma unroll
      for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = RPW * wv + (mt >> 1) < vh && (mt & 1) * 16 + q * 4 + i < vw;
  #pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc[mt][nt][i] = ok ? acc[mt][nt][i] : 0.f;
        }
    }
    constexpr int PASS_PX = PROWS * FTW;
    float* stg = (float*)smem;                                    // [PASS_PX][OUT_LD]
    float* red = (float*)(smem + PASS_PX * OUT_LD * 4);           // [NCW][64] x 2
    float* bprm = red + 2 * NCW * 64;                             // [4][64] BN-backward constants
    static_assert(PASS_PX * OUT_LD * 4 + (2 * NCW + 4) * 64 * 4 <= FWD_LDS, "epilogue LDS");
    __syncthreads();  // all waves are done with the K loop's LDS
    if (a.stats != nullptr) {
      // per wave: its rows' channel sums and M2 about the wave's own mean, both from the fp32
      // accumulators (two register passes, lane sums by the permlane swaps); the 4 waves are then
      // Chan-combined by 64 threads -- one barrier, one LDS round trip
      const int nw = max(0, min(RPW, vh - RPW * wv)) * vw;  // valid pixels in this wave's rows
      const float inv_nw = nw > 0 ? 1.f / (float)nw : 0.f;
      const bool part = vh < FTH || vw < FTW;                 // block-uniform: an edge tile
      float s1[4], s2[4];
  #pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        f32x2 v = {0.f, 0.f};
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt) v += (f32x2){acc[mt][nt][0], acc[mt][nt][1]} + (f32x2){acc[mt][nt][2], acc[mt][nt][3]};
        s1[nt] = xor32_sum(xor16_sum(v.x + v.y));
      }
  #pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float mw = s1[nt] * inv_nw;
        const f32x2 m2 = {-mw, -mw};
        f32x2 v = {0.f, 0.f};
        if (!part) {
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const f32x2 d0 = (f32x2){acc[mt][nt][0], acc[mt][nt][1]} + m2;
            const f32x2 d1 = (f32x2){acc[mt][nt][2], acc[mt][nt][3]} + m2;
            v = __builtin_elementwise_fma(d0, d0, v);
            v = __builtin_elementwise_fma(d1, d1, v);
          }
        } else {  // the pixels outside the image contribute nothing (no (0 - mw)^2 to cancel afterwards)
  #pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const bool rok = RPW * wv + (mt >> 1) < vh;
            const int c0 = (mt & 1) * 16 + q * 4;
            f32x2 d0 = (f32x2){acc[mt][nt][0], acc[mt][nt][1]} + m2;
            f32x2 d1 = (f32x2){acc[mt][nt][2], acc[mt][nt][3]} + m2;
            d0.x = rok && c0 + 0 < vw ? d0.x : 0.f;
            d0.y = rok && c0 + 1 < vw ? d0.y : 0.f;
            d1.x = rok && c0 + 2 < vw ? d1.x : 0.f;
            d1.y = rok && c0 + 3 < vw ? d1.y : 0.f;
            v = __builtin_elementwise_fma(d0, d0, v);
            v = __builtin_elementwise_fma(d1, d1, v);
          }
        }
        s2[nt] = xor32_sum(xor16_sum(v.x + v.y));
      }
      if (q == 0)
  #pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          red[wv * 64 + nt * 16 + li] = s1[nt];
          red[NCW * 64 + wv * 64 + nt * 16 + li] = s2[nt];
        }
      __syncthreads();
      const float cnt = (float)(vh * vw);
      if (tid < 64 && co0 + tid < a.cout) {
        float sum = 0.f, m2 = 0.f;
  #pragma unroll
        for (int w = 0; w < NCW; ++w) sum += red[w * 64 + tid];
        const float mean = sum / cnt;
  #pragma unroll
        for (int w = 0; w < NCW; ++w) {
          const int nwv = max(0, min(RPW, vh - RPW * w)) * vw;
          if (nwv > 0) {
            const float d = red[w * 64 + tid] / (float)nwv - mean;
            m2 += red[NCW * 64 + w * 64 + tid] + (float)nwv * d * d;
          }
        }
        a.stats[((long long)tile * 2 + 0) * a.cout + co0 + tid] = sum;
        a.stats[((long long)tile * 2 + 1) * a.cout + co0 + tid] = m2;
      }
      if (cob == 0 && tid == 0) a.stats[(long long)2 * a.cout * a.ntiles + tile] = cnt;
    }
  #if CONV_STAMP
    st_ep[0] = conv_stamp();
  #endif
    T* yp = (T*)a.y;
    f32x2 km[E / 2], ki[E / 2], ks[E / 2], kh[E / 2];  // BN-backward mean, istd, scale, shift of the unit
    if (bnb && tid < BN) {
      const bool ok = co0 + tid < a.cout;
      bprm[tid] = ok ? a.bmean[co0 + tid] : 0.f;
      bprm[BN + tid] = ok ? a.bistd[co0 + tid] : 0.f;
      bprm[2 * BN + tid] = ok ? a.bsc[co0 + tid] : 0.f;
      bprm[3 * BN + tid] = ok ? a.bsh[co0 + tid] : 0.f;
    }
    constexpr int SJ = PASS_PX * UPX / NTH;      // output units per thread per pass
    constexpr int PXJ = NTH / UPX;                // pixels per unit step
    static_assert(FTW % PXJ == 0, "a unit step covers a fraction of one tile row (row compile-time per step)");
    const int tu = tid;
    // output / y addresses: a block-uniform base (the tile's corner) + row x row stride + the thread's
    // (column, unit) offset, instead of a 64-bit pixel index per unit
    const long long yrs = (long long)a.W * a.yct;
    const long long tile_px = (long long)(n * a.H + y0) * a.W + x0;
    T* const ybase = yp + tile_px * a.yct + a.yco + co0;
    float* const yfbase = (float*)a.y + tile_px * a.yct + a.yco + co0;
    const long long brs = (long long)a.W * a.byct;
    const T* const bybase = BNB ? (const T*)a.by + tile_px * a.byct + a.byco + co0 : nullptr;
    constexpr bool PRE = sizeof(T) == 2;         // bf16: prefetch the pass's y (BN-backward input)
  #pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
      // the fused BN-backward reduction reads y at every output unit: issue those loads before the
      // staging barrier so their latency overlaps it (the stores below would otherwise serialise
      // each load behind the previous unit's store)
      uint4 ryb[PRE ? SJ : 1];
      if constexpr (PRE) {
        if (bnb) {
  #pragma unroll
          for (int j = 0; j < SJ; ++j) {
            const int r = pass * PROWS + (PXJ * j) / FTW, c = tu / UPX + (PXJ * j) % FTW, u = ucol;
            const int co = co0 + u * E;
            ryb[j] = make_uint4(0, 0, 0, 0);
            if (r < vh && c < vw && co < a.cout)
              ryb[j] = *(const uint4*)(bybase + (long long)r * brs + (c * a.byct + u * E));
          }
        }
      }
      if (RPW * wv >= pass * PROWS && RPW * wv < (pass + 1) * PROWS) {
  #pragma unroll
        for (int mt = 0; mt < MT; ++mt)
  #pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int px = (RPW * wv - pass * PROWS + (mt >> 1)) * FTW + (mt & 1) * 16 + q * 4 + i;
  #pragma unroll
            for (int nt = 0; nt < 4; ++nt) stg[px * OUT_LD + nt * 16 + li] = acc[mt][nt][i];
          }
      }
      __syncthreads();
  #if CONV_STAMP
      st_ep[1 + 2 * pass] = conv_stamp();
  #endif
      if (BNB && pass == 0) {  // this thread's channel unit is fixed: its BN-backward constants into registers
  #pragma unroll
        for (int e = 0; e < E / 2; ++e) {
          const int cc = ucol * E + 2 * e;
          km[e] = *(const f32x2*)(bprm + cc);
          ki[e] = *(const f32x2*)(bprm + BN + cc);
          ks[e] = *(const f32x2*)(bprm + 2 * BN + cc);
          kh[e] = *(const f32x2*)(bprm + 3 * BN + cc);
        }
      }
  #pragma unroll
      for (int j = 0; j < SJ; ++j) {
        // unit tid + j NTH = (pixel px, channel unit u): u = tid mod UPX, px = tid / UPX + PXJ j, and since
        // PXJ divides FTW the row of px is compile-time per (pass, j)
        const int r = pass * PROWS + (PXJ * j) / FTW, c = tu / UPX + (PXJ * j) % FTW, u = ucol;
        const int px = (r - pass * PROWS) * FTW + c;
        const int co = co0 + u * E;
        if (r < vh && c < vw && co < a.cout) {
          const float* sp = stg + px * OUT_LD + u * E;
          float f[E];
  #pragma unroll
          for (int e = 0; e < E; ++e) f[e] = sp[e];
          const long long off = (long long)r * yrs + (c * a.yct + u * E);
          EUNET_DASSERT(tile_px + (long long)r * a.W + c < (long long)a.N * a.H * a.W && co + E <= a.cout &&
                        a.yco + co + E <= a.yct);
          const uint4 packed = Vec16<T>::pack(f);
          if constexpr (sizeof(TO) == sizeof(T)) {  // (non-temporal: the output is read back after it left L2)
            __builtin_nontemporal_store(__builtin_bit_cast(u32x4, packed), (u32x4*)(ybase + off));
          } else {  // fp32 output of a bf16 kernel: E = 8 floats, two 16-byte stores
            float* yo = yfbase + off;
            *(float4*)yo = make_float4(f[0], f[1], f[2], f[3]);
            *(float4*)(yo + 4) = make_float4(f[4], f[5], f[6], f[7]);
          }
          if constexpr (BNB) {
            float gr[E], yv[E];
            Vec16<T>::unpack(packed, gr);
            if constexpr (PRE) Vec16<T>::unpack(ryb[j], yv);
            else Vec16<T>::unpack(*(const uint4*)(bybase + (long long)r * brs + (c * a.byct + u * E)), yv);
  #pragma unroll
            for (int e = 0; e < E; e += 2) {  // packed fp32: each element rounded as the scalar ops round it
              const f32x2 y2 = {yv[e], yv[e + 1]};
              const f32x2 xh = (y2 - km[e >> 1]) * ki[e >> 1];
              const f32x2 pre = __builtin_elementwise_fma(y2, ks[e >> 1], kh[e >> 1]);
              const f32x2 gp = {pre.x > 0.f ? gr[e] : 0.f, pre.y > 0.f ? gr[e + 1] : 0.f};
              bp1[e >> 1] += gp;
              bp2[e >> 1] = __builtin_elementwise_fma(gp, xh, bp2[e >> 1]);
            }
          }
        }
      }
  #if CONV_STAMP
      st_ep[2 + 2 * pass] = conv_stamp();
  #endif
      if (pass + 1 < NPASS) __syncthreads();
    }
  }
  if (bnb) {  // fixed-order reduction of the per-thread channel sums: the lanes of a wave that share a
             // channel unit (lane = ucol mod UPX) by DPP / permlane xor sums, then the 4 waves through LDS
    float bs1[E], bs2[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float v1 = bp1[e >> 1][e & 1], v2 = bp2[e >> 1][e & 1];
      if constexpr (UPX == 8) {  // lane bit 3: row_ror:8 within each row of 16 lanes
        v1 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v1), 0x128, 0xF, 0xF, false));
        v2 += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v2), 0x128, 0xF, 0xF, false));
      }
      bs1[e] = xor32_sum(xor16_sum(v1));
      bs2[e] = xor32_sum(xor16_sum(v2));
    }
    __syncthreads();
    float* r2 = (float*)smem;  // [NW waves][UPX units][2E]
    if (lane < UPX) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        r2[(wv * UPX + lane) * 2 * E + e] = bs1[e];
        r2[(wv * UPX + lane) * 2 * E + E + e] = bs2[e];
      }
    }
    __syncthreads();
    if (tid < 2 * BN) {
      const int which = tid / BN, cc = tid % BN, u = cc / E, e = cc % E;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += r2[(w * UPX + u) * 2 * E + which * E + e];
      if (co0 + cc < a.cout) a.bpart[((long long)tile * 2 + which) * a.cout + co0 + cc] = t;
    }
  }
#if CONV_STAMP
  const unsigned long long st_e = conv_stamp();
  if (tid == 0 && blockIdx.x < STAMP_BLOCKS) {
    unsigned long long* o = g_conv_stamps + (size_t)blockIdx.x * STAMP_N;
    o[0] = st_t0;
    o[1] = st_e - st_t0;
    o[2] = st_stage;
    o[3] = st_mfma;
    o[4] = st_e - st_a;
    o[5] = st_ep[0] - st_a;
    o[6] = st_ep[1] - st_ep[0];
    o[7] = st_ep[2] - st_ep[1];
    o[8] = st_ep[3] - st_ep[2];
    o[9] = st_ep[4] - st_ep[3];
    o[10] = st_e - st_ep[4];
  }
#endif
}


// ---------------------------------------------------------------------------
// weight packing: torch [Cout][Cin][3][3] fp32 -> [Cin_p/KC][4][Cout_p][9][E]
// transpose_flip: pack W'[o=ci][i=co][t] = W[co][ci][8-t] (dgrad operand)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void pack_elem(const float* w, int cout, int cin, int flip, T* wp, int cout_p, int cin_p,
                                          long long id) {
  constexpr int E = Vec16<T>::N, KC = KCh<T>::v;
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

template <typename T>
__global__ void pack_kernel(const float* w, int cout, int cin, int flip, T* wp, int cout_p, int cin_p) {
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id < (long long)cin_p * cout_p * 9) pack_elem<T>(w, cout, cin, flip, wp, cout_p, cin_p, id);
}

// every weight tensor of a step packed in one launch: the blocks of tensor i are
// [bstart[i], bstart[i + 1]) of a flat grid (no idle blocks for the small tensors), a thread
// writes one 16-byte unit of E consecutive GEMM input channels (same values as pack_elem)
struct PackBatch {
  eunet_pack_desc d[EUNET_PACK_MAX];
  int cout_p[EUNET_PACK_MAX], cin_p[EUNET_PACK_MAX];
  int bstart[EUNET_PACK_MAX + 1];
  int n;
};
template <typename T>
__global__ __launch_bounds__(256) void pack_many_kernel(PackBatch b) {
  constexpr int E = Vec16<T>::N, KC = KCh<T>::v;
  const int bid = blockIdx.x;
  int k = 0;
  for (int i = 1; i < b.n; ++i) k = bid >= b.bstart[i] ? i : k;  // block-uniform
  const eunet_pack_desc& d = b.d[k];
  const int cout_p = b.cout_p[k];
  const long long u = (long long)(bid - b.bstart[k]) * 256 + threadIdx.x;  // 16-byte unit
  if (u >= (long long)b.cin_p[k] * cout_p * 9 / E) return;
  long long r = u;
  const int t = (int)(r % 9); r /= 9;
  const int o = (int)(r % cout_p); r /= cout_p;
  const int qq = (int)(r % 4);
  const int kc = (int)(r / 4);
  const int i0 = kc * KC + qq * E;
  float v[E];
  bool ok[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {  // every load first (index 0 for padding), then the selects
    const int i = i0 + e;
    ok[e] = d.flip ? (o < d.cin && i < d.cout) : (o < d.cout && i < d.cin);
    const long long src = !ok[e] ? 0 : d.flip ? ((long long)i * d.cin + o) * 9 + (8 - t) : ((long long)o * d.cin + i) * 9 + t;
    v[e] = d.w[src];
  }
#pragma unroll
  for (int e = 0; e < E; ++e) asm volatile("" : "+v"(v[e]));
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = ok[e] ? v[e] : 0.f;
  *(uint4*)((T*)d.wp + u * E) = Vec16<T>::pack(v);
}

// ---------------------------------------------------------------------------
// wgrad
// ---------------------------------------------------------------------------
struct WgArgs {
  const void* x; int N, H, W, xct, xco, cin;
  const float* isc; const float* ish; int iss;
  const void* dy; int dct, dco, cout;
  float* dw; float* db;
  int tx, ty, ntiles, per_split, nsplit;
};

// LDS layout of the wgrad stages.  A ds_read_b64_tr_b16 serves 2 x 32 lanes; a 32-lane half reads 8
// consecutive pixels of one tile row (lo: columns 0-7, hi: 8-15 of the k-step's row) x 2 channel groups x 2
// 8-byte halves -- 256 bytes that must cover the 64 banks once:
//  - dY tile [128 px][8 units of 16 B]: pixel p's channel unit u is stored at unit u ^ wd_swz(p), p & 6: the
//    4 same-parity pixels of a read (one 256-byte row holds 2 pixels) take 4 distinct unit rotations;
//  - X halo [4 octant pairs][DPL][2 octants x 16 B]: a read's 8 pixels x 2 octants of its wave's pair are 16
//    consecutive 16-byte slots.  A pixel's octant pair is 32 contiguous bytes in global memory, so a DMA
//    wave-instruction touches 32 lines (octant planes: 64, round-6 r6wc).
__device__ __forceinline__ int wd_swz(int p) { return p & 6; }

// Block order: logical L = (split, co-block, ci-block), ci fastest, XCD-contiguous
// (see xcd_map): the blocks sharing a split's X / dY tiles share one L2.
__device__ __forceinline__ void wg_map(int b, int nsplit, int ncob, int ncib, int& split, int& cob, int& cib) {
  const int total = nsplit * ncob * ncib, full = total & ~7;
  const int L = b < full ? (b & 7) * (full >> 3) + (b >> 3) : b;
  cib = L % ncib;
  const int r = L / ncib;
  cob = r % ncob;
  split = r / ncob;
}

// bf16 wgrad: pixels are the GEMM K.  Block = (pixel split, 64 co, 64 ci); wave w owns ci 16w..16w+15 for all
// 64 co and 9 taps (36 accumulators): a 32-pixel k-step is 8 dY^T + 18 X transposed fragment reads
// (ds_read_b64_tr_b16) for 36 MFMAs.  Two blocks per CU.  Split partials are reduced in fixed order in fp64
// (wgrad_reduce).  Round 6: double-buffered over 8 x 16-pixel tiles, whose X halo + dY tile (40 KB) fit twice
// in a block's 80 KB of LDS, so tile t + 1 is copied by LDS-DMA while tile t's MFMAs run (the round-5 kernel
// staged 8 x 32 tiles into one stage: with its copies skipped after a split's first tile -- a diagnostic with
// wrong results -- the 13 layers ran 3.72 vs 4.86 ms, profiles/r06_ab.txt r6wn).  The copies are issued by inline asm (buffer_load_dwordx4 ... lds, M0 = the
// LDS destination), so the compiler sees no LDS-DMA: it would otherwise order every LDS read of the current
// stage behind the other stage's copy in flight (vmcnt(0)).  The waits are explicit instead: vmcnt(0) before
// the barrier that opens a tile (its copy, issued one tile earlier, has landed), and the barrier after the
// in-place BN+ReLU pass is lgkmcnt(0) + s_barrier (no fence: __syncthreads' would wait for the copy).
constexpr int KCW = 64;                         // ci channels per block
constexpr int DTH = 8, DTW = 16;                // pixel tile
constexpr int DHW = DTW + 2;                    // 18
constexpr int DHPX = (DTH + 2) * DHW;           // 180 halo pixels
constexpr int DPL = 384;                        // octant-pair plane (slots): 2 x 180 used, 6144 B = 24 bank rows
constexpr int DWX = 4 * DPL * 16;               // X halo [4 pairs][DPL][16 B]
constexpr int DWD = DTH * DTW * 64 * 2;         // dY tile [128 px][64 co] bf16
constexpr int DSTAGE = DWX + DWD;               // 40960
constexpr int DWX_ITERS = 4 * DPL / NTHR;       // 6 wave-instructions per wave
constexpr int DWD_ITERS = DTH * DTW * 8 / NTHR; // 4
static_assert(4 * DPL == NTHR * DWX_ITERS && DTH * DTW * 8 == NTHR * DWD_ITERS, "whole wave-instructions");
static_assert(2 * DHPX <= DPL && DPL % 16 == 0, "a pair plane holds the halo, bank-row aligned");
static_assert(2 * DSTAGE <= 80 * 1024, "two stages per block, two blocks per CU");
static_assert(DPL > NTHR, "dma_x: one pair-plane boundary per wave-instruction range at most");

// 16 bytes per lane from buffer rsrc at byte offset voff (range-checked: out of range reads zeros) into LDS at
// M0 + 16 lane; lds must be wave-uniform
__device__ __forceinline__ void dma16_lds(u32x4 rsrc, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(lds), "v"(voff), "s"(rsrc) : "memory", "m0");
}
__device__ __forceinline__ u32x4 rsrc_of(const void* base, uint32_t bytes) {
  const unsigned long long b = (unsigned long long)base;
  return (u32x4){(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b),
                 (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32)),
                 (uint32_t)__builtin_amdgcn_readfirstlane((int)bytes), 0x00020000u};
}

__global__ __launch_bounds__(NTHR, 2) void conv3x3_wgrad_bf16_kernel(WgArgs a) {
  __shared__ __attribute__((aligned(16))) char wst[2 * DSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int split, cob, kc;
  wg_map(blockIdx.x, a.nsplit, cdiv(a.cout, 64), cdiv(a.cin, KCW), split, cob, kc);
  const int co0 = cob * 64;
  const int t_begin = split * a.per_split;
  const int t_end = min(a.ntiles, t_begin + a.per_split);
  EUNET_DASSERT(split < a.nsplit && co0 < a.cout && kc * KCW < a.cin && t_begin < a.ntiles);
  const int tpi = a.tx * a.ty;
  const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  // a lane's k-step pixels: lo = row 2 ks + (g >> 1), column 4 (g & 1) + q4; hi = 8 columns on (same wd_swz)
  const int pcol = 4 * (g & 1) + q4;
  const int sw16 = (((p4 >> 1) ^ wd_swz(pcol)) * 8 + 4 * (p4 & 1)) * 2;

  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[t][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x2 dbv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) dbv[e] = (f32x2){0.f, 0.f};
  if (blockIdx.x & 1) __builtin_amdgcn_s_sleep(40);  // phase offset (conv3x3_fwd_kernel)

  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)wst;  // LDS byte address
  const uint32_t wlds = lds0 + (uint32_t)__builtin_amdgcn_readfirstlane(wv) * 1024u;    // + this wave's 1 KB
  // dY unit tid + 256 i = tile pixel p = (tid >> 3) + 32 i (row 2 i + (tid >> 7), column (tid >> 3) & 15),
  // LDS unit tid & 7 holding channel unit du
  const int dp = tid >> 3, dcol = dp & (DTW - 1), drow = dp >> 4, du = (tid & 7) ^ wd_swz(dp);
  const bool dch_ok = co0 + du * 8 < a.cout;
  const uint32_t rstep = (uint32_t)(a.W * a.dct) * 2u;
  const uint32_t dlane = (uint32_t)((dcol * a.dct + a.dco + co0 + du * 8) * 2) + (uint32_t)drow * rstep;
  const uint32_t dslice = (uint32_t)(a.H * a.W * a.dct) * 2u, xslice = (uint32_t)(a.H * a.W * a.xct) * 2u;
  auto dma_d = [&](int st, int n, int y0, int x0) {
    const u32x4 dr = rsrc_of((const bf16_t*)a.dy + (long long)n * a.H * a.W * a.dct, dslice);
    const bool xok = dch_ok & (dcol < a.W - x0);
    const uint32_t rb = (uint32_t)((y0 * a.W + x0) * a.dct) * 2u;
    const uint32_t l = wlds + (uint32_t)(st * DSTAGE + DWX);
#pragma unroll
    for (int i = 0; i < DWD_ITERS; ++i) {
      const bool ok = xok & (y0 + 2 * i + drow < a.H);
      const uint32_t off = dlane + rb + 2u * i * rstep;
      EUNET_DASSERT(!ok || off + 16u <= dslice);
      dma16_lds(dr, ok ? off : FWD_OOB, l + 4096u * i);
    }
  };
  // X halo raw into LDS: slot s = tid + 256 i = (oc >> 1) * DPL + 2 hp + (oc & 1)
  auto dma_x = [&](int st, int n, int y0, int x0) {
    const u32x4 xr = rsrc_of((const bf16_t*)a.x + (long long)n * a.H * a.W * a.xct, xslice);
    const int tb = ((y0 - 1) * a.W + (x0 - 1)) * a.xct + a.xco + kc * KCW;  // element (y0 - 1, x0 - 1)
    const uint32_t l = wlds + (uint32_t)(st * DSTAGE);
    int t = tid;
    asm volatile("" : "+v"(t));  // per tile: hoisted, the 6 lanes' offsets and masks would be live across the k-loop
#pragma unroll
    for (int i = 0; i < DWX_ITERS; ++i) {
      const int k = NTHR * i / DPL, tk = DPL * (k + 1) - NTHR * i;
      const bool bump = tk < NTHR && t >= tk;
      const int pr = k + bump, r = t + NTHR * i - DPL * pr;
      const int oc = 2 * pr + (r & 1), hp = r >> 1;
      const int hy = (int)((uint32_t)hp / DHW), hx = hp - hy * DHW;
      const bool ok = ((uint32_t)hp < (uint32_t)DHPX) & ((uint32_t)(y0 - 1 + hy) < (uint32_t)a.H) &
                      ((uint32_t)(x0 - 1 + hx) < (uint32_t)a.W) & (kc * KCW + oc * 8 < a.cin);
      const uint32_t off = (uint32_t)(tb + (hy * a.W + hx) * a.xct + oc * 8) * 2u;
      EUNET_DASSERT(!ok || off + 16u <= xslice);
      dma16_lds(xr, ok ? off : FWD_OOB, l + 4096u * i);
    }
  };
  // BN+ReLU of the staged halo in place (padding stays 0): wave w owns pair plane w -- octants 2w, 2w + 1, the
  // ones its fragment reads use -- lane l its slots l + 64 j (octant 2w + (l & 1), pixel (l >> 1) + 32 j); the
  // octant's 8 scales / shifts are loaded before the tile's opening barrier
  const int xo = 2 * wv + (lane & 1);
  const bool xo_ok = kc * KCW + xo * 8 < a.cin;
  auto load_aff = [&](int n, f32x4* sc) {
    const float* ps = a.isc + (long long)n * a.iss + kc * KCW + xo * 8;
    const float* ph = a.ish + (long long)n * a.iss + kc * KCW + xo * 8;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    sc[0] = xo_ok ? *(const f32x4*)ps : z;
    sc[1] = xo_ok ? *(const f32x4*)(ps + 4) : z;
    sc[2] = xo_ok ? *(const f32x4*)ph : z;
    sc[3] = xo_ok ? *(const f32x4*)(ph + 4) : z;
  };
  auto bnrelu_x = [&](char* S, int y0, int x0, const f32x4* sc) {
    if (!xo_ok) return;
    const float scv[8] = {sc[0][0], sc[0][1], sc[0][2], sc[0][3], sc[1][0], sc[1][1], sc[1][2], sc[1][3]};
    const float shv[8] = {sc[2][0], sc[2][1], sc[2][2], sc[2][3], sc[3][0], sc[3][1], sc[3][2], sc[3][3]};
    char* const plane = S + (wv * DPL + lane) * 16;
    constexpr int G = 3, NI = (2 * DHPX + 63) / 64;  // 6 slot rounds in 2 groups of 3
    static_assert(NI % G == 0, "bnrelu_x groups");
    static_assert((3 * DPL + 63 + 64 * (NI - 1) + 1) * 16 <= DSTAGE, "bnrelu_x: group reads stay inside the stage");
#pragma unroll 1
    for (int i0 = 0; i0 < NI; i0 += G) {
      u32x4 w[G];
      bool ok[G];
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int hp = (lane >> 1) + 32 * (i0 + j), hy = hp / DHW, hx = hp - hy * DHW;
        const int yy = y0 + hy - 1, xx = x0 + hx - 1;
        ok[j] = (hp < DHPX) & ((uint32_t)yy < (uint32_t)a.H) & ((uint32_t)xx < (uint32_t)a.W);
        w[j] = *(const u32x4*)(plane + 64 * (i0 + j) * 16);
      }
#pragma unroll
      for (int j = 0; j < G; ++j) {
        u32x4 o;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const f32x2 x = {__uint_as_float(w[j][d] << 16), __uint_as_float(w[j][d] & 0xFFFF0000u)};
          const f32x2 r = __builtin_elementwise_fma(x, (f32x2){scv[2 * d], scv[2 * d + 1]}, (f32x2){shv[2 * d], shv[2 * d + 1]});
          const s16x2 b = __builtin_bit_cast(s16x2, pk_bf16(r[0], r[1]));
          o[d] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(b, (s16x2){0, 0}));
        }
        if (ok[j]) *(u32x4*)(plane + 64 * (i0 + j) * 16) = o;
      }
    }
  };
  // tile coordinates advance incrementally (scalar): sample tn, tile row tyi, tile column txi
  int tn = t_begin / tpi, tyi = (t_begin - tn * tpi) / a.tx, txi = t_begin - tn * tpi - tyi * a.tx;
  const bool tf = a.isc != nullptr;
  {  // the split's first tile into stage 0
    const int n = __builtin_amdgcn_readfirstlane(tn);
    dma_x(0, n, __builtin_amdgcn_readfirstlane(tyi) * DTH, __builtin_amdgcn_readfirstlane(txi) * DTW);
    dma_d(0, n, __builtin_amdgcn_readfirstlane(tyi) * DTH, __builtin_amdgcn_readfirstlane(txi) * DTW);
  }
  for (int tile = t_begin; tile < t_end; ++tile) {
    const int st = (tile - t_begin) & 1;
    char* const S = wst + st * DSTAGE;
    const int n = __builtin_amdgcn_readfirstlane(tn);
    const int y0 = __builtin_amdgcn_readfirstlane(tyi) * DTH, x0 = __builtin_amdgcn_readfirstlane(txi) * DTW;
    if (++txi == a.tx) {
      txi = 0;
      if (++tyi == a.ty) { tyi = 0; ++tn; }
    }
    f32x4 sc[4];
    if (tf) load_aff(n, sc);
    // this tile's copy (issued a tile earlier) has landed; every wave is done reading the other stage.  The
    // wait is the builtin, so the compiler knows its own loads (the scales) are complete too and puts no
    // vmcnt(0) before their use -- which would wait for the next tile's copy
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    if (tile + 1 < t_end) {
      const int n1 = __builtin_amdgcn_readfirstlane(tn);
      const int y1 = __builtin_amdgcn_readfirstlane(tyi) * DTH, x1 = __builtin_amdgcn_readfirstlane(txi) * DTW;
      dma_x(st ^ 1, n1, y1, x1);
      dma_d(st ^ 1, n1, y1, x1);
    }
    if (tf) {
      // wave w transforms octants 2w, 2w + 1 (threads tid >> 5), which are exactly the X octants its own
      // fragment reads use (oc = 2 wv + (p4 >> 1)): its LDS writes precede its reads in program order, so no
      // block barrier -- each wave starts its MFMAs when its own octants are done
      bnrelu_x(S, y0, x0, sc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const char* const Xs = S;
    const char* const Ds = S + DWX;
    if (a.db != nullptr && kc == 0) {
      const bf16_t* d = (const bf16_t*)Ds;
#pragma unroll
      for (int i = 0; i < DTH * DTW / 32; ++i) {
        const int px = (tid >> 3) + 32 * i;
        const u32x4 w = *(const u32x4*)(d + px * 64 + ((tid & 7) ^ wd_swz(px)) * 8);
#pragma unroll
        for (int e = 0; e < 4; ++e) dbv[e] += (f32x2){__uint_as_float(w[e] << 16), __uint_as_float(w[e] & 0xFFFF0000u)};
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll 1
    for (int ks = 0; ks < DTH * DTW / 32; ++ks) {
      // k-step ks: tile pixels 32 ks .. 32 ks + 31 = rows 2 ks, 2 ks + 1 (lane groups g = 0, 1 / 2, 3)
      bf16x8 af[4];
      const int pxa = ks * 32 + 16 * (g >> 1) + pcol;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int uo = (32 * ct) ^ sw16;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + pxa * 128 + uo));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + (pxa + 8) * 128 + uo));
        af[ct] = cat_bf16x4(lo, hi);
      }
      const int hrow = 2 * ks + (g >> 1);  // X octants 2 wv + (p4 >> 1): the wave's pair plane
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t - ky * 3;
        const int hp = (hrow + ky) * DHW + pcol + kx;
        const char* base = Xs + (wv * DPL + 2 * hp + (p4 >> 1)) * 16 + (p4 & 1) * 8;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base + 16 * 16));
        const bf16x8 bfr = cat_bf16x4(lo, hi);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
          acc[t][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ct], bfr, acc[t][ct], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
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
        if (co < a.cout && ci < a.cin) {
          EUNET_DASSERT(split < a.nsplit);
          out[((long long)co * 9 + t) * a.cin + ci] = acc[t][ct][e];
        }
      }
  if (a.db != nullptr && kc == 0) {
    float* dbred = (float*)wst;  // [32 pixel groups][64 co]
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) dbred[(tid >> 3) * 64 + (tid & 7) * 8 + e] = dbv[e >> 1][e & 1];
    __syncthreads();
    if (tid < 64 && co0 + tid < a.cout) {
      float t = 0.f;
      for (int r = 0; r < 32; ++r) t += dbred[r * 64 + tid];
      a.db[(long long)split * a.cout + co0 + tid] = t;
    }
  }
}

// fp32 wgrad (exact fp32: v_mfma_f32_16x16x4_f32, 64 FLOP/clk/SIMD).  Pixels are the GEMM K.
// Block = (pixel split, 64 co, 32 ci) over 4 x 32 pixel tiles; wave w owns ci tile w & 1 and
// co tiles 2 (w >> 1) .. +1 for all 9 taps (18 accumulators).  One k-step = 4 pixels: 2 A
// (dY^T) + 9 B (X) single-dword LDS reads feed 18 MFMAs (576 clk), so the loop is MFMA-bound.
// LDS images are channel-tile-major ([tile][pixel][16 ch] floats): the 4 pixel rows a fragment
// read touches fall in 4 distinct 16-bank groups (conflict-free).  58 KB per block, two blocks
// per CU; the next tile is loaded into registers while the current one is computed
// (one LDS stage, register double buffer).
constexpr int WF_TH = 4, WF_TW = 32;                 // pixel tile
constexpr int WF_HW = WF_TW + 2;                     // 34
constexpr int WF_HP = (WF_TH + 2) * WF_HW;           // 204 halo pixels
constexpr int WF_CI = 32, WF_CO = 64;                // channels per block
constexpr int WF_XU = WF_HP * WF_CI / 4;             // 1632 16-B halo units
constexpr int WF_DU = WF_TH * WF_TW * WF_CO / 4;     // 2048 16-B dY units
constexpr int WF_XI = (WF_XU + NTHR - 1) / NTHR;     // 7
constexpr int WF_DI = WF_DU / NTHR;                  // 8
constexpr int WF_XS = (WF_CI / 16) * WF_HP * 16;     // floats of the X image
constexpr int WF_LDS = (WF_XS + (WF_CO / 16) * WF_TH * WF_TW * 16 + 4 * 64) * 4;  // 59 392 B
static_assert(2 * WF_LDS <= 160 * 1024, "fp32 wgrad: two blocks per CU");

__global__ __launch_bounds__(NTHR, 2) void conv3x3_wgrad_f32_kernel(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Xs = (float*)smem;               // [2 ci tiles][204 px][16]
  float* Ds = Xs + WF_XS;                 // [4 co tiles][128 px][16]
  float* dbs = Ds + (WF_CO / 16) * WF_TH * WF_TW * 16;  // [4][64]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int split, cob, cib;
  wg_map(blockIdx.x, a.nsplit, cdiv(a.cout, WF_CO), cdiv(a.cin, WF_CI), split, cob, cib);
  const int co0 = cob * WF_CO, ci0 = cib * WF_CI;
  const int t_begin = split * a.per_split;
  const int t_end = min(a.ntiles, t_begin + a.per_split);
  const int tpi = a.tx * a.ty;
  const int kq = lane >> 4, li = lane & 15;
  const int ct0 = 2 * (wv >> 1), cit = wv & 1;
  const bool do_db = a.db != nullptr && cib == 0;

  f32x4 acc[2][9];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;  // co = co0 + (tid & 63), pixels (tid >> 6) + 4 i

  uint4 rx[WF_XI], rd[WF_DI];
  unsigned rok = 0;  // bit i: halo unit i is inside the image (BN+ReLU applies; padding stays 0)
  auto gload = [&](int tile) {
    const int n = tile / tpi, trem = tile - n * tpi;
    const int y0 = (trem / a.tx) * WF_TH, x0 = (trem % a.tx) * WF_TW;
    rok = 0;
#pragma unroll
    for (int i = 0; i < WF_XI; ++i) {
      const int u = tid + i * NTHR;  // unit = (ci tile, halo pixel, quad m)
      const int m = u & 3, hp = (u >> 2) % WF_HP, tl = (u >> 2) / WF_HP;
      const int hy = hp / WF_HW, hx = hp - hy * WF_HW;
      const int yy = y0 + hy - 1, xx = x0 + hx - 1, c = ci0 + tl * 16 + 4 * m;
      rx[i] = make_uint4(0, 0, 0, 0);
      if (u < WF_XU && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W && c < a.cin) {
        rx[i] = *(const uint4*)((const float*)a.x + ((long long)(n * a.H + yy) * a.W + xx) * a.xct + a.xco + c);
        rok |= 1u << i;
      }
    }
#pragma unroll
    for (int i = 0; i < WF_DI; ++i) {
      const int u = tid + i * NTHR;  // unit = (co tile, pixel, quad m)
      const int m = u & 3, px = (u >> 2) % (WF_TH * WF_TW), tl = (u >> 2) / (WF_TH * WF_TW);
      const int yy = y0 + px / WF_TW, xx = x0 + px % WF_TW, co = co0 + tl * 16 + 4 * m;
      rd[i] = make_uint4(0, 0, 0, 0);
      if (yy < a.H && xx < a.W && co < a.cout)
        rd[i] = *(const uint4*)((const float*)a.dy + ((long long)(n * a.H + yy) * a.W + xx) * a.dct + a.dco + co);
    }
  };
  auto lwrite = [&](int tile) {
    const int n = tile / tpi;
#pragma unroll
    for (int i = 0; i < WF_XI; ++i) {
      const int u = tid + i * NTHR;
      if (u >= WF_XU) continue;
      uint4 v = rx[i];
      if (a.isc != nullptr && ((rok >> i) & 1u)) {
        const int m = u & 3, tl = (u >> 2) / WF_HP, c = ci0 + tl * 16 + 4 * m + n * a.iss;
        float f[4];
        Vec16<float>::unpack(v, f);
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = fmaxf(fmaf(f[e], a.isc[c + e], a.ish[c + e]), 0.f);
        v = Vec16<float>::pack(f);
      }
      *(uint4*)(Xs + 4 * u) = v;  // unit order == [tile][pixel][16] layout
    }
#pragma unroll
    for (int i = 0; i < WF_DI; ++i) *(uint4*)(Ds + 4 * (tid + i * NTHR)) = rd[i];
  };

  if (t_begin < t_end) gload(t_begin);
  for (int tile = t_begin; tile < t_end; ++tile) {
    __syncthreads();  // the previous tile's fragment reads are done
    lwrite(tile);
    __syncthreads();
    if (tile + 1 < t_end) gload(tile + 1);  // in flight during this tile's MFMAs
    if (do_db) {
#pragma unroll 4
      for (int i = 0; i < WF_TH * WF_TW / 4; ++i) {
        const int px = (tid >> 6) + 4 * i, co = tid & 63;
        dbacc += Ds[((co >> 4) * WF_TH * WF_TW + px) * 16 + (co & 15)];
      }
    }
    const float* xb = Xs + cit * WF_HP * 16 + li;
    const float* d0 = Ds + (ct0 * WF_TH * WF_TW) * 16 + li;
    const float* d1 = d0 + WF_TH * WF_TW * 16;
#pragma unroll 2
    for (int ks = 0; ks < WF_TH * WF_TW / 4; ++ks) {
      const int px = 4 * ks + kq, r = px / WF_TW, c = px - r * WF_TW;
      const float a0 = d0[px * 16], a1 = d1[px * 16];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ky = t / 3, kx = t - 3 * ky;
        const float bv = xb[((r + ky) * WF_HW + c + kx) * 16];
        acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bv, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, bv, acc[1][t], 0, 0, 0);
      }
    }
  }
  // D[m = co][n = ci]: lane holds co = tile base + 4 kq + i, ci = tile base + li
  float* out = a.dw + (long long)split * a.cout * 9 * a.cin;
  const int ci = ci0 + cit * 16 + li;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = co0 + (ct0 + j) * 16 + 4 * kq + i;
        if (co < a.cout && ci < a.cin) out[((long long)co * 9 + t) * a.cin + ci] = acc[j][t][i];
      }
  if (do_db) {
    dbs[wv * 64 + lane] = dbacc;
    __syncthreads();
    if (tid < 64 && co0 + tid < a.cout)
      a.db[(long long)split * a.cout + co0 + tid] = dbs[tid] + dbs[64 + tid] + dbs[128 + tid] + dbs[192 + tid];
  }
}

// Deterministic split reduction: a block reduces 64 consecutive elements; thread (sg, tq) sums
// splits sg, sg + 16, ... of elements 4tq..4tq+3 (16-byte loads, 8 in flight, fp64), then the 16
// split groups are added in a fixed pairwise order.  Blocks past the dW range reduce the bias
// partials.
constexpr int RSG = 16;
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* part, const float* dbp, int nsplit, int cout,
                                                           int cin, int taps, float* dw, float* db) {
  __shared__ double red[RSG][64];
  const int tq = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const long long per = (long long)cout * taps * cin;
  const long long nbw = (per + 63) / 64;
  const bool isdw = blockIdx.x < nbw;
  const long long e0 = (isdw ? (long long)blockIdx.x : (long long)blockIdx.x - nbw) * 64 + 4 * tq;
  const long long cnt = isdw ? per : cout;
  const float* src = isdw ? part : dbp;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  if (cnt % 4 == 0 && e0 < cnt) {
#pragma unroll 8
    for (int k = sg; k < nsplit; k += RSG) {
      const float4 v = *(const float4*)(src + (long long)k * cnt + e0);
      s[0] += (double)v.x;
      s[1] += (double)v.y;
      s[2] += (double)v.z;
      s[3] += (double)v.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (e0 + i < cnt)
        for (int k = sg; k < nsplit; k += RSG) s[i] += (double)src[(long long)k * cnt + e0 + i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[sg][4 * tq + i] = s[i];
  __syncthreads();
  const int tx = threadIdx.x;
  const long long e = e0 - 4 * tq + tx;
  if (tx >= 64 || e >= cnt) return;
  double t[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) t[g] = red[2 * g][tx] + red[2 * g + 1][tx];
  const double u = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
  if (isdw) {
    const int ci = (int)(e % cin);
    const long long r = e / cin;
    const int tp = (int)(r % taps);
    const int co = (int)(r / taps);
    dw[((long long)co * cin + ci) * taps + tp] = (float)u;
  } else {
    db[e] = (float)u;
  }
}

bool act_ok(const eunet_act* a) {
  return a && a->ptr && a->n > 0 && a->h > 0 && a->w > 0 && a->c > 0 && a->coff >= 0 &&
         a->coff + a->c <= a->ctot && (a->dtype == EUNET_F32 || a->dtype == EUNET_BF16);
}

int elems16(int dtype) { return dtype == EUNET_BF16 ? 8 : 4; }
int kchunk(int dtype) { return 4 * elems16(dtype); }

template <bool DG>
int launch_fwd(const FwdArgs& a, int dtype, void* stream, bool out_f32 = false, bool bt = false) {
  const long long esz = dtype == EUNET_BF16 ? 2 : 4;
  EUNET_REQUIRE((long long)a.H * a.W * a.xct * esz < (long long)FWD_OOB,
                "conv3x3: one sample's input (%d x %d x %d) must be < 3 GiB (buffer-descriptor staging)", a.H, a.W, a.xct);
  EUNET_REQUIRE((long long)a.nkc * kchunk(dtype) * a.cout_pad * 9 * esz < (1ll << 31), "conv3x3: packed weights >= 2 GiB");
  dim3 grid(a.ntiles * (a.cout_pad / BN));
  const bool bnb = DG && a.bpart != nullptr;
  EUNET_REQUIRE(!(out_f32 && bnb), "conv3x3: an fp32-output data gradient has no fused BN-backward reduction");
  auto go = [&](auto kern) {
    allow_lds(kern, FWD_LDS);
    kern<<<grid, FT, FWD_LDS, (hipStream_t)stream>>>(a);
  };
  if (dtype == EUNET_BF16 && out_f32) {
    go(conv3x3_fwd_kernel<bf16_t, true, float>);
  } else if (dtype == EUNET_BF16 && DG && bt) {
    if (bnb) go(conv3x3_fwd_kernel<bf16_t, true, bf16_t, true, true>);
    else go(conv3x3_fwd_kernel<bf16_t, true, bf16_t, true, false>);
  } else if (dtype == EUNET_BF16) {
    const int tail = a.cout % BN;
    if (tail > 0 && tail <= BN / 2) {  // a half-empty tail co-block: the CT instantiations
      if (bnb) go(conv3x3_fwd_kernel<bf16_t, true, bf16_t, false, true, false, true>);
      else if (!DG && a.isc == nullptr) go(conv3x3_fwd_kernel<bf16_t, false, bf16_t, false, false, true, true>);
      else go(conv3x3_fwd_kernel<bf16_t, DG, bf16_t, false, false, false, true>);
    } else if (bnb) {
      go(conv3x3_fwd_kernel<bf16_t, true, bf16_t, false, true>);
    } else if (!DG && a.isc == nullptr) {
      go(conv3x3_fwd_kernel<bf16_t, false, bf16_t, false, false, true>);
    } else {
      go(conv3x3_fwd_kernel<bf16_t, DG>);
    }
  } else {
    if (bnb) go(conv3x3_fwd_kernel<float, true, float, false, true>);
    else go(conv3x3_fwd_kernel<float, DG>);
  }
  EUNET_LAUNCH_CHECK("conv3x3_fwd");
  return EUNET_OK;
}

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

int eunet_conv3x3_pack_many(const eunet_pack_desc* descs, int n, int dtype, void* stream) {
  EUNET_REQUIRE(descs && n > 0 && n <= EUNET_PACK_MAX, "conv3x3_pack_many: 1..%d tensors", EUNET_PACK_MAX);
  PackBatch b;
  const int E = dtype == EUNET_BF16 ? 8 : 4;
  long long blocks = 0;
  for (int i = 0; i < n; ++i) {
    const eunet_pack_desc& d = descs[i];
    EUNET_REQUIRE(d.w && d.wp && d.cout > 0 && d.cin > 0, "conv3x3_pack_many: bad descriptor %d", i);
    EUNET_REQUIRE(((uintptr_t)d.wp & 15) == 0, "conv3x3_pack_many: packed operand %d not 16-byte aligned", i);
    b.d[i] = d;
    const int go = d.flip ? d.cin : d.cout, gi = d.flip ? d.cout : d.cin;
    b.cout_p[i] = cdiv(go, BN) * BN;
    b.cin_p[i] = cdiv(gi, kchunk(dtype)) * kchunk(dtype);  // a multiple of 4 E
    b.bstart[i] = (int)blocks;
    blocks += ((long long)b.cout_p[i] * b.cin_p[i] * 9 / E + 255) / 256;
  }
  EUNET_REQUIRE(blocks < (1ll << 31), "conv3x3_pack_many: too large");
  b.bstart[n] = (int)blocks;
  b.n = n;
  if (dtype == EUNET_BF16) pack_many_kernel<bf16_t><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(b);
  else pack_many_kernel<float><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(b);
  EUNET_LAUNCH_CHECK("conv3x3_pack_many");
  return EUNET_OK;
}

int eunet_conv3x3_tiles(const eunet_act* y, int* tiles) {
  EUNET_REQUIRE(act_ok(y) && tiles, "conv3x3_tiles: bad args");
  *tiles = y->n * cdiv(y->h, FTH) * cdiv(y->w, FTW);
  return EUNET_OK;
}

int eunet_conv3x3_fwd(const eunet_act* x, const float* in_scale, const float* in_shift, int in_nstride,
                      const void* wp, const float* bias, const eunet_act* y, float* stats, void* stream) {
  EUNET_REQUIRE(act_ok(x) && act_ok(y) && wp, "conv3x3_fwd: bad tensors");
  EUNET_REQUIRE(x->dtype == y->dtype, "conv3x3_fwd: dtype mismatch");
  EUNET_REQUIRE(x->n == y->n && x->h == y->h && x->w == y->w, "conv3x3_fwd: spatial mismatch");
  const int E = elems16(x->dtype);
  EUNET_REQUIRE(x->c % E == 0 && x->ctot % E == 0 && x->coff % E == 0,
                "conv3x3_fwd: input channels/stride/offset must be multiples of %d", E);
  EUNET_REQUIRE((in_scale == nullptr) == (in_shift == nullptr), "conv3x3_fwd: scale/shift pair");
  FwdArgs a;
  a.x = x->ptr; a.N = x->n; a.H = x->h; a.W = x->w; a.xct = x->ctot; a.xco = x->coff; a.cin = x->c;
  EUNET_REQUIRE(in_nstride == 0 || (in_scale && in_nstride >= x->c), "conv3x3_fwd: in_nstride");
  a.isc = in_scale; a.ish = in_shift; a.iss = in_nstride;
  a.wp = wp; a.cout_pad = cdiv(y->c, BN) * BN; a.nkc = cdiv(x->c, kchunk(x->dtype));
  a.bias = bias;
  a.y = y->ptr; a.yct = y->ctot; a.yco = y->coff; a.cout = y->c;
  a.stats = stats; a.tx = cdiv(x->w, FTW); a.ty = cdiv(x->h, FTH); a.ntiles = x->n * a.tx * a.ty;
  a.by = nullptr; a.byct = 0; a.byco = 0;
  a.bmean = a.bistd = a.bsc = a.bsh = nullptr; a.bpart = nullptr; a.gsc = nullptr;
  a.tyin = nullptr; a.tcoef = nullptr; a.tgo = nullptr;
  a.pro1 = 1;
  EUNET_REQUIRE(y->c % E == 0 && y->ctot % E == 0 && y->coff % E == 0,
                "conv3x3_fwd: output channels/stride/offset must be multiples of %d", E);
  return launch_fwd<false>(a, x->dtype, stream);
}

int eunet_conv3x3_dgrad(const eunet_act* dy, const void* wp_t, const eunet_act* gx, const float* gscale,
                        void* stream) {
  EUNET_REQUIRE(act_ok(dy) && act_ok(gx) && wp_t, "conv3x3_dgrad: bad args");
  // gx is dy's dtype, or fp32 for a bf16 dy (the output rounded to fp32 instead of bf16)
  const bool out_f32 = dy->dtype == EUNET_BF16 && gx->dtype == EUNET_F32;
  EUNET_REQUIRE(dy->dtype == gx->dtype || out_f32, "conv3x3_dgrad: dtype mismatch");
  EUNET_REQUIRE(dy->n == gx->n && dy->h == gx->h && dy->w == gx->w, "conv3x3_dgrad: spatial mismatch");
  const int E = elems16(dy->dtype);
  EUNET_REQUIRE(dy->c % E == 0 && dy->ctot % E == 0 && dy->coff % E == 0 && gx->c % E == 0 && gx->ctot % E == 0 &&
                    gx->coff % E == 0,
                "conv3x3_dgrad: channels/strides must be multiples of %d", E);
  FwdArgs a;
  a.x = dy->ptr; a.N = dy->n; a.H = dy->h; a.W = dy->w; a.xct = dy->ctot; a.xco = dy->coff; a.cin = dy->c;
  a.isc = nullptr; a.ish = nullptr; a.iss = 0;
  a.wp = wp_t; a.cout_pad = cdiv(gx->c, BN) * BN; a.nkc = cdiv(dy->c, kchunk(dy->dtype));
  a.bias = nullptr;
  a.y = gx->ptr; a.yct = gx->ctot; a.yco = gx->coff; a.cout = gx->c;
  a.stats = nullptr; a.tx = cdiv(dy->w, FTW); a.ty = cdiv(dy->h, FTH); a.ntiles = dy->n * a.tx * a.ty;
  a.by = nullptr; a.byct = 0; a.byco = 0;
  a.bmean = a.bistd = a.bsc = a.bsh = nullptr; a.bpart = nullptr; a.gsc = gscale;
  a.tyin = nullptr; a.tcoef = nullptr; a.tgo = nullptr;
  a.pro1 = 1;
  return launch_fwd<true>(a, dy->dtype, stream, out_f32);
}

int eunet_conv3x3_dgrad_bnbwd(const eunet_act* dy, const void* wp_t, const eunet_act* gx, const eunet_act* y,
                              const float* mean, const float* invstd, const float* scale, const float* shift,
                              const float* gscale, float* part, void* stream) {
  EUNET_REQUIRE(act_ok(dy) && act_ok(gx) && act_ok(y) && wp_t && mean && invstd && scale && shift && part,
                "conv3x3_dgrad_bnbwd: bad args");
  EUNET_REQUIRE(dy->dtype == gx->dtype && y->dtype == gx->dtype, "conv3x3_dgrad_bnbwd: dtype mismatch");
  EUNET_REQUIRE(dy->n == gx->n && dy->h == gx->h && dy->w == gx->w && y->n == gx->n && y->h == gx->h &&
                    y->w == gx->w && y->c == gx->c,
                "conv3x3_dgrad_bnbwd: shape mismatch");
  const int E = elems16(dy->dtype);
  EUNET_REQUIRE(dy->c % E == 0 && dy->ctot % E == 0 && dy->coff % E == 0 && gx->c % E == 0 && gx->ctot % E == 0 &&
                    gx->coff % E == 0 && y->ctot % E == 0 && y->coff % E == 0,
                "conv3x3_dgrad_bnbwd: channels/strides must be multiples of %d", E);
  FwdArgs a;
  a.x = dy->ptr; a.N = dy->n; a.H = dy->h; a.W = dy->w; a.xct = dy->ctot; a.xco = dy->coff; a.cin = dy->c;
  a.isc = nullptr; a.ish = nullptr; a.iss = 0;
  a.wp = wp_t; a.cout_pad = cdiv(gx->c, BN) * BN; a.nkc = cdiv(dy->c, kchunk(dy->dtype));
  a.bias = nullptr;
  a.y = gx->ptr; a.yct = gx->ctot; a.yco = gx->coff; a.cout = gx->c;
  a.stats = nullptr; a.tx = cdiv(dy->w, FTW); a.ty = cdiv(dy->h, FTH); a.ntiles = dy->n * a.tx * a.ty;
  a.by = y->ptr; a.byct = y->ctot; a.byco = y->coff;
  a.bmean = mean; a.bistd = invstd; a.bsc = scale; a.bsh = shift; a.bpart = part; a.gsc = gscale;
  a.tyin = nullptr; a.tcoef = nullptr; a.tgo = nullptr;
  a.pro1 = 1;
  return launch_fwd<true>(a, dy->dtype, stream);
}

int eunet_conv3x3_dgrad_fused(const eunet_act* g, const eunet_act* y_in, const float* coef, const eunet_act* gy_out,
                              const void* wp_t, const eunet_act* gx, const eunet_act* y_next, const float* mean,
                              const float* invstd, const float* scale, const float* shift, float* part,
                              const float* gscale, void* stream) {
  EUNET_REQUIRE(act_ok(g) && act_ok(y_in) && coef && act_ok(gx) && wp_t, "conv3x3_dgrad_fused: bad args");
  EUNET_REQUIRE(g->dtype == gx->dtype && y_in->dtype == g->dtype, "conv3x3_dgrad_fused: dtype mismatch");
  EUNET_REQUIRE(g->n == gx->n && g->h == gx->h && g->w == gx->w, "conv3x3_dgrad_fused: spatial mismatch");
  // y_in (and gy_out) are addressed with g's unit offsets: the same shape and channel layout
  EUNET_REQUIRE(y_in->n == g->n && y_in->h == g->h && y_in->w == g->w && y_in->c == g->c && y_in->ctot == g->ctot &&
                    y_in->coff == g->coff,
                "conv3x3_dgrad_fused: y_in must have g's shape and channel layout");
  if (gy_out)
    EUNET_REQUIRE(act_ok(gy_out) && gy_out->dtype == g->dtype && gy_out->n == g->n && gy_out->h == g->h &&
                      gy_out->w == g->w && gy_out->c == g->c && gy_out->ctot == g->ctot && gy_out->coff == g->coff,
                  "conv3x3_dgrad_fused: gy_out must have g's shape and channel layout");
  const bool red = y_next != nullptr;
  EUNET_REQUIRE(red == (part != nullptr) && (!red || (act_ok(y_next) && mean && invstd && scale && shift)),
                "conv3x3_dgrad_fused: the next-BN reduction needs y_next, mean, invstd, scale, shift and part");
  if (red)
    EUNET_REQUIRE(y_next->dtype == gx->dtype && y_next->n == gx->n && y_next->h == gx->h && y_next->w == gx->w &&
                      y_next->c == gx->c,
                  "conv3x3_dgrad_fused: y_next shape mismatch");
  const int E = elems16(g->dtype);
  EUNET_REQUIRE(g->c % E == 0 && g->ctot % E == 0 && g->coff % E == 0 && gx->c % E == 0 && gx->ctot % E == 0 &&
                    gx->coff % E == 0 && (!red || (y_next->ctot % E == 0 && y_next->coff % E == 0)),
                "conv3x3_dgrad_fused: channels/strides must be multiples of %d", E);
  FwdArgs a;
  a.x = g->ptr; a.N = g->n; a.H = g->h; a.W = g->w; a.xct = g->ctot; a.xco = g->coff; a.cin = g->c;
  a.isc = nullptr; a.ish = nullptr; a.iss = 0;
  a.wp = wp_t; a.cout_pad = cdiv(gx->c, BN) * BN; a.nkc = cdiv(g->c, kchunk(g->dtype));
  a.bias = nullptr;
  a.y = gx->ptr; a.yct = gx->ctot; a.yco = gx->coff; a.cout = gx->c;
  a.stats = nullptr; a.tx = cdiv(g->w, FTW); a.ty = cdiv(g->h, FTH); a.ntiles = g->n * a.tx * a.ty;
  a.by = red ? y_next->ptr : nullptr; a.byct = red ? y_next->ctot : 0; a.byco = red ? y_next->coff : 0;
  a.bmean = mean; a.bistd = invstd; a.bsc = scale; a.bsh = shift; a.bpart = part; a.gsc = gscale;
  a.tyin = y_in->ptr; a.tcoef = coef; a.tgo = gy_out ? gy_out->ptr : nullptr;
  a.pro1 = 1;
  if (g->dtype != EUNET_BF16) {
    // fp32: the transform runs as its own pass into gy_out (the fp32 staging has no registers for
    // it), then the plain data gradient reads gy_out -- the same values
    EUNET_REQUIRE(gy_out, "conv3x3_dgrad_fused: fp32 needs gy_out (the transform is materialised)");
    const int rc = eunet_bn_bwd_apply_coef(g, y_in, coef, gy_out, stream);
    if (rc != EUNET_OK) return rc;
    a.x = gy_out->ptr; a.tyin = nullptr; a.tcoef = nullptr; a.tgo = nullptr;
  }
  return launch_fwd<true>(a, g->dtype, stream, false, a.tcoef != nullptr);
}


// weight-gradient blocks per launch: two resident per CU (1024 / 2048 measured equal / slower in
// the bench, where the wgrad shares the chip with the data-gradient stream: profiles/r02_ab_conv.txt)
constexpr int WG_BLOCKS = 512;  // weight-gradient blocks per launch (two per CU)
int eunet_conv3x3_wgrad_splits(const eunet_act* dy, int cin, int dtype, int* nsplit) {
  EUNET_REQUIRE(act_ok(dy) && nsplit && cin > 0, "conv3x3_wgrad_splits: bad args");
  const bool bf = dtype == EUNET_BF16;
  const int ntiles = dy->n * cdiv(dy->h, bf ? DTH : WF_TH) * cdiv(dy->w, bf ? DTW : WF_TW);
  const int blocks = cdiv(dy->c, 64) * cdiv(cin, bf ? KCW : WF_CI);
  int s = cdiv(WG_BLOCKS, blocks);
  {
    // fewest launch waves per unit of work: a split count whose blocks leave a nearly empty last wave
    // (the decoder's concat inputs: 48 / 12 / 3 block columns -> 528 / 516 / 513 blocks) runs that
    // wave's tail alone; pick s in [s0/2, 2 s0] minimising waves / s (ties: fewer splits)
    const int s0 = s;
    long long bw = 1, bs = 0;  // best waves / best s as the fraction bw / bs
    for (int c = (s0 + 1) / 2; c <= 2 * s0; ++c) {
      const long long w = cdiv(c * blocks, WG_BLOCKS);
      if (c >= 1 && (bs == 0 || w * bs < bw * c)) bw = w, bs = c;
    }
    s = (int)bs;
  }
  s = s < 1 ? 1 : s;
  s = s > ntiles ? ntiles : s;
  // keep partials <= 256 MiB
  const long long per = (long long)dy->c * 9 * cin * 4;
  while (s > 1 && per * s > (256ll << 20)) --s;
  const int per_split = cdiv(ntiles, s);
  *nsplit = cdiv(ntiles, per_split);
  return EUNET_OK;
}

#if CONV_STAMP
int eunet_conv_stamps(void* out, size_t bytes) {  // diagnostic builds only (tools/conv_stamps.py)
  EUNET_REQUIRE(out && bytes <= sizeof(g_conv_stamps), "conv_stamps: bad args");
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_conv_stamps), bytes, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return EUNET_ERR_HIP;
  return EUNET_OK;
}
#endif

int eunet_conv3x3_wgrad(const eunet_act* x, const float* in_scale, const float* in_shift, int in_nstride,
                        const eunet_act* dy, float* dw_part, float* db_part, int nsplit, void* stream) {
  EUNET_REQUIRE(act_ok(x) && act_ok(dy) && dw_part && nsplit > 0, "conv3x3_wgrad: bad args");
  EUNET_REQUIRE(x->dtype == dy->dtype, "conv3x3_wgrad: dtype mismatch");
  EUNET_REQUIRE(x->n == dy->n && x->h == dy->h && x->w == dy->w, "conv3x3_wgrad: spatial mismatch");
  const int E = elems16(x->dtype);
  EUNET_REQUIRE(x->c % E == 0 && x->ctot % E == 0 && x->coff % E == 0 && dy->c % E == 0 &&
                    dy->ctot % E == 0 && dy->coff % E == 0,
                "conv3x3_wgrad: channels/strides must be multiples of %d", E);
  WgArgs a;
  a.x = x->ptr; a.N = x->n; a.H = x->h; a.W = x->w; a.xct = x->ctot; a.xco = x->coff; a.cin = x->c;
  EUNET_REQUIRE(in_nstride == 0 || (in_scale && in_nstride >= x->c), "conv3x3_wgrad: in_nstride");
  a.isc = in_scale; a.ish = in_shift; a.iss = in_nstride;
  a.dy = dy->ptr; a.dct = dy->ctot; a.dco = dy->coff; a.cout = dy->c;
  a.dw = dw_part; a.db = db_part;
  const bool bf = x->dtype == EUNET_BF16;
  EUNET_REQUIRE(!bf || ((long long)a.H * a.W * a.xct * 2 < (long long)FWD_OOB &&
                        (long long)a.H * a.W * a.dct * 2 < (long long)FWD_OOB),
                "conv3x3_wgrad: sample slice >= 3 GiB");
  a.tx = cdiv(x->w, bf ? DTW : WF_TW); a.ty = cdiv(x->h, bf ? DTH : WF_TH); a.ntiles = x->n * a.tx * a.ty;
  a.per_split = cdiv(a.ntiles, nsplit);
  a.nsplit = nsplit;
  EUNET_REQUIRE(cdiv(a.ntiles, a.per_split) == nsplit, "conv3x3_wgrad: nsplit not from wgrad_splits");
  if (x->dtype == EUNET_BF16) {
    dim3 grid(nsplit * cdiv(dy->c, 64) * cdiv(x->c, KCW));
    conv3x3_wgrad_bf16_kernel<<<grid, NTHR, 0, (hipStream_t)stream>>>(a);
  } else {
    dim3 grid(nsplit * cdiv(dy->c, WF_CO) * cdiv(x->c, WF_CI));
    allow_lds(conv3x3_wgrad_f32_kernel, WF_LDS);
    conv3x3_wgrad_f32_kernel<<<grid, NTHR, WF_LDS, (hipStream_t)stream>>>(a);
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
  const unsigned nb = (unsigned)((per + 63) / 64 + (db != nullptr ? (cout + 63) / 64 : 0));
  wgrad_reduce_kernel<<<nb, 256, 0, (hipStream_t)stream>>>(dw_part, db_part, nsplit, cout, cin, taps, dw, db);
  EUNET_LAUNCH_CHECK("wgrad_reduce");
  return EUNET_OK;
}

}  // extern "C"
