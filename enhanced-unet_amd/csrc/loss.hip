// Combined segmentation loss, fused and batched (one launch for all samples).
//
// Reference: FocalLoss (train_eval.py:28-60; the Trainer builds it with alpha [1,8,5],
// gamma 5, CE class weights [1,20,10] at :74-79), Trainer.dice_loss (:134-157, weights
// [1,15,8]), Trainer.tversky_loss (:159-181, weights [1,12,6], alpha 0.7),
// _compute_combined_loss (:183-197; 2.5/2.5/1.0 at :82-85) and the per-sample loop + /B
// of Trainer.train_epoch (:262-337).
//   focal_n = mean_px alpha_t (1-pt)^gamma ce,  ce = -w_t log p_t,  pt = exp(-ce)
//   dice_n  = (1/D) sum_c wd_c (1 - (2 I_c + 1e-6)/(S_c + T_c + 1e-6))
//   tv_n    = (1/D) sum_c wt_c (1 - (I_c + 1e-6)/(I_c + a fp_c + (1-a) fn_c + 1e-6))
// with I = sum p t, S = sum p, T = sum t per (sample, class) and D the num_classes the
// reference divides by (3 in _compute_combined_loss for any K, :192-193; for K=2 this is
// exactly its K=3 loss with a third logit at -inf, pinned by tests/golden).
//   loss = w_focal * (sum_n sum_px focal) / F_den + (1/N) sum_n (w_dice dice_n + w_tv tv_n)
// F_den = N*H*W (the pixel mean of FocalLoss, and of the per-sample loop's mean over
// samples), or sum of w_t (nn.CrossEntropyLoss's weighted mean, focal_norm = 1).
// Pixels whose target is ignore_index contribute ce = 0 (F.cross_entropy ignore_index).
// Targets outside [0, K) that are not ignore_index are an error in the reference
// (F.cross_entropy raises / device-asserts): they are counted into sums[N*NV + 1] for the
// host to report at its next synchronisation, and contribute nothing here.
// Backward is analytic per pixel from the saved per-(sample,class) sums.
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr int LPIX = 1024;  // pixels per partial tile

// the Trainer's enhanced_unet configuration (train_eval.py:74-87, 140, 164, 175)
const eunet_loss_params kReferenceParams = {
    {1.f, 20.f, 10.f}, {1.f, 8.f, 5.f}, 5.f, EUNET_NO_IGNORE, {1.f, 15.f, 8.f}, {1.f, 12.f, 6.f}, 0.7f, 2.5f, 2.5f, 1.f, 3.f, 0};

constexpr float EPS = 1e-6f;

template <int K>
__device__ __forceinline__ void softmax_px(const float* lg, long long plane, float (&p)[K], float& lse_m, float& m) {
  float l[K];
#pragma unroll
  for (int k = 0; k < K; ++k) l[k] = lg[k * plane];
  m = l[0];
#pragma unroll
  for (int k = 1; k < K; ++k) m = fmaxf(m, l[k]);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    p[k] = expf(l[k] - m);
    s += p[k];
  }
  const float inv = 1.f / s;
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] *= inv;
  lse_m = logf(s);  // log sum exp(l - m)
}

// (1-pt)^gamma and (1-pt)^(gamma-1); gamma 5 (the reference's) in the product form the
// fixtures were pinned with, small integers by repeated products, otherwise powf
__device__ __forceinline__ void focal_pow(float om, float gamma, float& pg, float& pg1) {
  if (gamma == 5.f) {
    const float om2 = om * om, om4 = om2 * om2;
    pg = om4 * om;
    pg1 = om4;
    return;
  }
  const int gi = (int)gamma;
  if ((float)gi == gamma && gi >= 0 && gi <= 8) {
    float r = 1.f;
    for (int i = 1; i < gi; ++i) r *= om;
    pg1 = gi >= 1 ? r : 0.f;
    pg = gi >= 1 ? r * om : 1.f;
    return;
  }
  pg = powf(om, gamma);
  pg1 = powf(om, gamma - 1.f);
}

template <int K>
__global__ __launch_bounds__(NT) void loss_fwd_kernel(const float* logits, const int64_t* target, int HW,
                                                      eunet_loss_params prm, float* part) {
  constexpr int NV = 3 + 3 * K;  // focal sum, I/S/T per class, ce-weight sum, bad-target count
  __shared__ float red[4][NV];
  const int n = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long long plane = HW;
  const float* lg = logits + (long long)n * K * HW;
  const int64_t* tg = target + (long long)n * HW;
  float acc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) acc[i] = 0.f;
  const int p0 = blockIdx.x * LPIX;
  const int p1 = min(HW, p0 + LPIX);
  for (int p = p0 + tid; p < p1; p += NT) {
    float pr[K], lse_m, m;
    softmax_px<K>(lg + p, plane, pr, lse_m, m);
    const int64_t traw = tg[p];
    const bool ign = traw == (int64_t)prm.ignore_index;
    const bool valid = !ign && traw >= 0 && traw < K;
    const int t = valid ? (int)traw : 0;
    if (valid) {
      const float logpt = lg[t * plane + p] - m - lse_m;
      const float ce = -prm.ce_weight[t] * logpt;
      const float pt = expf(-ce);
      float pg, pg1;
      focal_pow(1.f - pt, prm.gamma, pg, pg1);
      acc[0] += prm.alpha[t] * pg * ce;
      acc[1 + 3 * K] += prm.ce_weight[t];
    } else if (!ign) {
      acc[2 + 3 * K] += 1.f;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float tk = (traw == (int64_t)k) ? 1.f : 0.f;
      acc[1 + k] += pr[k] * tk;
      acc[1 + K + k] += pr[k];
      acc[1 + 2 * K + k] += tk;
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float s = wave_sum(acc[i]);
    if (lane == 0) red[wv][i] = s;
  }
  __syncthreads();
  if (tid < NV)
    part[((long long)n * gridDim.x + blockIdx.x) * NV + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
}

// One 256-thread block: per sample, the threads stride over the tile partials (fp64),
// a fixed-order LDS tree combines them (deterministic), thread 0 forms the sample's
// terms; the batch sums are taken in sample order.
template <int K>
__global__ __launch_bounds__(256) void loss_finalize_kernel(const float* part, int tiles, int N, int HW,
                                                            eunet_loss_params prm, float* sums, float* loss,
                                                            float* parts) {
  constexpr int NV = 3 + 3 * K;
  __shared__ double red[256][NV];
  __shared__ double per[64], fnum[64], fden[64], nbad[64];
  const int tid = threadIdx.x;
  for (int n = 0; n < N; ++n) {
    double v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = 0.0;
    for (int t = tid; t < tiles; t += 256)
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] += (double)part[((long long)n * tiles + t) * NV + i];
#pragma unroll
    for (int i = 0; i < NV; ++i) red[tid][i] = v[i];
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if (tid < off)
#pragma unroll
        for (int i = 0; i < NV; ++i) red[tid][i] += red[tid + off][i];
      __syncthreads();
    }
    if (tid == 0) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        v[i] = red[0][i];
        sums[n * NV + i] = (float)v[i];
      }
      double dice = 0.0, tv = 0.0;
      for (int k = 0; k < K; ++k) {
        const double I = v[1 + k], S = v[1 + K + k], T = v[1 + 2 * K + k];
        dice += prm.dice_weight[k] * (1.0 - (2.0 * I + EPS) / (S + T + EPS));
        const double fp = S - I, fn = T - I;
        const double a = prm.tversky_alpha;
        tv += prm.tversky_weight[k] * (1.0 - (I + EPS) / (I + a * fp + (1.0 - a) * fn + EPS));
      }
      dice /= prm.class_div;
      tv /= prm.class_div;
      const double den = prm.focal_norm ? v[1 + 3 * K] : (double)HW;
      if (parts) {
        parts[n * 3 + 0] = (float)(v[0] / den);
        parts[n * 3 + 1] = (float)dice;
        parts[n * 3 + 2] = (float)tv;
      }
      per[n] = prm.w_dice * dice + prm.w_tversky * tv;
      fnum[n] = v[0];
      fden[n] = den;
      nbad[n] = v[2 + 3 * K];
    }
    __syncthreads();
  }
  if (tid == 0) {
    double s = 0.0, fn = 0.0, fd = 0.0, nb = 0.0;
    for (int i = 0; i < N; ++i) {
      s += per[i];
      fn += fnum[i];
      fd += fden[i];
      nb += nbad[i];
    }
    const double focal = fd > 0.0 ? fn / fd : 0.0;  // all pixels ignored: F.cross_entropy's mean is nan; 0 here
    loss[0] = (float)(prm.w_focal * focal + s / (double)N);
    sums[N * NV] = (float)fd;
    sums[N * NV + 1] = (float)nb;
  }
}

template <int K>
__global__ void loss_bwd_kernel(const float* logits, const int64_t* target, int N, int HW, eunet_loss_params prm,
                                const float* sums, const float* gloss, float* glog) {
  constexpr int NV = 3 + 3 * K;
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long long)N * HW) return;
  const int n = (int)(id / HW);
  const int p = (int)(id - (long long)n * HW);
  const long long plane = HW;
  const float* lg = logits + (long long)n * K * HW + p;
  float pr[K], lse_m, m;
  softmax_px<K>(lg, plane, pr, lse_m, m);
  const int64_t traw = target[id];
  const bool valid = traw != (int64_t)prm.ignore_index && traw >= 0 && traw < K;
  const int t = valid ? (int)traw : 0;
  float fcoef = 0.f;  // d (w_focal * focal term) / d ce * w_t
  if (valid) {
    const float logpt = lg[t * plane] - m - lse_m;
    const float ce = -prm.ce_weight[t] * logpt;
    const float pt = expf(-ce);
    float pg, pg1;
    focal_pow(1.f - pt, prm.gamma, pg, pg1);
    const float dfdce = prm.alpha[t] * (pg + ce * prm.gamma * pg1 * pt);
    fcoef = prm.w_focal * dfdce * prm.ce_weight[t] / sums[N * NV];
  }
  const float invn = 1.f / (float)N;
  const float* sm = sums + n * NV;
  float dp[K];
  float sdp = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float I = sm[1 + k], S = sm[1 + K + k], T = sm[1 + 2 * K + k];
    const float tk = (traw == (int64_t)k) ? 1.f : 0.f;
    const float ud = S + T + EPS;
    const float dd = (prm.dice_weight[k] / prm.class_div) * (-2.f * tk / ud + (2.f * I + EPS) / (ud * ud));
    const float a = prm.tversky_alpha;
    const float den = I + a * (S - I) + (1.f - a) * (T - I) + EPS;
    const float dt = -(prm.tversky_weight[k] / prm.class_div) * (tk / den - a * (I + EPS) / (den * den));
    dp[k] = prm.w_dice * dd + prm.w_tversky * dt;
    sdp += pr[k] * dp[k];
  }
  const float g0 = gloss[0];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float tk = (valid && t == k) ? 1.f : 0.f;
    const float g = invn * pr[k] * (dp[k] - sdp) + fcoef * (pr[k] - tk);
    glog[(long long)n * K * HW + k * plane + p] = g * g0;
  }
}

}  // namespace

extern "C" {

int eunet_loss_reference_params(eunet_loss_params* prm) {
  EUNET_REQUIRE(prm, "loss_reference_params: null");
  *prm = kReferenceParams;
  return EUNET_OK;
}

int eunet_loss_sums_len(int n, int k, int* len) {
  EUNET_REQUIRE(len && n > 0 && k >= 1 && k <= 3, "loss_sums_len: bad args");
  *len = n * (3 + 3 * k) + 2;
  return EUNET_OK;
}

int eunet_loss_workspace_bytes(int n, int k, int h, int w, size_t* bytes) {
  EUNET_REQUIRE(bytes && n > 0 && k >= 1 && k <= 3 && h > 0 && w > 0, "loss_workspace_bytes: bad args");
  const int tiles = cdiv(h * w, LPIX);
  *bytes = (size_t)n * tiles * (3 + 3 * k) * sizeof(float);
  return EUNET_OK;
}

int eunet_loss_fwd(const float* logits, const int64_t* target, int n, int k, int h, int w,
                   const eunet_loss_params* params, float* sums, float* loss, float* parts, void* ws, void* stream) {
  EUNET_REQUIRE(logits && target && sums && loss && ws && n > 0 && n <= 64 && k >= 1 && k <= 3,
                "loss_fwd: bad args (N <= 64, K <= 3)");
  const eunet_loss_params prm = params ? *params : kReferenceParams;
  EUNET_REQUIRE(prm.class_div > 0.f, "loss_fwd: class_div must be > 0");
  const int HW = h * w, tiles = cdiv(HW, LPIX);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(tiles, n);
#define LF(KK)                                                                                        \
  loss_fwd_kernel<KK><<<grid, NT, 0, s>>>(logits, target, HW, prm, (float*)ws);                       \
  loss_finalize_kernel<KK><<<1, 256, 0, s>>>((const float*)ws, tiles, n, HW, prm, sums, loss, parts);
  if (k == 1) { LF(1) } else if (k == 2) { LF(2) } else { LF(3) }
#undef LF
  EUNET_LAUNCH_CHECK("loss_fwd");
  return EUNET_OK;
}

int eunet_loss_bwd(const float* logits, const int64_t* target, int n, int k, int h, int w,
                   const eunet_loss_params* params, const float* sums, const float* gloss, float* glogits,
                   void* stream) {
  EUNET_REQUIRE(logits && target && sums && gloss && glogits && n > 0 && k >= 1 && k <= 3, "loss_bwd: bad args");
  const eunet_loss_params prm = params ? *params : kReferenceParams;
  const long long total = (long long)n * h * w;
  const unsigned g = (unsigned)((total + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (k == 1) loss_bwd_kernel<1><<<g, 256, 0, s>>>(logits, target, n, h * w, prm, sums, gloss, glogits);
  else if (k == 2) loss_bwd_kernel<2><<<g, 256, 0, s>>>(logits, target, n, h * w, prm, sums, gloss, glogits);
  else loss_bwd_kernel<3><<<g, 256, 0, s>>>(logits, target, n, h * w, prm, sums, gloss, glogits);
  EUNET_LAUNCH_CHECK("loss_bwd");
  return EUNET_OK;
}

}  // extern "C"
