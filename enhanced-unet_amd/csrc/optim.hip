// Gradient-norm clipping + AdamW, the tail of the Trainer step (reference train_eval.py:341-343:
// clip_grad_norm_(parameters, max_norm=1.0) then optimizer.step() of the AdamW built at :120, lr
// from the scheduler, betas (0.9, 0.999), weight_decay 1e-4).
//
// Three launches over every parameter tensor at once instead of PyTorch's ~14 (per-tensor norms,
// their norm, the clip coefficient in four elementwise kernels, the in-place scale, the step
// counters, two fused-AdamW launches):
//   opt_sumsq   fp64 partial sum of g^2 per block (blocks map to (tensor, 2048-element chunk) through a
//               device table); the first block of each tensor increments its AdamW step counter
//   opt_norm    one block: the partials in a fixed order -> total = sqrt(sum) (as fp32, like
//               torch's fp32 norm), clip coefficient min(1, max_norm / (total + 1e-6))
//   opt_adamw   per element, the op order and precisions of PyTorch's fused AdamW (ADAMW mode):
//               g *= coef (stored back: p.grad holds the clipped gradient, as after clip_grad_norm_),
//               p -= lr wd p, m = b1 m + (1-b1) g, v = b2 v + (1-b2) g^2,
//               p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps), bc_i = 1 - b_i^step
// HBM: 4 B/elem (sumsq) + 32 B/elem (adamw: p, g, m, v read and written).  The norm is an fp64 sum
// where torch sums fp32 per-tensor norms, so the coefficient (and through it every update) can
// differ from torch's in the last fp32 bits; tests hold it to 1e-6 relative.  Non-finite gradients: a
// NaN or inf element makes the fp64 sum NaN / inf, the coefficient NaN / 0 as in torch, so every
// gradient becomes NaN (NaN case) or 0 with NaN at the inf elements (inf case), as torch's clip leaves
// them.  Finite fp32 gradients whose per-tensor fp32 norm overflows (|g| ~ 1e19 and up) are the one
// case where the fp64 sum stays finite and the coefficient differs from torch's 0.
#include "common.h"

namespace {

constexpr int OPT_NT = 256, OPT_EPT = 8, OPT_EPB = OPT_NT * OPT_EPT;  // elements per block
constexpr int OPT_COLS = 7;  // table row: p, g, m, v, step, numel, first block

struct OptRow {
  float* p; float* g; float* m; float* v; float* step; long long n; long long b0;
};

// the gradients' pointers as a kernel argument (they move between steps; the table's other columns
// do not, so the device table is built once per parameter storage and no copy runs per step)
struct GradPtrs {
  float* g[EUNET_OPT_KARG_MAX];
};

__device__ __forceinline__ OptRow opt_row(const long long* tab, int nt, int blk, const GradPtrs& gp) {
  int lo = 0, hi = nt - 1;  // last row whose first block <= blk (block-uniform)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid * OPT_COLS + 6] <= blk) lo = mid;
    else hi = mid - 1;
  }
  const long long* r = tab + lo * OPT_COLS;
  float* g = nt <= EUNET_OPT_KARG_MAX ? gp.g[lo] : (float*)r[1];
  return {(float*)r[0], g, (float*)r[2], (float*)r[3], (float*)r[4], r[5], r[6]};
}

__global__ __launch_bounds__(OPT_NT) void opt_sumsq_kernel(const long long* tab, int nt, double* partial,
                                                           GradPtrs gp, const double* guard) {
  __shared__ double red[OPT_NT / 64];
  const int tid = threadIdx.x, blk = blockIdx.x;
  const OptRow r = opt_row(tab, nt, blk, gp);
  const long long e0 = (blk - r.b0) * (long long)OPT_EPB + tid;
  float v[OPT_EPT];
#pragma unroll
  for (int j = 0; j < OPT_EPT; ++j) {  // loads first (clamped index), then the select
    const long long e = e0 + (long long)j * OPT_NT;
    const float x = r.g[e < r.n ? e : r.n - 1];
    v[j] = e < r.n ? x : 0.f;
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < OPT_EPT; ++j) s += (double)v[j] * (double)v[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    partial[blk] = (red[0] + red[1]) + (red[2] + red[3]);
    // AdamW state_steps += 1 (torch increments before the update); not while the update guard is raised
    if (blk == r.b0 && (guard == nullptr || *guard == 0.0)) *r.step += 1.f;
  }
}

__global__ __launch_bounds__(1024) void opt_norm_kernel(const double* partial, int nb, float max_norm,
                                                        float* coef, float* norm_out) {
  __shared__ double red[16];
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int i = tid; i < nb; i += 1024) s += partial[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += red[i];
    const float total = (float)sqrt(t);
    const float cc = max_norm / (total + 1e-6f);
    // torch's clamp(max=1) keeps a NaN (a NaN / inf gradient poisons every parameter, as there)
    *coef = cc != cc ? cc : (cc < 1.f ? cc : 1.f);
    if (norm_out) *norm_out = total;
  }
}

__global__ __launch_bounds__(OPT_NT) void opt_adamw_kernel(const long long* tab, int nt, const float* coefp, double lr,
                                                           double b1, double b2, double eps, double wd, GradPtrs gp,
                                                           const double* guard) {
  // a raised update guard (eunet_set_update_guard: a loss of this step saw an out-of-range target)
  // leaves parameters, gradients and moments as they are -- the reference raises before this update
  if (guard != nullptr && *guard != 0.0) return;
  const int tid = threadIdx.x, blk = blockIdx.x;
  const OptRow r = opt_row(tab, nt, blk, gp);
  const long long e0 = (blk - r.b0) * (long long)OPT_EPB + tid;
  const float coef = *coefp;
  const float step = *r.step;  // already incremented by opt_sumsq
  // torch's fused AdamW: the hyper-parameters are doubles, the bias corrections doubles narrowed to
  // fp32, and each update line is evaluated in the precision C++ promotes it to (double where a
  // hyper-parameter takes part), then stored as fp32
  const float bc1 = (float)(1.0 - pow(b1, (double)step));
  const float bc2s = (float)sqrt(1.0 - pow(b2, (double)step));
  const float step_size = (float)(lr / (double)bc1);
  float gv[OPT_EPT], pp[OPT_EPT], mp[OPT_EPT], vp[OPT_EPT];
#pragma unroll
  for (int j = 0; j < OPT_EPT; ++j) {
    const long long e = e0 + (long long)j * OPT_NT;
    const long long ec = e < r.n ? e : r.n - 1;
    gv[j] = r.g[ec]; pp[j] = r.p[ec]; mp[j] = r.m[ec]; vp[j] = r.v[ec];
  }
#pragma unroll
  for (int j = 0; j < OPT_EPT; ++j) {
    const long long e = e0 + (long long)j * OPT_NT;
    if (e >= r.n) continue;
    const float g = gv[j] * coef;
    float p = (float)((double)pp[j] - lr * wd * (double)pp[j]);
    const float m = (float)(b1 * (double)mp[j] + (1.0 - b1) * (double)g);
    const float v = (float)(b2 * (double)vp[j] + (1.0 - b2) * (double)g * (double)g);
    const float denom = (float)((double)(sqrtf(v) / bc2s) + eps);
    p -= step_size * m / denom;
    r.g[e] = g; r.p[e] = p; r.m[e] = m; r.v[e] = v;
  }
}

}  // namespace

int eunet_opt_table(const eunet_opt_tensor* ts, int nt, int64_t* table, int* nblocks) {
  EUNET_REQUIRE(ts && nt > 0 && table && nblocks, "opt_table: bad args");
  long long b = 0;
  for (int k = 0; k < nt; ++k) {
    const eunet_opt_tensor& t = ts[k];
    EUNET_REQUIRE(t.param && t.grad && t.exp_avg && t.exp_avg_sq && t.step && t.numel > 0,
                  "opt_table: bad tensor %d", k);
    int64_t* r = table + (long long)k * OPT_COLS;
    r[0] = (int64_t)(uintptr_t)t.param; r[1] = (int64_t)(uintptr_t)t.grad;
    r[2] = (int64_t)(uintptr_t)t.exp_avg; r[3] = (int64_t)(uintptr_t)t.exp_avg_sq;
    r[4] = (int64_t)(uintptr_t)t.step; r[5] = t.numel; r[6] = b;
    b += (t.numel + OPT_EPB - 1) / OPT_EPB;
  }
  EUNET_REQUIRE(b < (1ll << 31), "opt_table: too many elements");
  *nblocks = (int)b;
  return EUNET_OK;
}

int eunet_clip_adamw(const int64_t* table, int nt, int nblocks, float* const* grads, float max_norm, double lr,
                     double beta1, double beta2, double eps, double weight_decay, double* partial, float* coef,
                     float* total_norm, void* stream) {
  EUNET_REQUIRE(table && nt > 0 && nblocks > 0 && partial && coef, "clip_adamw: bad args");
  GradPtrs gp = {};
  if (grads != nullptr) {
    EUNET_REQUIRE(nt <= EUNET_OPT_KARG_MAX, "clip_adamw: > %d gradient pointers: leave grads null", EUNET_OPT_KARG_MAX);
    for (int k = 0; k < nt; ++k) {
      EUNET_REQUIRE(grads[k], "clip_adamw: null gradient %d", k);
      gp.g[k] = grads[k];
    }
  } else {
    EUNET_REQUIRE(nt > EUNET_OPT_KARG_MAX, "clip_adamw: pass the gradient pointers (grads) for <= %d tensors",
                  EUNET_OPT_KARG_MAX);
  }
  hipStream_t s = (hipStream_t)stream;
  const double* guard = eunet::update_guard();
  opt_sumsq_kernel<<<nblocks, OPT_NT, 0, s>>>((const long long*)table, nt, partial, gp, guard);
  opt_norm_kernel<<<1, 1024, 0, s>>>(partial, nblocks, max_norm, coef, total_norm);
  opt_adamw_kernel<<<nblocks, OPT_NT, 0, s>>>((const long long*)table, nt, coef, lr, beta1, beta2, eps,
                                              weight_decay, gp, guard);
  EUNET_LAUNCH_CHECK("clip_adamw");
  return EUNET_OK;
}
