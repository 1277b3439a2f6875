/*
 * libeunet_hip -- C-ABI of the MI355X-native Enhanced-UNet training hot path.
 *
 * Conventions
 *   - Every entry point returns 0 on success or a negative EUNET_ERR_* code;
 *     eunet_last_error() returns the message (thread-local).
 *   - The library never allocates, frees or synchronises: all buffers and
 *     workspaces are owned by the caller (the torch caching allocator in the
 *     Python host); every launch is enqueued on the `stream` argument only
 *     (a hipStream_t passed as void*), so RCCL/DDP stream ordering stays valid.
 *   - Activations are NHWC views (eunet_act); dtype EUNET_F32 or EUNET_BF16.
 *     BatchNorm statistics, losses, weights-for-the-optimizer and all
 *     reductions are fp32 (partials combined in fp64).
 *   - Stateless and re-entrant.
 *
 * The reference exposes this path only as Python (no FFI): each entry point
 * below names the reference call site it replaces (file:line in
 * whh1747012859/Enhanced-UNet).  INTEGRATION.md shows the ctypes binding.
 */
#ifndef EUNET_H
#define EUNET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EUNET_OK 0
#define EUNET_ERR_INVALID (-1)
#define EUNET_ERR_HIP (-2)

enum { EUNET_F32 = 0, EUNET_BF16 = 1 };

/* NHWC view: element (n,y,x,c) lives at ptr + ((n*h + y)*w + x)*ctot + coff + c */
typedef struct {
  void* ptr;
  int n, h, w;  /* batch, rows, cols */
  int c;        /* channels in this view */
  int ctot;     /* channel stride of the underlying buffer (>= coff + c) */
  int coff;     /* first channel of the view inside the buffer */
  int dtype;    /* EUNET_F32 | EUNET_BF16 */
} eunet_act;

const char* eunet_version(void);
const char* eunet_last_error(void);

/* ---- layout conversion ----------------------------------------------------
 * images.to(device) + NCHW->NHWC (train_eval.py:242); x [N,C,H,W] fp32 */
int eunet_nchw_to_nhwc(const float* x, const eunet_act* out, void* stream);

/* ---- stream ordering (the backward's weight-gradient side stream; no reference counterpart: the
 * reference's backward is one stream, train_eval.py:230-243) -------------------------------------
 * `to` waits for everything enqueued on `from` so far (device-scope event release, no timing).  Both
 * streams must be on one device (any current device of the calling thread). */
int eunet_stream_wait(void* from, void* to);

/* ---- update guard (train_eval.py:325 -> FocalLoss:39: an out-of-range target raises inside the
 * loss of that batch, before its backward and optimizer.step(), so neither that batch nor any later
 * one updates the model) ----------------------------------------------------------------------------
 * guard: a device fp64 word on `device` (null: no guard).  While *guard != 0 at kernel time,
 * eunet_bn_finalize leaves the running statistics and num_batches_tracked untouched and
 * eunet_clip_adamw leaves parameters, gradients, moments and step counters untouched.  The Trainer
 * points it at the loss's out-of-range target counter, so a deferred (sync-free) epoch keeps the
 * reference's state at the raise and raises at its next host synchronisation.  The pointer is read
 * at launch (a captured graph keeps the one it was captured with). */
int eunet_set_update_guard(int device, const double* guard);

/* ---- Conv2d 3x3, padding 1 (models.py:219,222 / autograd) -----------------
 * Weights are re-packed every step from the fp32 torch parameter
 * [Cout][Cin][3][3] into the MFMA-ready layout.  transpose_flip=1 packs the
 * dgrad operand W'[ci][co][8-t] so dgrad runs through the forward kernel. */
int eunet_conv3x3_packed_bytes(int cout, int cin, int dtype, size_t* bytes);
int eunet_conv3x3_pack(const float* w, int cout, int cin, int transpose_flip, void* wp, int dtype,
                       void* stream);
/* up to EUNET_PACK_MAX packs in one launch (a step's forward and dgrad operands: the weights do
 * not change between the forward and the backward); each wp sized by eunet_conv3x3_packed_bytes */
#define EUNET_PACK_MAX 32
typedef struct {
  const float* w;  /* torch [cout][cin][3][3] fp32 */
  int cout, cin, flip;
  void* wp;
} eunet_pack_desc;
int eunet_conv3x3_pack_many(const eunet_pack_desc* descs, int n, int dtype, void* stream);
/* number of pixel tiles = rows of the BatchNorm statistics partial buffer */
int eunet_conv3x3_tiles(const eunet_act* y, int* tiles);
/* y = conv(t(x)) + bias, t = relu(x*in_scale+in_shift) per input channel when
 * in_scale != NULL (the preceding BN+ReLU fused into the operand load, zero
 * padding applied after the transform).  in_nstride = 0: one [cin] scale/shift
 * pair; > 0: per-sample pairs at in_scale + n*in_nstride (a BN+ReLU followed by a
 * Dropout2d keep-mask/(1-p), models.py:287,291, folded into the affine).  stats (nullable): [tiles][2][cout]
 * per-tile (sum, M2) plus [tiles] counts appended after 2*cout*tiles floats. */
int eunet_conv3x3_fwd(const eunet_act* x, const float* in_scale, const float* in_shift,
                      int in_nstride, const void* wp, const float* bias, const eunet_act* y, float* stats,
                      void* stream);
/* dgrad (wp_t packed with transpose_flip) fused with the reduction half of the
 * BatchNorm backward of the layer whose output gradient it produces (autograd of
 * models.py:220-221, BN+ReLU after the conv): y = that layer's pre-BN output,
 * part [tiles][2][gx.c] = per-tile (sum g', sum g' xhat), g' = gx [y scale + shift > 0],
 * xhat = (y - mean) invstd, gx as stored (rounded); scale / shift = the BN's forward
 * affine (eunet_bn_finalize), so the ReLU mask is bit-identical to the forward's and to
 * every other BN-backward kernel's.  Replaces conv3x3_fwd(dgrad) + bn_bwd_reduce;
 * colsum(part, tiles, 2C) -> (dbeta, dgamma).
 * gscale (nullable) [N][gx.c]: gx is scaled per sample and channel before the store
 * and the reduction (the backward of a Dropout2d between the BN+ReLU and this conv). */
int eunet_conv3x3_dgrad_bnbwd(const eunet_act* dy, const void* wp_t, const eunet_act* gx,
                              const eunet_act* y, const float* mean, const float* invstd,
                              const float* scale, const float* shift, const float* gscale,
                              float* part, void* stream);
/* dgrad with the whole BatchNorm backward of the layer it differentiates fused in (autograd of
 * models.py:219-224: conv -> BN -> ReLU; replaces bn_bwd_apply + dgrad).  g = gradient w.r.t. the
 * BN+ReLU output, y_in = the BN's input (the conv output, same shape and channel layout as g),
 * coef = eunet_bn_bwd_coef's [4][g.c] table; the operand staged for the MFMAs is
 * gy = k1 g [y k1 + kq > 0] + k2 y + k3 (the forward's ReLU mask), rounded to the dtype exactly as
 * eunet_bn_bwd_apply rounds it.  gy_out (nullable, g's layout) receives gy for the weight gradient
 * (bf16: stored from the staging by the co-block-0 launches; fp32: a separate apply pass, gy_out
 * then required).  y_next .. part (all or none): the reduction half of the NEXT BatchNorm backward
 * over gx, as eunet_conv3x3_dgrad_bnbwd.  gscale as eunet_conv3x3_dgrad. */
int eunet_conv3x3_dgrad_fused(const eunet_act* g, const eunet_act* y_in, const float* coef,
                              const eunet_act* gy_out, const void* wp_t, const eunet_act* gx,
                              const eunet_act* y_next, const float* mean, const float* invstd,
                              const float* scale, const float* shift, float* part, const float* gscale,
                              void* stream);
/* plain dgrad (autograd of models.py:219,222 w.r.t. the conv input): gx = conv(dy, W') with
 * wp_t packed transpose_flip; gscale (nullable) [N][gx.c] scales gx per sample and channel */
int eunet_conv3x3_dgrad(const eunet_act* dy, const void* wp_t, const eunet_act* gx, const float* gscale,
                        void* stream);
/* wgrad (split over pixel tiles): dw_part [nsplit][cout][9][cin] and
 * db_part [nsplit][cout] (db only when db_part != NULL) */
int eunet_conv3x3_wgrad_splits(const eunet_act* dy, int cin, int dtype, int* nsplit);
int eunet_conv3x3_wgrad(const eunet_act* x, const float* in_scale, const float* in_shift,
                        int in_nstride, const eunet_act* dy, float* dw_part, float* db_part, int nsplit,
                        void* stream);
/* reduce split partials -> torch layout dw [cout][cin][taps], db [cout] (fp64 combine) */
int eunet_wgrad_reduce(const float* dw_part, const float* db_part, int nsplit, int cout, int cin,
                       int taps, float* dw, float* db, void* stream);

/* ---- direct 3x3 conv for Cin <= 8: enc1.0 (models.py:203, Cin = in_channels) and the
 *      dual-branch fusion_head.0 (models.py:285, Cin = 2K); no bias when bias == NULL */
int eunet_conv_small_fwd(const eunet_act* x, const float* w, const float* bias,
                         const eunet_act* y, float* stats, void* stream);
int eunet_conv_small_wgrad_splits(const eunet_act* dy, int* nsplit);
int eunet_conv_small_wgrad(const eunet_act* x, const eunet_act* dy, float* dw_part,
                           float* db_part, int nsplit, void* stream);

/* ---- BatchNorm2d train-mode statistics (models.py:220,223; eps 1e-5, momentum 0.1)
 * combine per-tile (sum, M2, count) partials (Chan, fp64); update running
 * stats with the UNBIASED variance; emit mean, invstd and the fused affine
 * scale = gamma*invstd, shift = beta - mean*scale; num_batches_tracked (nullable,
 * int64) is incremented on the device. */
int eunet_bn_finalize(const float* stats, int tiles, int c, const float* gamma, const float* beta,
                      float eps, float momentum, float* run_mean, float* run_var, float* mean,
                      float* invstd, float* scale, float* shift, int64_t* num_batches_tracked,
                      void* stream);
/* eval-mode affine from running stats */
int eunet_bn_eval_affine(int c, const float* gamma, const float* beta, const float* run_mean,
                         const float* run_var, float eps, float* scale, float* shift, void* stream);

/* BN-apply + ReLU, out = relu(y * scale + shift) (models.py:219-222: the BatchNorm2d + ReLU between
 * the two convs of a DoubleConv), materialised once for the second conv's forward and weight
 * gradient (which then read it without applying the transform per staged halo pixel) */
int eunet_bnrelu(const eunet_act* y, const float* scale, const float* shift, const eunet_act* out, void* stream);

/* ---- fused BN-apply + ReLU consumers ----------------------------------------
 * pool: MaxPool2d(2) (models.py:214, 229-231); act (nullable) receives the
 * full-resolution activation (the skip tensor, written into its concat slot,
 * models.py:233-235). */
int eunet_bnrelu_pool(const eunet_act* y, const float* scale, const float* shift,
                      const eunet_act* act, const eunet_act* pooled, void* stream);
/* Upsample x2 bilinear, align_corners=False (models.py:215, 233-236) */
int eunet_bnrelu_upsample(const eunet_act* y, const float* scale, const float* shift,
                          const eunet_act* out, void* stream);
/* dec1 1x1 conv (models.py:212,236), commuted before the upsample:
 * z[p][k] = b[k] + sum_c w[k][c] * relu(bn(y))[p][c]; z fp32 NHWC [N,H,W,K] */
int eunet_bnrelu_conv1x1(const eunet_act* y, const float* scale, const float* shift,
                         const float* w, const float* b, int k, float* z, void* stream);

/* ---- enhance head at 2H + residual + 2x2 mean (models.py:308-313,336-337;
 *      train_eval.py:306-310 resize == 2x2 mean) ------------------------------
 * z: [N,H,W,K] fp32. out2h (nullable) [N,K,2H,2W] fp32 NCHW, logits
 * (nullable) [N,K,H,W] fp32 NCHW.  Head BN stats saved in mean/invstd (64).
 * dtype: EUNET_F32 = fp32 FMA path; EUNET_BF16 = bf16 MFMA GEMMs with fp32
 * accumulation (the reference's autocast precision for these convs). */
int eunet_head_workspace_bytes(int n, int h, int w, int k, int dtype, size_t* bytes);
int eunet_head_fwd(const float* z, int n, int h, int w, int k, const float* w1, const float* b1,
                   const float* gamma, const float* beta, const float* w2, const float* b2,
                   int training, float eps, float momentum, float* run_mean, float* run_var,
                   float* mean, float* invstd, float* out2h, float* logits, int dtype,
                   void* ws, void* stream);
/* backward from g_logits (or g_out2h when g_logits == NULL).  Writes gz and the
 * head parameter gradients gw1 [64][K][3][3], gb1, ggamma, gbeta, gw2 [K][64], gb2.
 * dtype as for head_fwd (EUNET_BF16: g_h never leaves the chip; the W1 gradient
 * is fused into the g_h pass). */
int eunet_head_bwd(const float* z, int n, int h, int w, int k, const float* w1, const float* b1,
                   const float* gamma, const float* beta, const float* w2, const float* mean,
                   const float* invstd, const float* g_logits, const float* g_out2h, float* gz,
                   float* gw1, float* gb1, float* ggamma, float* gbeta, float* gw2, float* gb2,
                   int dtype, void* ws, void* stream);

/* ---- combined loss (train_eval.py:28-60, 134-197, 262-337) ----------------
 * logits [N,K,H,W] fp32 NCHW, target [N,H,W] int64; K <= 3.  params (nullable = the
 * Trainer's enhanced_unet configuration, eunet_loss_reference_params):
 *   loss = w_focal * focal + (1/N) sum_n [w_dice dice_n + w_tversky tversky_n]
 *   focal = sum over all pixels of alpha_t (1 - pt)^gamma ce / F_den, ce = -w_t log p_t
 *           (F.cross_entropy weight = ce_weight, ignore_index pixels give ce = 0),
 *           F_den = N*H*W (FocalLoss.mean(), train_eval.py:60) or, focal_norm = 1, the sum
 *           of w_t (nn.CrossEntropyLoss(weight) mean reduction, train_eval.py:80)
 *   dice_n / tversky_n: Trainer.dice_loss / tversky_loss (:134-181), class mean over
 *           class_div classes (3 in _compute_combined_loss for any K, :192-193).
 * sums (caller-owned, saved for backward): eunet_loss_sums_len floats = [N][3+3K] partial
 * sums, then F_den, then the number of targets outside [0, K) that are not ignore_index
 * (an error in the reference: F.cross_entropy raises; the host reports it at its next sync).
 * loss: 1 fp32 on device.  parts (nullable): [N][3] focal/dice/tversky per sample. */
#define EUNET_NO_IGNORE (-2147483647 - 1) /* INT32_MIN */
typedef struct {
  float ce_weight[3];      /* FocalLoss class_weights (F.cross_entropy weight); 1 = none */
  float alpha[3];          /* FocalLoss alpha per class; 1 = none */
  float gamma;             /* FocalLoss gamma */
  int ignore_index;        /* FocalLoss ignore_index; EUNET_NO_IGNORE = none */
  float dice_weight[3];    /* Trainer.dice_loss class weights [1, 15, 8] */
  float tversky_weight[3]; /* Trainer.tversky_loss class weights [1, 12, 6] */
  float tversky_alpha;     /* 0.7 */
  float w_focal, w_dice, w_tversky;  /* term weights (2.5, 2.5, 1.0 for enhanced_unet) */
  float class_div;         /* num_classes of dice_loss / tversky_loss */
  int focal_norm;          /* 0 pixel mean, 1 ce-weight mean (CrossEntropyLoss) */
} eunet_loss_params;
int eunet_loss_reference_params(eunet_loss_params* params);
int eunet_loss_sums_len(int n, int k, int* len);
int eunet_loss_workspace_bytes(int n, int k, int h, int w, size_t* bytes);
int eunet_loss_fwd(const float* logits, const int64_t* target, int n, int k, int h, int w,
                   const eunet_loss_params* params, float* sums, float* loss, float* parts, void* ws,
                   void* stream);
/* glogits = d loss / d logits * (*gloss) (gloss: device scalar) */
int eunet_loss_bwd(const float* logits, const int64_t* target, int n, int k, int h, int w,
                   const eunet_loss_params* params, const float* sums, const float* gloss, float* glogits,
                   void* stream);

/* ---- backward helpers ----------------------------------------------------
 * BN(+ReLU) backward (autograd of models.py:220-224): g is the gradient w.r.t.
 * the ReLU output, y the pre-BN conv output, mean / invstd the batch statistics and
 * scale / shift the forward affine (scale = gamma invstd, shift = beta - mean scale, as
 * eunet_bn_finalize emits them).  The ReLU mask g' = g [y scale + shift > 0] is the
 * forward's, bit for bit, in every BN-backward kernel (reduce, apply, and the fused
 * reductions below), so the apply subtracts sums over exactly the g' it applies.
 * reduce -> part [tiles][2][c] (sum g', sum g'*xhat); colsum -> (dbeta, dgamma);
 * apply -> gy = scale (g' - dbeta/n - xhat dgamma/n). */
int eunet_bn_bwd_tiles(const eunet_act* y, int* tiles);
int eunet_bn_bwd_reduce(const eunet_act* g, const eunet_act* y, const float* mean,
                        const float* invstd, const float* scale, const float* shift, float* part,
                        void* stream);
/* deterministic column sum of a [rows][cols] fp32 partial matrix (fp64 two-stage) */
int eunet_colsum_ws_bytes(int rows, int cols, size_t* bytes);
int eunet_colsum(const float* part, int rows, int cols, float* out, void* ws, void* stream);
/* the same with columns >= split written to out_hi[col - split] (e.g. dbeta | dgamma straight
 * into their two gradient slots) */
int eunet_colsum_split(const float* part, int rows, int cols, int split, float* out_lo,
                       float* out_hi, void* ws, void* stream);
int eunet_bn_bwd_apply(const eunet_act* g, const eunet_act* y, const float* mean,
                       const float* invstd, const float* scale, const float* shift,
                       const float* dbeta, const float* dgamma, const eunet_act* gy,
                       void* stream);
/* Bounds-checked debug build (make -C enhanced-unet_amd debug -> libeunet_hip_debug.so, compiled with
 * -DEUNET_DEBUG): device-side checks on staging offsets, tile / split / block indices
 * and output addresses record the first failing check per source unit without trapping.
 * eunet_debug_enabled: 1 in the debug build, 0 in the release library (where the checks compile away).
 * eunet_debug_status: synchronises the device; *count = failed checks since the last reset,
 * *unit_line = unit * 100000 + source line of the first (units: 1 capi, 2 conv3x3, 3 bn_pool_up,
 * 4 head; 0 = none).  eunet_debug_selftest launches one deliberately failing check (capi unit). */
int eunet_debug_enabled(void);
int eunet_debug_status(unsigned* unit_line, unsigned* count, int reset);
int eunet_debug_selftest(void* stream);
/* BN-backward apply constants, coef [4][C] = (k1 = scale, kq = shift, k2, k3) with
 * gy = k1 g' + k2 y + k3 (count = N*H*W, the BN's batch); the table the fused consumers
 * (eunet_conv3x3_dgrad_fused) and eunet_bn_bwd_apply_coef read -- bit-identical to the constants
 * eunet_bn_bwd_apply forms itself. */
int eunet_bn_bwd_coef(const float* mean, const float* invstd, const float* scale, const float* shift,
                      const float* dbeta, const float* dgamma, long long count, int C, float* coef,
                      void* stream);
int eunet_bn_bwd_apply_coef(const eunet_act* g, const eunet_act* y, const float* coef, const eunet_act* gy,
                            void* stream);
/* MaxPool2d backward (first max in row-major order wins, recomputed from the
 * saved activation) + the skip-path gradient: gout = gskip + scatter(gpool) */
int eunet_pool_bwd_add(const eunet_act* act, const eunet_act* gpool, const eunet_act* gskip,
                       const eunet_act* gout, void* stream);
/* Upsample x2 backward (adjoint of the bilinear taps) */
int eunet_upsample_bwd(const eunet_act* ghi, const eunet_act* glo, void* stream);
/* The two producers above with the reduction half of eunet_bn_bwd_reduce fused in: gout / glo is
 * the gradient w.r.t. relu(bn(y)) of the DoubleConv output y (models.py:222-223), and
 * part[rows][2][C] receives (sum g', sum g' xhat) per block, rows from the *_rows query (0: the
 * channel count does not allow the fused form -- use the separate reduce).  The fused max-pool
 * adjoint does not read act (only its shape): it recomputes the activation from y as
 * eunet_bnrelu_pool stored it, round(relu(y scale + shift)), so act must be that tensor. */
int eunet_pool_bwd_add_bnr_rows(const eunet_act* gout, int* rows);
int eunet_pool_bwd_add_bnr(const eunet_act* act, const eunet_act* gpool, const eunet_act* gskip,
                           const eunet_act* gout, const eunet_act* y, const float* mean, const float* invstd,
                           const float* scale, const float* shift, float* part, void* stream);
/* gout may be NULL in eunet_pool_bwd_add_bnr: the gradient is then only reduced, and the block's apply
 * recomputes it -- eunet_bn_bwd_apply_pool = eunet_bn_bwd_apply on gout = gskip + scatter(gpool), formed and
 * rounded per 2x2 window as eunet_pool_bwd_add_bnr forms it (the same gy bit for bit, without gout's write and
 * read; even H and W).  Reference: the autograd of models.py:214, 228-230 (MaxPool2d(2) after each encoder block,
 * its input also the skip input of the decoder concat, :232-234) and models.py:222-223 (the block's second
 * BatchNorm). */
int eunet_bn_bwd_apply_pool(const eunet_act* gpool, const eunet_act* gskip, const eunet_act* y, const float* mean,
                            const float* invstd, const float* scale, const float* shift, const float* dbeta,
                            const float* dgamma, const eunet_act* gy, void* stream);
int eunet_upsample_bwd_bnr_rows(const eunet_act* glo, int* rows);
int eunet_upsample_bwd_bnr(const eunet_act* ghi, const eunet_act* glo, const eunet_act* y, const float* mean,
                           const float* invstd, const float* scale, const float* shift, float* part, void* stream);
/* dec1 1x1 backward: gact = W^T gz (w.r.t. relu(bn(y))), part [tiles][K*C + K]
 * = per-tile (gW, gb) partials */
int eunet_conv1x1_bwd_tiles(const eunet_act* y, int* tiles);
int eunet_conv1x1_bwd(const eunet_act* y, const float* scale, const float* shift,
                      const float* w, int k, const float* gz, const eunet_act* gact, float* part,
                      void* stream);
/* the same, also writing the BN-backward partial sums of y's BatchNorm over the gradient it
 * produces (what eunet_bn_bwd_reduce would compute from gact): bn_part [tiles][2][C] = per-tile
 * (sum g', sum g' xhat), g' = gact where relu(bn(y)) > 0 (scale/shift are that BN's affine form).
 * gact may be NULL: the gradient is then only reduced, not stored, and eunet_bn_bwd_apply_1x1
 * recomputes it for the apply. */
int eunet_conv1x1_bwd_bnr(const eunet_act* y, const float* scale, const float* shift,
                          const float* w, int k, const float* gz, const eunet_act* gact, float* part,
                          const float* mean, const float* invstd, float* bn_part, void* stream);
/* eunet_bn_bwd_apply for the gradient eunet_conv1x1_bwd_bnr produced without storing it: g = W^T gz
 * (w [K][C], gz [N*H*W][K] fp32) recomputed per pixel with conv1x1_bwd's arithmetic and rounding to
 * y's dtype, then gy = scale (g' - dbeta/n - xhat dgamma/n) as eunet_bn_bwd_apply -- the same gy bit for
 * bit, without the C-channel gradient's write and read.  Reference: the autograd of models.py:212, 236
 * (dec1 = Conv2d 1x1 on relu(bn(dec2's conv .3 output)), models.py:220-223). */
int eunet_bn_bwd_apply_1x1(const eunet_act* y, const float* w, int k, const float* gz, const float* mean,
                           const float* invstd, const float* scale, const float* shift, const float* dbeta,
                           const float* dgamma, const eunet_act* gy, void* stream);

/* ---- optimizer tail of the Trainer step (optim.hip; train_eval.py:341-343, AdamW from :120)
 * clip_grad_norm_(max_norm) + AdamW (decoupled weight decay) over every parameter tensor in three
 * launches.  One eunet_opt_tensor per parameter: its fp32 data, gradient (scaled in place by the
 * clip coefficient, as clip_grad_norm_ leaves it), AdamW exp_avg / exp_avg_sq and the fp32 device
 * step counter torch's fused AdamW keeps (incremented here).  eunet_opt_table writes the nt x 7
 * int64 host table (copy it to the device) and the launch's block count; partial holds nblocks
 * doubles; coef (1 float) receives the clip coefficient, total_norm (nullable) the gradient norm. */
typedef struct {
  float* param; float* grad; float* exp_avg; float* exp_avg_sq; float* step; long long numel;
} eunet_opt_tensor;
int eunet_opt_table(const eunet_opt_tensor* tensors, int nt, int64_t* table, int* nblocks);
/* grads: host array of the nt gradient pointers (nt <= EUNET_OPT_KARG_MAX; they travel as a kernel
 * argument, so a table built once serves steps whose gradients move), or null for larger nt (the
 * table's grad column is used) */
#define EUNET_OPT_KARG_MAX 256
int eunet_clip_adamw(const int64_t* table, int nt, int nblocks, float* const* grads, float max_norm,
                     double lr, double beta1, double beta2, double eps, double weight_decay,
                     double* partial, float* coef, float* total_norm, void* stream);

/* ---- evaluation path (evalpath.hip) ---------------------------------------
 * Semantic metric counts (metrics.py:29-58, calculate_semantic_metrics): pred, gt
 * int64 [n][hw]; counts int64 [n][3 classes][3] = (#pred==c, #gt==c, #both==c),
 * zeroed by the call.  IoU / Dice follow from the counts on the host. */
int eunet_semantic_counts(const int64_t* pred, const int64_t* gt, int n, long long hw,
                          int64_t* counts, void* stream);
/* calculate_iou / calculate_dice (metrics.py:12-26) of two int64 masks of n elements:
 * out int64[4] = (#(a!=0 & b!=0), #(a!=0 | b!=0), sum a, sum b), zeroed by the call */
int eunet_binary_overlap(const int64_t* a, const int64_t* b, long long n, int64_t* out,
                         void* stream);
/* Bilinear resample, align_corners=False, PyTorch upsample_bilinear2d index math
 * (F.interpolate in train_eval.py:413, 441-449): x [planes][hin][win] ->
 * y [planes][hout][wout]; scale_* = 1/scale_factor or hin/hout; flip_* mirror the
 * destination index (torch.flip, train_eval.py:427-437). */
int eunet_resize_bilinear(const float* x, int planes, int hin, int win, float* y, int hout,
                          int wout, float scale_h, float scale_w, int flip_h, int flip_w,
                          void* stream);
/* softmax over K (2 or 3) of logits [K][hp][wp], cropped to [h][w] and optionally
 * flipped (F.softmax + crop, train_eval.py:414-417) -> probs [K][h][w] */
int eunet_softmax_crop(const float* logits, int k, int hp, int wp, int h, int w, int flip_h,
                       int flip_w, float* probs, void* stream);
/* TTA mean (train_eval.py:453): mode 0 acc = p, 1 acc += p, 2 acc = (acc + p) / count */
int eunet_accumulate(float* acc, const float* p, long long n, int mode, float count,
                     void* stream);
/* _convert_probs_to_mask (train_eval.py:455-568): probs [K][h][w] (K = 3; K = 2 with a
 * zero dead-cell probability) -> mask int64 [h][w]; counts: 2 int64 of workspace. */
int eunet_probs_to_mask(const float* probs, int k, int h, int w, int64_t* mask,
                        int64_t* counts, void* stream);

/* ---- dual-branch fusion (fusion.hip) -----------------------------------------
 * SMP-path EnhancedUNet (models.py:253-302, 316-333): ff = cat(unetpp, deeplab) with the
 * branch outputs za, zb NHWC fp32 [n,h,w,K]; all gate tensors fp32 NHWC.  Per-tile
 * partials: BN statistics in the eunet_bn_finalize layout ([tiles][2][C] + counts),
 * gradient partials [tiles][cols] reduced with eunet_colsum.  K <= 3.
 * tiles: pixel tiles of the per-pixel kernels; gate_tiles: 16x32 tiles of gate_bwd3. */
int eunet_fusion_tiles(int n, int h, int w, int* tiles, int* gate_tiles);
/* attention_gate.0 (3x3, 2K->K, no bias; models.py:280): a [P][K] + BN1 stats; also
 * copies za, zb to the NCHW aux outputs (_aux_outputs, models.py:329-332) */
int eunet_gate_fwd(const float* za, const float* zb, int n, int h, int w, int k, const float* w1,
                   float* a, float* st1, float* aux_a, float* aux_b, void* stream);
/* GELU(BN1) + attention_gate.3 (1x1 K->2K, models.py:282-283): b [P][2K] + BN2 stats */
int eunet_gate_mid_fwd(const float* za, const float* zb, int n, int h, int w, int k, const float* a,
                       const float* sc1, const float* sh1, const float* w2, float* b, float* st2,
                       void* stream);
/* Sigmoid(BN2) * ff (models.py:284, 322-323) -> f2 [n,h,w,8] view c = 2K, compute dtype */
int eunet_gate_out_fwd(const float* za, const float* zb, int n, int h, int w, int k, const float* b,
                       const float* sc2, const float* sh2, const eunet_act* f2, void* stream);
/* fusion_head.11 on relu(bn3(y3)) + fusion_residual on f2 (models.py:294, 296, 325-328)
 * -> out NCHW fp32 [n,K,h,w] */
int eunet_fusion_out_fwd(const float* za, const float* zb, int k, const eunet_act* y3,
                         const float* sc3, const float* sh3, const float* w11, const float* b11,
                         const float* b, const float* sc2, const float* sh2, const float* wr,
                         const float* br, float* out, void* stream);
/* backward of the residual + output layout: gz [P][K] (NHWC, for eunet_conv1x1_bwd),
 * gf2res [P][2K] = Wr^T gout, part [tiles][K*2K + K] = (dWr, dbr) partials */
int eunet_fusion_out_bwd(const float* za, const float* zb, int n, int h, int w, int k,
                         const float* gout, const float* b, const float* sc2, const float* sh2,
                         const float* wr, float* gz, float* gf2res, float* part, void* stream);
/* gate backward: (1) sigmoid/product: gffd [P][2K], gbhat [P][2K], BN2 partials [tiles][2][2K];
 * (2) BN2 apply, 1x1, GELU': gabn [P][K], partials [tiles][2K*K + 2K] = (dWg2, BN1 sums);
 * (3) BN1 apply + transposed 3x3 + aux-output gradients (nullable, NCHW) -> branch gradients
 *     gz_a, gz_b [P][K]; partials [gate_tiles][K*2K*9] of dWg1 */
int eunet_gate_bwd1(const float* za, const float* zb, int k, const eunet_act* gf2conv,
                    const float* gf2res, const float* b, const float* mean2, const float* istd2,
                    const float* gam2, const float* bet2, float* gffd, float* gbhat, float* part,
                    void* stream);
int eunet_gate_bwd2(int n, int h, int w, int k, const float* gbhat, const float* b,
                    const float* mean2, const float* istd2, const float* gam2, const float* dbet2,
                    const float* dgam2, const float* a, const float* mean1, const float* istd1,
                    const float* gam1, const float* bet1, const float* w2, float* gabn, float* part,
                    void* stream);
int eunet_gate_bwd3(const float* za, const float* zb, int n, int h, int w, int k,
                    const float* gabn, const float* a, const float* mean1, const float* istd1,
                    const float* gam1, const float* dbet1, const float* dgam1, const float* w1,
                    const float* gffd, const float* gaux_a, const float* gaux_b, float* gz_a,
                    float* gz_b, float* part, void* stream);
/* Dropout2d(p) after a BN+ReLU (models.py:287, 291) folded into per-sample affines:
 * keep [n][c] in {0,1} -> nscale/nshift [n][c] = scale/shift * keep/(1-p) (for the
 * in_nstride operand transform of eunet_conv3x3_fwd / _wgrad) and gscale (nullable)
 * [n][c] = keep/(1-p) (for eunet_conv3x3_dgrad_bnbwd) */
int eunet_dropout_affine(const float* scale, const float* shift, const float* keep, int n, int c,
                         float p, float* nscale, float* nshift, float* gscale, void* stream);
/* consistency term of the auxiliary supervision (train_eval.py:207-232): loss =
 * sum_b c_b (1/n) sum_i MSE(softmax(branch_b[i]), softmax(fused[i])), c_b = 0.4 w_b;
 * part: [n][tiles][2] workspace (eunet_consistency_tiles).  bwd ACCUMULATES into the
 * three NCHW gradients, scaled by the device scalar gloss. */
int eunet_consistency_tiles(int h, int w, int* tiles);
int eunet_consistency_fwd(const float* fused, const float* br0, const float* br1, int n, int k,
                          int h, int w, float c0, float c1, float* part, float* loss,
                          void* stream);
int eunet_consistency_bwd(const float* fused, const float* br0, const float* br1, int n, int k,
                          int h, int w, float c0, float c1, const float* gloss, float* gfused,
                          float* g0, float* g1, void* stream);

/* ---- device-side data path (datapath.hip; dataset.py:133-321) ----------------
 * rasterize: LabelMe polygons (int32 (x, y) vertices as dataset.py:185-188 truncates them;
 * polygon i = pts[poly_off[i] .. poly_off[i+1]), label 1 live / 2 dead) -> int64 semantic
 * mask [h][w], later polygons overwrite earlier ones (dataset.py:197-201).  Fill rule:
 * even-odd at the pixel centre, plus every lattice pixel on an edge. */
int eunet_rasterize_polygons(const int* pts, const int* poly_off, const int* labels, int npoly,
                             int h, int w, int64_t* mask, void* stream);
/* per-instance uint8 masks [npoly][h][w] (dataset.py:184-193, 'instance_masks'), same fill rule,
 * mirrored horizontally (flip_h) / vertically (flip_v) as the training flips mirror every
 * instance mask (dataset.py:209-222) */
int eunet_rasterize_instances(const int* pts, const int* poly_off, int npoly, int h, int w, int flip_h,
                              int flip_v, uint8_t* masks, void* stream);
/* cv2.flip (dataset.py:208-222): mode 1 horizontal, 0 vertical; HWC uint8 / int64 mask */
int eunet_flip_u8(const uint8_t* src, uint8_t* dst, int h, int w, int c, int mode, void* stream);
int eunet_flip_mask(const int64_t* src, int64_t* dst, int h, int w, int mode, void* stream);
/* numpy pixel augmentations in the reference's order, each rounded to uint8 as numpy does:
 * flags bit0 brightness (:243), bit1 contrast (:251), bit2 + noise[n] fp32 (:266-268),
 * bit3 gamma LUT[256] (:273-276) */
int eunet_augment_u8(uint8_t* img, long long n, int flags, double alpha, double beta,
                     const float* noise, const uint8_t* lut, void* stream);
/* dataset.py:225-257 without the host round trip for the live ratio: counts = the [3][3]
 * eunet_semantic_counts of the (flipped) semantic mask (device); flags bit 0 brightness, bit 1
 * contrast; u_alpha / u_beta = the random.random() draws that random.uniform(a, b) = a + (b-a) u
 * would have made in the reference's ratio-dependent branches (one draw in every branch). */
int eunet_augment_ratio_u8(uint8_t* img, long long n, const long long* counts, int flags, double u_alpha,
                           double u_beta, void* stream);
/* transforms.ToTensor (dataset.py:302-305): HWC uint8 -> CHW float32 / 255 */
int eunet_to_tensor(const uint8_t* img, int h, int w, int c, float* out, void* stream);
/* bilinear uint8 resize with cv2 INTER_LINEAR's half-pixel mapping (dataset.py:145-157);
 * cv2's fixed-point weights are not reproduced (parity unpinned: cv2 is absent) */
int eunet_resize_u8(const uint8_t* src, int hi, int wi, int c, uint8_t* dst, int ho, int wo,
                    void* stream);

/* ---- cv2 image operations of the data / evaluation paths (imgproc.hip) -------------------------
 * Replace the cv2 calls of dataset.py:58-131 (cell-specific preprocessing), dataset.py:255-294
 * (HSV / CLAHE / sharpen augmentations) and train_eval.py:365-395 (Evaluator preprocessing).
 * All images HWC uint8 RGB, npix = h * w.  cv2 is absent from this image: the formulas follow
 * OpenCV's documented algorithms (parity unpinned). */
/* COLOR_RGB2LAB / COLOR_LAB2RGB for 8U (dataset.py:63, 71, 268, 272; train_eval.py:380-385): cv2's
 * bit-exact fixed-point conversion (RGB2Lab_b / Lab2RGBinteger of OpenCV >= 3.4 color_lab.cpp).  The
 * tables are built on the host once and copied to each device on its first call (synchronous). */
int eunet_rgb2lab_u8(const uint8_t* rgb, uint8_t* lab, long long npix, void* stream);
int eunet_lab2rgb_u8(const uint8_t* lab, uint8_t* rgb, long long npix, void* stream);
/* The host-side Lab tables (no device needed; a checker's view of what the kernels use): gamma[256],
 * cbrt[3072], yf[512], invgamma[4096] as uint16 then c_fwd[9], c_inv[9] as int32 -- 15 744 + 72 bytes. */
int eunet_lab_tables(void* out, size_t bytes);
/* cv2.COLOR_RGB2GRAY: (4899 R + 9617 G + 1868 B + 8192) >> 14 */
int eunet_rgb2gray_u8(const uint8_t* rgb, uint8_t* gray, long long npix, void* stream);
/* in place RGB -> HSV (8U, H in [0, 180)) -> adjust -> RGB.  mode bit0: S *= sat_mul
 * (dataset.py:257-261); bit1: H = (H + hue_add) mod 180, V *= val_mul (:288-292); fp32 with
 * clip and astype(uint8) truncation as the reference's float32 arrays */
int eunet_hsv_adjust_u8(uint8_t* rgb, long long npix, float sat_mul, float hue_add, float val_mul,
                        int mode, void* stream);
/* cv2.createCLAHE(clip_limit, (tiles_x, tiles_y)).apply.  mode 0: src/dst gray [h][w];
 * mode 1: src is a Lab image, its L channel is equalised and dst receives the RGB image
 * (LAB2RGB fused, dataset.py:65-71 / train_eval.py:375-381).  luts: tiles_x*tiles_y*256 bytes */
int eunet_clahe_u8(const uint8_t* src, int mode, int h, int w, double clip_limit, int tiles_x,
                   int tiles_y, uint8_t* luts, uint8_t* dst, void* stream);
/* cv2.filter2D(src, -1, k9) with a 3x3 kernel (row-major), BORDER_REFLECT_101; src != dst */
int eunet_filter3x3_u8(const uint8_t* src, uint8_t* dst, int h, int w, int c, const float* k9,
                       void* stream);
/* GaussianBlur(3x3, 1.0) + addWeighted(src, 1.3, blur, -0.3, 0) (dataset.py:126-128); src != dst */
int eunet_unsharp_u8(const uint8_t* src, uint8_t* dst, int h, int w, int c, void* stream);
/* Sobel magnitude / |Laplacian| (CV_64F) of a gray image, each max-normalised to uint8 and
 * blended 0.7 / 0.3 (dataset.py:78-91).  ws: eunet_edge_features_workspace_bytes */
int eunet_edge_features_workspace_bytes(int h, int w, size_t* bytes);
int eunet_edge_features_u8(const uint8_t* gray, int h, int w, void* ws, uint8_t* edges, void* stream);
/* in place img *= 1.1 where live_mask > 0 (dataset.py:103-107) */
int eunet_live_boost_u8(uint8_t* img, const int64_t* live_mask, long long npix, void* stream);
/* dataset.py:109-124: where dead_mask > 0 the CLAHE'd gray dead_gray replaces clahe_img (dead_gray
 * null = no dead pixels), then edge blend 0.9 / 0.1 and 0.85 / 0.15 mix with orig */
int eunet_cell_mix_u8(const uint8_t* orig, const uint8_t* clahe_img, const uint8_t* edges,
                      const int64_t* dead_mask, const uint8_t* dead_gray, long long npix,
                      uint8_t* out, void* stream);
/* Evaluator input (train_eval.py:367-377): CHW float -> HWC uint8, x * 255 when max(x) <= 1
 * (max reduced on the device), astype(uint8) truncation.  ws: eunet_chw_to_u8_workspace_bytes */
int eunet_chw_to_u8_workspace_bytes(int c, int h, int w, size_t* bytes);
int eunet_chw_to_u8(const float* x, int c, int h, int w, void* ws, uint8_t* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* EUNET_H */
