"""CPU restatement of the reference Enhanced-UNet training step (TEST INFRASTRUCTURE).

Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
the checker and the timed CPU baseline -- never by the product path.

What is restated (all citations into /root/reference):
  * BasicUNet               models.py:199-240  (DoubleConv = models.py:217-225)
  * EnhancedUNet fallback   models.py:304-314 (enhance head), 334-339 (residual)
  * get_model key schema    models.py:590-624  (109 state_dict keys)
  * FocalLoss               train_eval.py:28-60  (alpha=[1,8,5], gamma=5, w=[1,20,10], :74-79)
  * FocalLoss(alpha, gamma, ignore_index, class_weights) in general (focal_loss)
  * Trainer.dice_loss       train_eval.py:134-157 (class weights [1,15,8], eps 1e-6)
  * Trainer.tversky_loss    train_eval.py:159-181 (class weights [1,12,6], alpha 0.7)
  * _compute_combined_loss  train_eval.py:183-197 (2.5*focal + 2.5*dice + 1.0*tversky, :82-85)
  * Trainer.train_epoch     train_eval.py:236-353 (reflect / zero pad to /32 :248-253, 276-296,
                                                  per-sample bilinear resize :306-310, /B,
                                                  clip_grad_norm_(1.0) :341, AdamW :120,343)
  * LR schedule             train_eval.py:122-132 + stepping train_eval.py:1103-1111

Generalisations the build needs (the reference pins only base=64, in=3, K=3):
  * base_ch / in_ch / num_classes are parameters; widths b,2b,4b,8b; the enhance
    head keeps its hard-wired 64 mid channels (models.py:309).
  * K=2 loss == the reference K=3 loss with a third logit at -inf (its Dice and
    Tversky terms are then exactly 0 but the reference still divides by 3,
    train_eval.py:157,181).  tests/golden pins this against the reference.
Parity of this module is pinned by tests/golden/*.npz (see tests/test_oracle.py).
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .weights import formula_state_dict

# ---------------------------------------------------------------------------
# parameter schema (reference naming: models.py:199-213, 306-313)
# ---------------------------------------------------------------------------
FOCAL_ALPHA = (1.0, 8.0, 5.0)        # train_eval.py:75
CE_WEIGHT = (1.0, 20.0, 10.0)        # train_eval.py:74
DICE_W = (1.0, 15.0, 8.0)            # train_eval.py:140
TVERSKY_W = (1.0, 12.0, 6.0)         # train_eval.py:164
GAMMA = 5.0                          # train_eval.py:79
TV_ALPHA = 0.7                       # train_eval.py:159
W_FOCAL, W_DICE, W_TV = 2.5, 2.5, 1.0  # train_eval.py:83-85
LOSS_DIV = 3                         # reference hard-wires num_classes=3 (:192-193)


def block_table(base: int, in_ch: int) -> List[Tuple[str, int, int]]:
    b = base
    return [("enc1", in_ch, b), ("enc2", b, 2 * b), ("enc3", 2 * b, 4 * b),
            ("enc4", 4 * b, 8 * b), ("dec4", 8 * b + 4 * b, 4 * b),
            ("dec3", 4 * b + 2 * b, 2 * b), ("dec2", 2 * b + b, b)]


def state_spec(base: int = 64, in_ch: int = 3, num_classes: int = 3):
    """(key, shape, fan_in|None) in reference state_dict order; fan_in None = BN."""
    spec = []

    def bn(prefix, c):
        spec.extend([(f"{prefix}.weight", (c,), None), (f"{prefix}.bias", (c,), None),
                     (f"{prefix}.running_mean", (c,), None), (f"{prefix}.running_var", (c,), None),
                     (f"{prefix}.num_batches_tracked", (), None)])

    for name, ci, co in block_table(base, in_ch):
        p = f"model.{name}"
        spec.append((f"{p}.0.weight", (co, ci, 3, 3), ci * 9))
        spec.append((f"{p}.0.bias", (co,), ci * 9))
        bn(f"{p}.1", co)
        spec.append((f"{p}.3.weight", (co, co, 3, 3), co * 9))
        spec.append((f"{p}.3.bias", (co,), co * 9))
        bn(f"{p}.4", co)
    spec.append(("model.dec1.weight", (num_classes, base, 1, 1), base))
    spec.append(("model.dec1.bias", (num_classes,), base))
    spec.append(("enhance.0.weight", (64, num_classes, 3, 3), num_classes * 9))
    spec.append(("enhance.0.bias", (64,), num_classes * 9))
    bn("enhance.1", 64)
    spec.append(("enhance.3.weight", (num_classes, 64, 1, 1), 64))
    spec.append(("enhance.3.bias", (num_classes,), 64))
    return spec


def formula_weights(base=64, in_ch=3, num_classes=3, dtype=torch.float64) -> Dict[str, torch.Tensor]:
    sd = formula_state_dict(state_spec(base, in_ch, num_classes))
    out = {}
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            out[k] = torch.tensor(0, dtype=torch.long)
        else:
            out[k] = torch.from_numpy(np.asarray(v)).to(dtype)
    return out


# ---------------------------------------------------------------------------
# forward (functional; models.py:227-238 and 334-339)
# ---------------------------------------------------------------------------
def _bn(S, prefix, h, training, momentum=0.1, eps=1e-5):
    if training:
        S[prefix + ".num_batches_tracked"] += 1
    return F.batch_norm(h, S[prefix + ".running_mean"], S[prefix + ".running_var"],
                        S[prefix + ".weight"], S[prefix + ".bias"], training, momentum, eps)


# Branch pinning (test infrastructure).  The step is piecewise smooth: ReLU (models.py:221, 224, 311)
# and MaxPool2d (models.py:214) choose a branch per element, and an fp32 implementation whose
# activations sit within rounding of a kink or a tie may take the other one -- then its gradient
# jumps by a finite amount against any oracle that chose differently.  With `pins` (from the GPU's
# own saved pre-BN activations and BN affines, tests/_pins.py) the oracle evaluates the SAME
# function on the branch configuration the kernels took: ReLU(h) -> h * mask, max-pool -> gather at
# the given 2x2 argmax.  Where the masks agree with the oracle's own branches (every element not at
# a kink) this is the reference forward exactly; its backward is the exact derivative there.
def _relu(h, pin):
    return F.relu(h) if pin is None else h * pin.to(h.dtype)


def _pool(h, idx):
    """MaxPool2d(2) (models.py:214); with idx [B,C,H/2,W/2] in 0..3 (row-major in the 2x2 window):
    the element at idx instead of the max."""
    if idx is None:
        return F.max_pool2d(h, 2)
    B, C, H, W = h.shape
    w = h.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    return w.gather(-1, idx.long().unsqueeze(-1)).squeeze(-1)


def _double_conv(S, name, h, training, pins=None, prefix="model.", record=None):
    """record: optional dict receiving the BatchNorm outputs (the ReLU inputs) under name + '.1' / '.4'."""
    p = f"{prefix}{name}"
    pins = pins or {}
    h = F.conv2d(h, S[p + ".0.weight"], S[p + ".0.bias"], padding=1)
    h = _bn(S, p + ".1", h, training)
    if record is not None:
        record[name + ".1"] = h.detach()
    h = _relu(h, pins.get(name + ".1"))
    h = F.conv2d(h, S[p + ".3.weight"], S[p + ".3.bias"], padding=1)
    h = _bn(S, p + ".4", h, training)
    if record is not None:
        record[name + ".4"] = h.detach()
    return _relu(h, pins.get(name + ".4"))


def _up2(h):
    return F.interpolate(h, scale_factor=2, mode="bilinear", align_corners=False)


def trunk(S, x, training, pins=None, prefix="model.", record=None):
    """BasicUNet encoder/decoder (models.py:227-235): d2.  pins: optional branch configuration
    {'enc1.1': mask, ..., 'dec2.4': mask, 'pool1' .. 'pool3': argmax} (see _relu / _pool);
    record: optional dict receiving every ReLU input (_double_conv)."""
    pins = pins or {}
    dc = lambda nm, h: _double_conv(S, nm, h, training, pins, prefix, record)  # noqa: E731
    e1 = dc("enc1", x)
    e2 = dc("enc2", _pool(e1, pins.get("pool1")))
    e3 = dc("enc3", _pool(e2, pins.get("pool2")))
    e4 = dc("enc4", _pool(e3, pins.get("pool3")))
    d4 = dc("dec4", torch.cat([_up2(e4), e3], 1))
    d3 = dc("dec3", torch.cat([_up2(d4), e2], 1))
    d2 = dc("dec2", torch.cat([_up2(d3), e1], 1))
    return d2, dict(e1=e1, e2=e2, e3=e3, e4=e4, d4=d4, d3=d3, d2=d2)


def forward(S: Dict[str, torch.Tensor], x: torch.Tensor, training: bool = True,
            return_levels: bool = False, pins=None, record=None):
    """x [B,C,H,W] -> logits [B,K,2H,2W]; BN running stats in S are updated in train mode.
    pins: branch configuration of the trunk (trunk()) and of the head's ReLU ('enhance.1');
    record: optional dict receiving the trunk's ReLU inputs (trunk(); tests/_pins.py audit)."""
    d2, lv = trunk(S, x, training, pins, record=record)
    u = F.conv2d(_up2(d2), S["model.dec1.weight"], S["model.dec1.bias"])
    h = F.conv2d(u, S["enhance.0.weight"], S["enhance.0.bias"], padding=1)
    h = _relu(_bn(S, "enhance.1", h, training), (pins or {}).get("enhance.1"))
    out = u + F.conv2d(h, S["enhance.3.weight"], S["enhance.3.bias"])
    if return_levels:
        return out, dict(lv, u=u)
    return out


# ---------------------------------------------------------------------------
# loss (train_eval.py:28-60, 134-197), one sample: logits [K,H,W], target [H,W]
# ---------------------------------------------------------------------------
def combined_loss(logits: torch.Tensor, target: torch.Tensor, parts: bool = False):
    K = logits.shape[0]
    dt = logits.dtype
    t = target.long()
    logp = torch.log_softmax(logits, 0)
    p = logp.exp()
    w = torch.tensor(CE_WEIGHT[:K], dtype=dt)
    a = torch.tensor(FOCAL_ALPHA[:K], dtype=dt)
    ce = -w[t] * logp.gather(0, t[None])[0]
    pt = torch.exp(-ce)
    focal = (a[t] * (1 - pt) ** GAMMA * ce).mean()
    dice = logits.new_zeros(())
    tv = logits.new_zeros(())
    for c in range(K):
        pc = p[c]
        tc = (t == c).to(dt)
        inter = (pc * tc).sum()
        dice = dice + DICE_W[c] * (1.0 - (2.0 * inter + 1e-6) / (pc.sum() + tc.sum() + 1e-6))
        fp = (pc * (1 - tc)).sum()
        fn = ((1 - pc) * tc).sum()
        tv = tv + TVERSKY_W[c] * (1.0 - (inter + 1e-6) / (inter + TV_ALPHA * fp + (1 - TV_ALPHA) * fn + 1e-6))
    dice = dice / LOSS_DIV
    tv = tv / LOSS_DIV
    total = W_FOCAL * focal + W_DICE * dice + W_TV * tv
    if parts:
        return total, dict(focal=focal, dice=dice, tversky=tv)
    return total


def focal_loss(inputs, targets, alpha=None, gamma=2.0, ignore_index=None, class_weights=None):
    """train_eval.FocalLoss(alpha, gamma, ignore_index, class_weights).forward (train_eval.py:37-60)
    on batched [N,K,...] inputs."""
    if ignore_index is not None:
        ce = F.cross_entropy(inputs, targets, ignore_index=ignore_index, reduction="none", weight=class_weights)
    else:
        ce = F.cross_entropy(inputs, targets, reduction="none", weight=class_weights)
    pt = torch.exp(-ce)
    if alpha is not None:
        if isinstance(alpha, (list, torch.Tensor)):
            alpha_t = torch.zeros_like(ce)
            for i, a in enumerate(alpha):
                if ignore_index is None or i != ignore_index:
                    alpha_t[targets == i] = a
            fl = alpha_t * (1 - pt) ** gamma * ce
        else:
            fl = alpha * (1 - pt) ** gamma * ce
    else:
        fl = (1 - pt) ** gamma * ce
    return fl.mean()


def dice_loss(pred, target, num_classes=3):
    """Trainer.dice_loss (train_eval.py:134-157), batched [N,K,H,W] / [N,H,W]."""
    ps = F.softmax(pred, dim=1)
    out = []
    for c in range(num_classes):
        pc, tc = ps[:, c], (target == c).to(pred.dtype)
        inter = (pc * tc).sum(dim=(1, 2))
        union = pc.sum(dim=(1, 2)) + tc.sum(dim=(1, 2))
        out.append(((1.0 - (2.0 * inter + 1e-6) / (union + 1e-6)) * DICE_W[c]).mean())
    return sum(out) / len(out)


def tversky_loss(pred, target, num_classes=3, alpha=0.7):
    """Trainer.tversky_loss (train_eval.py:159-181), batched."""
    ps = F.softmax(pred, dim=1)
    out = []
    for c in range(num_classes):
        pc, tc = ps[:, c], (target == c).to(pred.dtype)
        tp = (pc * tc).sum(dim=(1, 2))
        fp = (pc * (1 - tc)).sum(dim=(1, 2))
        fn = ((1 - pc) * tc).sum(dim=(1, 2))
        tv = (tp + 1e-6) / (tp + alpha * fp + (1 - alpha) * fn + 1e-6)
        out.append(((1.0 - tv) * TVERSKY_W[c]).mean())
    return sum(out) / len(out)


def pad32(images: torch.Tensor, masks: torch.Tensor):
    """train_eval.py:248-253 + 276-296: images reflect-padded and masks zero-padded at the bottom /
    right to the next multiple of 32 before the forward and the loss."""
    h, w = images.shape[-2:]
    h_pad, w_pad = (32 - h % 32) % 32, (32 - w % 32) % 32
    if h_pad or w_pad:
        images = F.pad(images, (0, w_pad, 0, h_pad), mode="reflect")
        masks = F.pad(masks[:, None], (0, w_pad, 0, h_pad), mode="constant", value=0)[:, 0]
    return images, masks


def batch_loss(out2h: torch.Tensor, target: torch.Tensor):
    """train_eval.py:262-337: per-sample resize 2H->H (bilinear) + combined loss, /B."""
    B = out2h.shape[0]
    H, W = target.shape[-2:]
    loss = 0.0
    for i in range(B):
        o = out2h[i]
        if o.shape[1:] != (H, W):
            o = F.interpolate(o[None], size=(H, W), mode="bilinear", align_corners=False)[0]
        loss = loss + combined_loss(o, target[i])
    return loss / B


# ---------------------------------------------------------------------------
# train step (train_eval.py:236-353) with AdamW(4e-3, wd 1e-4) + clip 1.0
# ---------------------------------------------------------------------------
class OracleTrainer:
    def __init__(self, S: Dict[str, torch.Tensor], total_epochs: int = 50, lr: float = 4e-3):
        self.S = S
        self.keys = [k for k in S if not (k.endswith("running_mean") or k.endswith("running_var")
                                          or k.endswith("num_batches_tracked"))]
        for k in self.keys:
            S[k].requires_grad_(True)
        self.params = [S[k] for k in self.keys]
        self.total_epochs = max(1, total_epochs)
        self.optimizer = torch.optim.AdamW(self.params, lr=lr, weight_decay=1e-4, betas=(0.9, 0.999))
        self.warmup_epochs = max(1, min(5, self.total_epochs // 6))
        self.scheduler = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(
            self.optimizer, T_0=max(10, self.total_epochs // 3), T_mult=2, eta_min=1e-7)
        self.warmup_scheduler = torch.optim.lr_scheduler.LinearLR(
            self.optimizer, start_factor=0.001, end_factor=1.0, total_iters=self.warmup_epochs)

    def epoch_lr_step(self, epoch: int) -> float:
        """train_eval.py:1104-1111 -- called once per epoch before train_epoch."""
        if epoch < self.warmup_epochs:
            self.warmup_scheduler.step()
        else:
            self.scheduler.step()
        return self.optimizer.param_groups[0]["lr"]

    def step(self, images: torch.Tensor, masks: torch.Tensor, clip: bool = True):
        self.optimizer.zero_grad()
        images, masks = pad32(images, masks)
        out = forward(self.S, images, training=True)
        loss = batch_loss(out, masks)
        loss.backward()
        if clip:
            torch.nn.utils.clip_grad_norm_(self.params, max_norm=1.0)
        self.optimizer.step()
        return float(loss.item())


def lr_trajectory(total_epochs: int, lr: float = 4e-3) -> List[float]:
    S = {"w": torch.zeros(1, requires_grad=True)}
    t = OracleTrainer.__new__(OracleTrainer)
    t.total_epochs = max(1, total_epochs)
    t.optimizer = torch.optim.AdamW([S["w"]], lr=lr, weight_decay=1e-4)
    t.warmup_epochs = max(1, min(5, t.total_epochs // 6))
    t.scheduler = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(
        t.optimizer, T_0=max(10, t.total_epochs // 3), T_mult=2, eta_min=1e-7)
    t.warmup_scheduler = torch.optim.lr_scheduler.LinearLR(
        t.optimizer, start_factor=0.001, end_factor=1.0, total_iters=t.warmup_epochs)
    return [OracleTrainer.epoch_lr_step(t, e) for e in range(t.total_epochs)]


# ---------------------------------------------------------------------------
# synthetic bright-field tiles, seeded per global sample index
# ---------------------------------------------------------------------------
def flops_per_pixel(base: int, in_ch: int, K: int) -> float:
    """Train FLOP per input pixel (SURVEY.md §3.3 closed form)."""
    b, c = base, in_ch
    return 6.0 * (9 * c * b + 157.5 * b * b + 44 * b * K) - 18.0 * c * b


def avgpool_equals_resize(out2h: torch.Tensor) -> float:
    a = F.interpolate(out2h, scale_factor=0.5, mode="bilinear", align_corners=False)
    b = F.avg_pool2d(out2h, 2)
    return float((a - b).abs().max())


__all__ = ["state_spec", "formula_weights", "forward", "combined_loss", "batch_loss", "pad32", "focal_loss", "dice_loss",
           "tversky_loss",
           "OracleTrainer", "lr_trajectory", "block_table", "flops_per_pixel", "math"]
