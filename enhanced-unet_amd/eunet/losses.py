"""Fused combined loss (focal + Dice + Tversky) as one autograd node, and the reference's
loss modules on top of it.

Reference: train_eval.py:28-60 (FocalLoss), :80 (nn.CrossEntropyLoss(weight)), 134-181
(dice/tversky), 183-197 (_compute_combined_loss), 262-337 (per-sample loop, sum, /B).
One kernel pass computes every sample's per-class sums; backward is analytic per pixel.
Each term is differentiable on its own: the kernel takes the term weights
(eunet_loss_params), so FocalLoss / dice_loss / tversky_loss / CrossEntropyLoss are the
same kernel with the other weights at zero.

Targets outside [0, K) (other than ignore_index) make the reference raise inside
F.cross_entropy -- on the GPU as an asynchronous device assert that surfaces at the next
synchronisation.  Here the kernel counts them on the device and check_targets() raises
ValueError at the next host synchronisation of the training loop (Trainer.step's
loss.item(), the end of Trainer.train_epoch), or immediately with combined_loss(...,
validate=True).
"""
from __future__ import annotations

from typing import Optional, Sequence, Union

import torch
import torch.nn as nn

from . import ops
from ._lib import LossParams

NO_IGNORE = -(2 ** 31)  # EUNET_NO_IGNORE


_host_copies = {}  # id(tensor) -> (weakref, _version, values): no device sync per training step


def _host_values(t: torch.Tensor):
    """t's values as a Python list.  A device tensor is copied once and re-copied only after an
    in-place change (t._version): the Trainer rebuilds its loss parameters every step from
    self.focal_loss.class_weights, a cuda tensor, and a .cpu() there would drain the launch queue."""
    import weakref
    hit = _host_copies.get(id(t))
    if hit is not None and hit[0]() is t and hit[1] == t._version:
        return hit[2]
    vals = t.detach().cpu().reshape(-1).tolist()
    if len(_host_copies) > 64:
        _host_copies.clear()
    _host_copies[id(t)] = (weakref.ref(t), t._version, vals)
    return vals


def _triple(v, default: float, what: str):
    """A per-class table of 3 floats from None / a scalar / a list / a tensor (missing classes 0)."""
    if v is None:
        return [default] * 3
    if isinstance(v, torch.Tensor):
        v = _host_values(v)
    if isinstance(v, (int, float)):
        return [float(v)] * 3
    v = [float(a) for a in v]
    if len(v) > 3:
        raise ValueError(f"{what}: at most 3 classes are supported, got {len(v)} values")
    return v + [0.0] * (3 - len(v))


def make_params(*, ce_weight=None, alpha=None, gamma: float = 5.0, ignore_index: Optional[int] = None,
                dice_weight=(1.0, 15.0, 8.0), tversky_weight=(1.0, 12.0, 6.0), tversky_alpha: float = 0.7,
                w_focal: float = 2.5, w_dice: float = 2.5, w_tversky: float = 1.0, class_div: float = 3.0,
                focal_norm: int = 0) -> LossParams:
    """eunet_loss_params; the defaults other than ce_weight/alpha are the Trainer's enhanced_unet
    configuration (train_eval.py:74-87, 140, 164, 175).  alpha as FocalLoss treats it: a list
    gives per-class values (classes past its end get 0, train_eval.py:50-53), a scalar applies to
    every class, None means 1."""
    p = LossParams()
    p.ce_weight[:] = _triple(ce_weight, 1.0, "class_weights")
    p.alpha[:] = _triple(alpha, 1.0, "alpha")
    p.gamma = float(gamma)
    p.ignore_index = NO_IGNORE if ignore_index is None else int(ignore_index)
    p.dice_weight[:] = _triple(dice_weight, 1.0, "dice weights")
    p.tversky_weight[:] = _triple(tversky_weight, 1.0, "tversky weights")
    p.tversky_alpha = float(tversky_alpha)
    p.w_focal, p.w_dice, p.w_tversky = float(w_focal), float(w_dice), float(w_tversky)
    p.class_div = float(class_div)
    p.focal_norm = int(focal_norm)
    return p


_REFERENCE = None


def reference_params() -> LossParams:
    """The Trainer's enhanced_unet loss (the library's built-in default)."""
    global _REFERENCE
    if _REFERENCE is None:
        _REFERENCE = ops.loss_reference_params()
    return _REFERENCE


# ---- out-of-range target bookkeeping (see module docstring) --------------------------------
_bad = {}  # device -> fp64 [1] accumulator of out-of-range targets since the last check
_bad_pending = False  # a loss call (or a graph replay holding one) ran since the last check


def bad_target_accumulator(device) -> torch.Tensor:
    """The persistent per-device counter the loss adds its out-of-range count to, in place: a
    captured step graph (train_eval.StepGraph) keeps accumulating into it on every replay."""
    dev = torch.device(device)
    acc = _bad.get(dev)
    if acc is None:
        acc = _bad[dev] = torch.zeros(1, dtype=torch.float64, device=dev)
    return acc


def mark_pending():
    global _bad_pending
    _bad_pending = True


def _record_bad(sums: torch.Tensor):
    bad_target_accumulator(sums.device).add_(sums[-1:])
    mark_pending()


def check_targets():
    """Raise ValueError if any loss call since the last check saw a target outside [0, K)
    (synchronises with the device)."""
    global _bad_pending
    if not _bad_pending:
        return
    _bad_pending = False
    n = 0
    for acc in _bad.values():
        n += int(acc.item())
        acc.zero_()
    if n:
        raise ValueError(f"{n} target value(s) outside [0, num_classes) reached the loss "
                         f"(F.cross_entropy would raise: class index out of bounds)")


class CombinedLossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, params, track_targets):
        logits = logits.contiguous().float()
        target = target.contiguous().long()
        n, k, h, w = logits.shape
        if target.shape != (n, h, w):
            raise ValueError(f"target {tuple(target.shape)} does not match logits {tuple(logits.shape)}")
        dev = logits.device
        sums = torch.empty(ops.loss_sums_len(n, k), dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        parts = torch.empty(n, 3, dtype=torch.float32, device=dev)
        ws = torch.empty(ops.loss_workspace_bytes(n, k, h, w), dtype=torch.uint8, device=dev)
        ops.loss_fwd(logits, target, params, sums, loss, parts, ws)
        if track_targets:
            _record_bad(sums)
        ctx.save_for_backward(logits, target, sums)
        ctx.params = params
        ctx.mark_non_differentiable(parts)
        return loss, parts

    @staticmethod
    def backward(ctx, gloss, gparts):
        logits, target, sums = ctx.saved_tensors
        glog = torch.empty_like(logits)
        ops.loss_bwd(logits, target, ctx.params, sums, gloss.contiguous().float().reshape(1), glog)
        return glog, None, None, None


class ConsistencyFunction(torch.autograd.Function):
    """sum_b c_b (1/B) sum_i MSE(softmax(branch_b[i]), softmax(fused[i])) (train_eval.py:207-232;
    the fused probabilities are not detached in the reference, so both sides get gradients)."""

    @staticmethod
    def forward(ctx, fused, br0, br1, c0, c1):
        fused, br0, br1 = (t.contiguous().float() for t in (fused, br0, br1))
        n, k, h, w = fused.shape
        part = torch.empty(n * ops.consistency_tiles(h, w) * 2, dtype=torch.float32, device=fused.device)
        loss = torch.empty((), dtype=torch.float32, device=fused.device)
        ops.consistency_fwd(fused, br0, br1, c0, c1, part, loss)
        ctx.save_for_backward(fused, br0, br1)
        ctx.c = (c0, c1)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        fused, br0, br1 = ctx.saved_tensors
        gf, g0, g1 = (torch.zeros_like(t) for t in (fused, br0, br1))
        ops.consistency_bwd(fused, br0, br1, ctx.c[0], ctx.c[1], gloss.contiguous().float().reshape(1), gf, g0, g1)
        return gf, g0, g1, None, None


def consistency_loss(fused, br0, br1, c0: float, c1: float):
    return ConsistencyFunction.apply(fused, br0, br1, float(c0), float(c1))


def combined_loss(logits: torch.Tensor, target: torch.Tensor, return_parts: bool = False,
                  params: Optional[LossParams] = None, validate: bool = False, track_targets: bool = True):
    """Batched train_eval loss: logits [B,K,H,W] (already at mask size), target [B,H,W]
    -> (1/B) sum_b [w_focal focal_b + w_dice dice_b + w_tversky tversky_b] (params: None =
    the reference Trainer's 2.5 / 2.5 / 1.0 configuration)."""
    loss, parts = CombinedLossFunction.apply(logits, target, params, track_targets)
    if validate:
        check_targets()
    return (loss, parts) if return_parts else loss


def _as_pixels(inputs: torch.Tensor, targets: torch.Tensor):
    """[N,K,*] logits / [N,*] targets -> [1,K,1,P] / [1,1,P] (pixel-mean losses only)."""
    if inputs.dim() < 2:
        raise ValueError(f"expected [N, C, ...] logits, got {tuple(inputs.shape)}")
    k = inputs.shape[1]
    if targets.shape != inputs.shape[:1] + inputs.shape[2:]:
        raise ValueError(f"target {tuple(targets.shape)} does not match input {tuple(inputs.shape)}")
    lg = inputs.float().movedim(1, -1).reshape(-1, k).t().reshape(1, k, 1, -1)
    return lg, targets.reshape(1, 1, -1)


class FocalLoss(nn.Module):
    """train_eval.FocalLoss (train_eval.py:28-60): mean over all pixels of
    alpha_t (1-pt)^gamma ce, ce = F.cross_entropy(inputs, targets, weight=class_weights,
    ignore_index, reduction='none'), pt = exp(-ce).  inputs [N,K,...] (K <= 3) on the GPU."""

    def __init__(self, alpha: Union[None, float, Sequence[float], torch.Tensor] = None, gamma: float = 2.0,
                 ignore_index: Optional[int] = None, class_weights: Optional[torch.Tensor] = None):
        super().__init__()
        self.alpha = alpha
        self.gamma = gamma
        self.ignore_index = ignore_index
        self.class_weights = class_weights

    def params(self) -> LossParams:
        return make_params(ce_weight=self.class_weights, alpha=self.alpha, gamma=self.gamma,
                           ignore_index=self.ignore_index, w_focal=1.0, w_dice=0.0, w_tversky=0.0)

    def forward(self, inputs, targets):
        lg, tg = _as_pixels(inputs, targets)
        return combined_loss(lg, tg, params=self.params())


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss(weight=...) as the reference Trainer builds it (train_eval.py:80):
    class-weighted mean of -log p_t (sum w_t nll / sum w_t), on the fused loss kernel."""

    def __init__(self, weight: Optional[torch.Tensor] = None, ignore_index: int = -100,
                 reduction: str = "mean"):
        super().__init__()
        if reduction != "mean":
            raise ValueError("only reduction='mean' (the reference's use) is built")
        self.weight = weight
        self.ignore_index = ignore_index

    def forward(self, inputs, targets):
        lg, tg = _as_pixels(inputs, targets)
        p = make_params(ce_weight=self.weight, alpha=None, gamma=0.0, ignore_index=self.ignore_index,
                        w_focal=1.0, w_dice=0.0, w_tversky=0.0, focal_norm=1)
        return combined_loss(lg, tg, params=p)


def dice_loss(pred, target, num_classes: int = 3):
    """Trainer.dice_loss (train_eval.py:134-157): classes range(num_classes), weights [1,15,8],
    mean over samples of each class term, then / num_classes."""
    w = [1.0, 15.0, 8.0]
    w = [w[c] if c < num_classes else 0.0 for c in range(3)]
    p = make_params(dice_weight=w, w_focal=0.0, w_dice=1.0, w_tversky=0.0, class_div=float(num_classes))
    return combined_loss(pred, target, params=p, track_targets=False)


def tversky_loss(pred, target, num_classes: int = 3, alpha: float = 0.7):
    """Trainer.tversky_loss (train_eval.py:159-181): weights [1,12,6], Tversky alpha."""
    w = [1.0, 12.0, 6.0]
    w = [w[c] if c < num_classes else 0.0 for c in range(3)]
    p = make_params(tversky_weight=w, tversky_alpha=alpha, w_focal=0.0, w_dice=0.0, w_tversky=1.0,
                    class_div=float(num_classes))
    return combined_loss(pred, target, params=p, track_targets=False)


__all__ = ["combined_loss", "consistency_loss", "check_targets", "make_params", "reference_params", "FocalLoss",
           "CrossEntropyLoss", "dice_loss", "tversky_loss"]
