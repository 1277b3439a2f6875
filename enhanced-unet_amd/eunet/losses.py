"""Fused combined loss (focal + Dice + Tversky) as one autograd node.

Reference: train_eval.py:28-60 (FocalLoss), 134-181 (dice/tversky), 183-197
(_compute_combined_loss), 262-337 (per-sample loop, sum, /B).  One kernel pass
computes every sample's per-class sums; backward is analytic per pixel.
"""
from __future__ import annotations

import torch

from . import ops


class CombinedLossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, return_parts=False):
        logits = logits.contiguous().float()
        target = target.contiguous().long()
        n, k, h, w = logits.shape
        if target.shape != (n, h, w):
            raise ValueError(f"target {tuple(target.shape)} does not match logits {tuple(logits.shape)}")
        dev = logits.device
        sums = torch.empty(n * (1 + 3 * k), dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        parts = torch.empty(n, 3, dtype=torch.float32, device=dev)
        ws = torch.empty(ops.loss_workspace_bytes(n, k, h, w), dtype=torch.uint8, device=dev)
        ops.loss_fwd(logits, target, sums, loss, parts, ws)
        ctx.save_for_backward(logits, target, sums)
        ctx.mark_non_differentiable(parts)
        return loss, parts

    @staticmethod
    def backward(ctx, gloss, gparts):
        logits, target, sums = ctx.saved_tensors
        glog = torch.empty_like(logits)
        ops.loss_bwd(logits, target, sums, gloss.contiguous().float().reshape(1), glog)
        return glog, None, None


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


def combined_loss(logits: torch.Tensor, target: torch.Tensor, return_parts: bool = False):
    """Batched train_eval loss: logits [B,K,H,W] (already at mask size), target [B,H,W]
    -> (1/B) sum_b [2.5 focal_b + 2.5 dice_b + 1.0 tversky_b]."""
    loss, parts = CombinedLossFunction.apply(logits, target)
    return (loss, parts) if return_parts else loss
