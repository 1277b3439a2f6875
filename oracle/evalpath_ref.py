"""CPU restatement of the reference evaluation path (TEST INFRASTRUCTURE).

Used only by tests/, smoke() and bench.py (the Dice-vs-CPU-reference check) as
the checker -- never by the product path.

Restated (citations into /root/reference):
  * calculate_iou / calculate_dice      metrics.py:12-26
  * calculate_semantic_metrics          metrics.py:29-58
  * Evaluator._run_model_single         train_eval.py:397-417
  * Evaluator._run_tta_inference        train_eval.py:419-453
  * Evaluator._convert_probs_to_mask    train_eval.py:455-568 (K=3; K=2 with a zero
                                        dead-cell probability, the build's generalisation)
Pinned by tests/golden/{metrics,probs_mask,tta_c3k3}.npz (tests/test_oracle.py).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

from . import eunet_ref as R


def calculate_iou(m1: np.ndarray, m2: np.ndarray) -> float:
    inter = int(np.logical_and(m1, m2).sum())
    union = int(np.logical_or(m1, m2).sum())
    if union == 0:
        return 1.0 if inter == 0 else 0.0
    return inter / union


def calculate_dice(m1: np.ndarray, m2: np.ndarray) -> float:
    inter = int(np.logical_and(m1, m2).sum())
    s = int(np.asarray(m1).sum()) + int(np.asarray(m2).sum())  # sums of VALUES (metrics.py:24)
    if s == 0:
        return 1.0
    return 2 * inter / s


def calculate_semantic_metrics(pred: np.ndarray, gt: np.ndarray) -> Dict[str, float]:
    m: Dict[str, float] = {}
    for cid, name in enumerate(("background", "live", "dead")):
        p, g = pred == cid, gt == cid
        m[f"sem_{name}_iou"] = calculate_iou(p, g)
        m[f"sem_{name}_dice"] = calculate_dice(p, g)
    m["sem_mean_iou"] = (m["sem_live_iou"] + m["sem_dead_iou"]) / 2
    m["sem_mean_iou_all"] = (m["sem_background_iou"] + m["sem_live_iou"] + m["sem_dead_iou"]) / 3
    m["sem_mean_dice"] = (m["sem_live_dice"] + m["sem_dead_dice"]) / 2
    return m


def _split(probs):
    probs = np.asarray(probs, dtype=np.float32)
    bg, live = probs[0], probs[1]
    dead = probs[2] if probs.shape[0] == 3 else np.zeros_like(bg)
    return probs, bg, live, dead


def mask_pass1(probs: np.ndarray) -> np.ndarray:
    """train_eval.py:465-531: argmax, confidence filters, promotions, low-confidence cleanup."""
    probs, bg, live, dead = _split(probs)
    f = np.float32
    pm = np.argmax(probs, axis=0).astype(np.int64)
    max_prob = probs.max(axis=0)
    pm[(pm == 1) & ((live < f(0.42)) | (live <= bg * f(1.15)))] = 0
    pm[(pm == 2) & ((dead < f(0.5)) | (dead <= bg * f(1.3)) | (bg > f(0.3)) | (live > dead * f(0.9)))] = 0
    hl = (pm == 0) & (live > f(0.42)) & (live > bg * f(1.15)) & (live > dead * f(1.05))
    pm[hl] = 1
    hd = (pm == 0) & (dead > f(0.5)) & (dead > bg * f(1.3)) & (dead > live * f(1.1)) & (bg < f(0.3)) & ~hl
    pm[hd] = 2
    pm[(pm == 1) & (dead > live * f(1.15)) & (dead > f(0.45))] = 2
    pm[(pm == 2) & (live > dead * f(1.15)) & (live > f(0.42))] = 1
    pm[max_prob < f(0.3)] = 0
    return pm


def mask_regime(probs: np.ndarray) -> tuple:
    """(live_ratio, dead_ratio) of the pass-1 mask: which refinement branch a case reaches."""
    pm = mask_pass1(probs)
    return float((pm == 1).mean()), float((pm == 2).mean())


def convert_probs_to_mask(probs: np.ndarray) -> np.ndarray:
    """probs [K,h,w] float32 (K = 3, or 2 with dead = 0) -> int64 mask [h,w]."""
    probs, bg, live, dead = _split(probs)
    f = np.float32
    h, w = probs.shape[1:]
    pm = mask_pass1(probs)
    live_ratio = (pm == 1).sum() / (h * w)
    dead_ratio = (pm == 2).sum() / (h * w)
    if live_ratio > 0.5:  # train_eval.py:537-545
        hc = (live > f(0.5)) & (live > bg * f(1.3)) & (bg < f(0.3))
        pm[(pm == 1) & ~hc] = 0
    if dead_ratio > 0.15:  # train_eval.py:547-563
        dm = pm == 2
        if dead_ratio > 0.4:
            hc = (dead > f(0.65)) & (dead > bg * f(1.6)) & (bg < f(0.2)) & (live < dead * f(0.7))
        elif dead_ratio > 0.25:
            hc = (dead > f(0.6)) & (dead > bg * f(1.5)) & (bg < f(0.25)) & (live < dead * f(0.8))
        else:
            hc = (dead > f(0.55)) & (dead > bg * f(1.4)) & (bg < f(0.25))
        pm[dm & ~hc] = 0
    return pm


def run_model_single(S, image: torch.Tensor) -> torch.Tensor:
    """image [C,h,w] -> probs [K,h,w] with the oracle network in eval mode."""
    h, w = image.shape[1:]
    hp, wp = (32 - h % 32) % 32, (32 - w % 32) % 32
    x = image.unsqueeze(0)
    if hp or wp:
        x = F.pad(x, (0, wp, 0, hp), mode="reflect")
    out = R.forward(S, x, training=False)
    out = F.interpolate(out, size=x.shape[-2:], mode="bilinear", align_corners=False)
    return F.softmax(out[0], dim=0)[:, :h, :w]


def run_tta(S, image: torch.Tensor) -> torch.Tensor:
    h, w = image.shape[1:]
    views = [run_model_single(S, image)]
    views.append(torch.flip(run_model_single(S, torch.flip(image, dims=[2])), dims=[2]))
    views.append(torch.flip(run_model_single(S, torch.flip(image, dims=[1])), dims=[1]))
    for s in (0.75, 1.25):
        sc = F.interpolate(image.unsqueeze(0), scale_factor=s, mode="bilinear", align_corners=False).squeeze(0)
        p = run_model_single(S, sc)
        views.append(F.interpolate(p.unsqueeze(0), size=(h, w), mode="bilinear", align_corners=False).squeeze(0))
    return torch.stack(views, 0).mean(0)
