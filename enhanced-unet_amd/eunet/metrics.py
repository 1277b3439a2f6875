"""Drop-in semantic metrics of reference metrics.py (metrics.py:12-58).

    calculate_iou(mask1, mask2) -> float             # metrics.py:12-18
    calculate_dice(mask1, mask2) -> float            # metrics.py:21-26
    calculate_semantic_metrics(pred, gt) -> dict     # metrics.py:29-58 (0 bg, 1 live, 2 dead)

The pixel counting runs on the GPU (eunet_semantic_counts, integer, exact);
inputs may be numpy arrays (copied to the device) or device tensors.  The
ratios are formed on the host exactly as the reference forms them (int / int
in float64).  No CPU counting path exists.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from . import ops

CLASS_NAMES = ("background", "live", "dead")


def _dev_long(m, device=None):
    if isinstance(m, torch.Tensor):
        t = m
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(m)))
    if not t.is_cuda:
        t = t.to(device or "cuda")
    return t.long()


def _iou(inter: int, a: int, b: int) -> float:
    union = a + b - inter
    if union == 0:
        return 1.0 if inter == 0 else 0.0
    return inter / union


def _dice(inter: int, a: int, b: int) -> float:
    if a + b == 0:
        return 1.0
    return 2 * inter / (a + b)


def _overlap(mask1, mask2):
    m1 = _dev_long(mask1)
    m2 = _dev_long(mask2, m1.device)
    if m1.shape != m2.shape:
        raise ValueError(f"mask shapes differ: {tuple(m1.shape)} vs {tuple(m2.shape)}")
    return ops.binary_overlap(m1, m2)


def calculate_iou(mask1, mask2) -> float:
    inter, union, _, _ = _overlap(mask1, mask2)
    if union == 0:
        return 1.0 if inter == 0 else 0.0
    return inter / union


def calculate_dice(mask1, mask2) -> float:
    """2 |a & b| / (sum a + sum b): the reference sums mask VALUES (metrics.py:24-26)."""
    inter, _, sa, sb = _overlap(mask1, mask2)
    return _dice(inter, sa, sb)


def semantic_counts(pred_mask, gt_mask) -> np.ndarray:
    """[3][3] int64 counts (#pred==c, #gt==c, #both==c) of one mask pair (or [n][3][3] for a batch)."""
    p = _dev_long(pred_mask)
    g = _dev_long(gt_mask, p.device)
    if p.shape != g.shape:
        raise ValueError(f"mask shapes differ: {tuple(p.shape)} vs {tuple(g.shape)}")
    if p.dim() <= 2:
        return ops.semantic_counts(p.reshape(1, -1), g.reshape(1, -1))[0].cpu().numpy()
    return ops.semantic_counts(p.reshape(p.shape[0], -1), g.reshape(g.shape[0], -1)).cpu().numpy()


def metrics_from_counts(counts) -> Dict[str, float]:
    m: Dict[str, float] = {}
    for cid, name in enumerate(CLASS_NAMES):
        a, b, inter = (int(v) for v in counts[cid])
        m[f"sem_{name}_iou"] = _iou(inter, a, b)
        m[f"sem_{name}_dice"] = _dice(inter, a, b)
    mean_iou = (m["sem_background_iou"] + m["sem_live_iou"] + m["sem_dead_iou"]) / 3
    m["sem_mean_iou"] = (m["sem_live_iou"] + m["sem_dead_iou"]) / 2
    m["sem_mean_iou_all"] = mean_iou
    m["sem_mean_dice"] = (m["sem_live_dice"] + m["sem_dead_dice"]) / 2
    return m


def calculate_semantic_metrics(pred_mask, gt_mask) -> Dict[str, float]:
    return metrics_from_counts(semantic_counts(pred_mask, gt_mask))
