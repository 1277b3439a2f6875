"""Synthetic bright-field cell tiles; no dataset is available offline.

x in [0,1]: smooth illumination field + Poisson(H*W/4000) elliptical cells
(radius U[4,14] px, darker halo, brighter core) + N(0, 0.03) noise, clamped.
mask: 0 background / 1 cell (K=2) or 1 live / 2 dead with p 0.7 / 0.3 (K=3).
Seeded per global sample index (seed = 1000 + index), generated on the host
once and moved to the device (the benchmark keeps them resident in HBM).
"""
from __future__ import annotations

import numpy as np
import torch


def tile(h: int, w: int, index: int, num_classes: int = 2, in_channels: int = 1):
    rng = np.random.default_rng(1000 + index)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    fx, fy, ph = rng.uniform(0.5, 2.0), rng.uniform(0.5, 2.0), rng.uniform(0, 2 * np.pi)
    img = 0.55 + 0.12 * np.sin(2 * np.pi * fx * xx / w + ph) * np.cos(2 * np.pi * fy * yy / h)
    mask = np.zeros((h, w), np.int64)
    ncell = rng.poisson(h * w / 4000.0)
    for _ in range(ncell):
        cy, cx = rng.uniform(0, h), rng.uniform(0, w)
        ra, rb = rng.uniform(4, 14), rng.uniform(4, 14)
        th = rng.uniform(0, np.pi)
        cls = 1 if (num_classes < 3 or rng.uniform() < 0.7) else 2
        r = int(np.ceil(max(ra, rb))) + 3
        y0, y1 = max(0, int(cy) - r), min(h, int(cy) + r + 1)
        x0, x1 = max(0, int(cx) - r), min(w, int(cx) + r + 1)
        if y0 >= y1 or x0 >= x1:
            continue
        dy, dx = yy[y0:y1, x0:x1] - cy, xx[y0:y1, x0:x1] - cx
        u = (dx * np.cos(th) + dy * np.sin(th)) / ra
        v = (-dx * np.sin(th) + dy * np.cos(th)) / rb
        d = np.sqrt(u * u + v * v)
        inside = d <= 1.0
        halo = (d > 0.8) & (d <= 1.25)
        img[y0:y1, x0:x1] -= 0.18 * halo
        img[y0:y1, x0:x1] += 0.25 * np.clip(1.0 - d / 0.8, 0.0, 1.0) * (0.6 if cls == 2 else 1.0)
        mask[y0:y1, x0:x1][inside] = cls
    img += rng.normal(0.0, 0.03, size=(h, w))
    img = np.clip(img, 0.0, 1.0).astype(np.float32)
    x = np.repeat(img[None], in_channels, axis=0)
    return x, mask


def batch(n: int, h: int, w: int, start_index: int = 0, num_classes: int = 2, in_channels: int = 1,
          device="cpu"):
    xs, ms = zip(*[tile(h, w, start_index + i, num_classes, in_channels) for i in range(n)])
    x = torch.from_numpy(np.stack(xs)).to(device)
    m = torch.from_numpy(np.stack(ms)).to(device)
    return x, m


def loader(n_batches: int, batch_size: int, h: int, w: int, start_index: int = 0, num_classes: int = 2,
           in_channels: int = 1):
    """A list of collate_fn-style batches (dataset.py:355-361) of synthetic tiles."""
    out = []
    for b in range(n_batches):
        x, m = batch(batch_size, h, w, start_index + b * batch_size, num_classes, in_channels)
        out.append({"images": x, "batch_items": [{"semantic_mask": m[i]} for i in range(batch_size)]})
    return out
