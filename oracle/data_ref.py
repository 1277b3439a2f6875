"""CPU restatement of the reference loader's per-pixel steps (TEST INFRASTRUCTURE).

Restated from dataset.py (citations into /root/reference); only tests/ import it.
  * brightness  np.clip(image * alpha, 0, 255).astype(np.uint8)            dataset.py:243
  * contrast    np.clip(image + beta, 0, 255).astype(np.uint8)             dataset.py:251
  * noise       np.clip(image.astype(np.float32) + noise, 0, 255).astype(np.uint8)   :266-268
  * gamma       table = [((i/255)**(1/g))*255].astype(uint8); cv2.LUT = table[image] :273-276
  * flips       cv2.flip(., 1) = [:, ::-1], cv2.flip(., 0) = [::-1]          :208-222
  * ToTensor    HWC uint8 -> CHW float32 / 255                               :302-305
These are the reference's own numpy expressions, so they pin the HIP kernels exactly.
The polygon fill is the build's documented rule (even-odd at the pixel centre + every
lattice pixel on an edge), NOT cv2.fillPoly (absent here): that row is parity-unpinned.
"""
from __future__ import annotations

import numpy as np


def brightness(img, alpha):
    return np.clip(img * alpha, 0, 255).astype(np.uint8)


def contrast(img, beta):
    return np.clip(img + beta, 0, 255).astype(np.uint8)


def add_noise(img, noise):
    return np.clip(img.astype(np.float32) + noise, 0, 255).astype(np.uint8)


def gamma(img, g):
    inv = 1.0 / g
    table = np.array([((i / 255.0) ** inv) * 255 for i in np.arange(0, 256)]).astype(np.uint8)
    return table[img]


def to_tensor(img):
    return (img.astype(np.float32) / np.float32(255.0)).transpose(2, 0, 1)


def rasterize(polys, labels, h, w):
    yy, xx = np.mgrid[0:h, 0:w]
    px, py = (xx + 0.5).astype(np.float32), (yy + 0.5).astype(np.float32)
    out = np.zeros((h, w), np.int64)
    for pts, lab in zip(polys, labels):
        pts = np.asarray(pts, np.int64)
        inside = np.zeros((h, w), bool)
        edge = np.zeros((h, w), bool)
        n = len(pts)
        for k in range(n):
            xi, yi = pts[k]
            xj, yj = pts[k - 1]
            cr = (xi - xj) * (yy - yj) - (yi - yj) * (xx - xj)
            edge |= (cr == 0) & (xx >= min(xi, xj)) & (xx <= max(xi, xj)) & (yy >= min(yi, yj)) & (yy <= max(yi, yj))
            if yi != yj:
                cond = (np.float32(yi) > py) != (np.float32(yj) > py)
                xc = np.float32(xj - xi) * (py - np.float32(yi)) / np.float32(yj - yi) + np.float32(xi)
                inside ^= cond & (px < xc)
        out[inside | edge] = lab
    return out
