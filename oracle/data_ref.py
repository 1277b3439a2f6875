"""CPU restatement of the reference loader's per-pixel steps (TEST INFRASTRUCTURE).

Restated from dataset.py (citations into /root/reference); only tests/ import it.
  * brightness  np.clip(image * alpha, 0, 255).astype(np.uint8)            dataset.py:243
  * contrast    np.clip(image + beta, 0, 255).astype(np.uint8)             dataset.py:251
  * noise       np.clip(image.astype(np.float32) + noise, 0, 255).astype(np.uint8)   :266-268
  * gamma       table = [((i/255)**(1/g))*255].astype(uint8); cv2.LUT = table[image] :273-276
  * flips       cv2.flip(., 1) = [:, ::-1], cv2.flip(., 0) = [::-1]          :208-222
  * ToTensor    HWC uint8 -> CHW float32 / 255                               :302-305
These are the reference's own numpy expressions, so they pin the HIP kernels exactly.
  * resize      cv2.resize(image, (w, h), interpolation=cv2.INTER_LINEAR) for uint8 images
                (dataset.py:151, 158): OpenCV's fixed-point algorithm (imgproc/src/resize.cpp),
                restated in resize_linear_u8 below -- parity unpinned against cv2 itself (absent).
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


# ---- cv2.resize INTER_LINEAR, 8U (OpenCV imgproc/src/resize.cpp) --------------------------------------
RESIZE_COEF_BITS = 11                  # INTER_RESIZE_COEF_BITS
RESIZE_ONE = 1 << RESIZE_COEF_BITS     # INTER_RESIZE_COEF_SCALE = 2048
SIMD_U8 = 16                           # v_uint8::nlanes of a 128-bit SIMD build (SSE2 / NEON)


def _coefs(n_dst, n_src):
    """Per destination index: (source index, ialpha0, ialpha1) as cv::resize computes them for
    INTER_LINEAR with fixed point: fx = (float)((dx + 0.5) * scale - 0.5) (double arithmetic, one
    cast), sx = floor(fx), fx -= sx; clamped at the borders (x only -- the caller clamps the rows);
    ialpha = saturate_cast<short>(cbuf * 2048), cbuf = (1.f - fx, fx), rounding half to even."""
    scale = 1.0 / (float(n_dst) / float(n_src))     # scale_x = 1. / inv_scale_x
    d = np.arange(n_dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    return s, f


def resize_linear_u8(img, ho, wo):
    """cv2.resize(img, (wo, ho), interpolation=INTER_LINEAR) for HWC uint8.

    * dsize == ssize: a copy.
    * exact 2x downscale in both directions (scale_x == scale_y == 2): cv2 switches to INTER_AREA,
      whose fast path is (a + b + c + d + 2) >> 2 per 2x2 block (ResizeAreaFastVec).
    * otherwise the fixed-point bilinear: horizontal pass (HResizeLinear) into int rows
      D = S[sx] * a0 + S[sx + 1] * a1 (x clamped: sx < 0 -> (0, 2048, 0); sx >= W - 1 -> (W - 1,
      2048, 0)), vertical pass on the two rows sy0, sy0 + 1 (clamped to [0, H - 1], coefficients
      not clamped): in the SIMD body (VResizeLinearVec_32s8u) dst = sat((mulhi(D0 >> 4, b0) +
      mulhi(D1 >> 4, b1) + 2) >> 2) with 16-bit mulhi; the row tail the vector loops leave
      (x >= the last multiple of 16 elements, then 8-element steps while x < width - 8) is
      scalar: dst = sat((b0 D0 + b1 D1 + 2^21) >> 22).  The reference's targets (multiples of 32
      pixels x 3 channels) are all SIMD body."""
    hi, wi = img.shape[:2]
    img3 = img if img.ndim == 3 else img[..., None]
    cn = img3.shape[2]
    if (hi, wi) == (ho, wo):
        return img.copy()
    sx_scale, sy_scale = 1.0 / (wo / wi), 1.0 / (ho / hi)
    ix, iy = int(np.rint(sx_scale)), int(np.rint(sy_scale))
    eps = np.finfo(np.float64).eps
    if abs(sx_scale - ix) < eps and abs(sy_scale - iy) < eps and ix == 2 and iy == 2:
        a = img3.astype(np.int32)
        s4 = a[0:2 * ho:2, 0:2 * wo:2] + a[0:2 * ho:2, 1:2 * wo:2] + a[1:2 * ho:2, 0:2 * wo:2] + a[1:2 * ho:2, 1:2 * wo:2]
        out = ((s4 + 2) >> 2).astype(np.uint8)
        return out if img.ndim == 3 else out[..., 0]
    sx, fx = _coefs(wo, wi)
    left = sx < 0
    right = sx >= wi - 1
    fx = np.where(left | right, np.float32(0), fx).astype(np.float32)
    sx = np.where(left, 0, np.where(right, wi - 1, sx))
    a0 = np.rint((np.float32(1) - fx) * np.float32(RESIZE_ONE)).astype(np.int64)
    a1 = np.rint(fx * np.float32(RESIZE_ONE)).astype(np.int64)
    sx1 = np.minimum(sx + 1, wi - 1)
    src = img3.astype(np.int64)
    rows = src[:, sx, :] * a0[None, :, None] + src[:, sx1, :] * a1[None, :, None]      # [hi, wo, cn] int
    sy, fy = _coefs(ho, hi)
    b0 = np.rint((np.float32(1) - fy) * np.float32(RESIZE_ONE)).astype(np.int64)
    b1 = np.rint(fy * np.float32(RESIZE_ONE)).astype(np.int64)
    r0 = rows[np.clip(sy, 0, hi - 1)].reshape(ho, wo * cn)
    r1 = rows[np.clip(sy + 1, 0, hi - 1)].reshape(ho, wo * cn)
    B0, B1 = b0[:, None], b1[:, None]
    vec = (((np.minimum(r0 >> 4, 32767) * B0) >> 16) + ((np.minimum(r1 >> 4, 32767) * B1) >> 16) + 2) >> 2
    sca = (B0 * r0 + B1 * r1 + (1 << 21)) >> 22
    width = wo * cn
    x = 0
    if width >= SIMD_U8:
        x = (width // SIMD_U8) * SIMD_U8
    while x < width - SIMD_U8 // 2:
        x += SIMD_U8 // 2
    cols = np.arange(width)[None, :]
    out = np.clip(np.where(cols < x, vec, sca), 0, 255).astype(np.uint8).reshape(ho, wo, cn)
    return out if img.ndim == 3 else out[..., 0]
