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
  * fillPoly    cv2.fillPoly(mask, [points], 1) (dataset.py:184-186, default LINE_8, shift 0):
                OpenCV 4.x's algorithm (modules/imgproc/src/drawing.cpp of 4.5.2 and later, the
                versions `opencv-python>=4.5.0` installs today): CollectPolyEdges draws every edge
                with the 8-connected Bresenham Line (LineIterator, endpoints clipped by clipLine)
                and collects the non-horizontal edges in XY_SHIFT = 16 fixed point (x + 1/2 for
                in-image edges; clipped endpoints re-projected), FillEdgeCollection fills each
                scanline between consecutive active edges of the x-sorted list.  Restated in
                fill_poly_u8 below -- parity unpinned against cv2 itself (absent).
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


# ---- cv2.fillPoly, LINE_8, shift 0 (OpenCV 4.x imgproc/src/drawing.cpp) ------------------------------
XY_SHIFT = 16
XY_ONE = 1 << XY_SHIFT


def _cdiv(a, b):
    """C++ integer division (truncation toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def clip_line(w, h, p1, p2):
    """clipLine(Size2l, Point2l&, Point2l&): Cohen-Sutherland against [0, w-1] x [0, h-1], the
    crossings offset by (int64)(double(a - y) * (x2 - x1) / (y2 - y1)).  Returns (inside, p1, p2)."""
    (x1, y1), (x2, y2) = p1, p2
    right, bottom = w - 1, h - 1
    if w <= 0 or h <= 0:
        return False, (x1, y1), (x2, y2)
    c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8
    c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8
    if (c1 & c2) == 0 and (c1 | c2) != 0:
        if c1 & 12:
            a = 0 if c1 < 8 else bottom
            x1 += int(float(a - y1) * (x2 - x1) / (y2 - y1))
            y1 = a
            c1 = (x1 < 0) + (x1 > right) * 2
        if c2 & 12:
            a = 0 if c2 < 8 else bottom
            x2 += int(float(a - y2) * (x2 - x1) / (y2 - y1))
            y2 = a
            c2 = (x2 < 0) + (x2 > right) * 2
        if (c1 & c2) == 0 and (c1 | c2) != 0:
            if c1:
                a = 0 if c1 == 1 else right
                y1 += int(float(a - x1) * (y2 - y1) / (x2 - x1))
                x1 = a
                c1 = 0
            if c2:
                a = 0 if c2 == 1 else right
                y2 += int(float(a - x2) * (y2 - y1) / (x2 - x1))
                x2 = a
                c2 = 0
    return (c1 | c2) == 0, (x1, y1), (x2, y2)


def line8(img, p1, p2, color=1):
    """Line(img, pt1, pt2, color, 8): LineIterator(img, pt1, pt2, 8, leftToRight=true) -- endpoints
    clipped to the image, the left endpoint first, Bresenham with err = dx - 2 dy, count = dx + 1."""
    h, w = img.shape
    (x1, y1), (x2, y2) = p1, p2
    if not (0 <= x1 < w and 0 <= x2 < w and 0 <= y1 < h and 0 <= y2 < h):
        ok, (x1, y1), (x2, y2) = clip_line(w, h, (x1, y1), (x2, y2))
        if not ok:
            return
    dx, dy = x2 - x1, y2 - y1
    if dx < 0:  # leftToRight: start from the left endpoint
        dx, dy = -dx, -dy
        x1, y1, x2, y2 = x2, y2, x1, y1
    sy = -1 if dy < 0 else 1
    dy = abs(dy)
    # (major step, minor step) in (x, y); the steep case swaps the axes
    if dy > dx:
        dx, dy = dy, dx
        major, minor = (0, sy), (1, 0)
    else:
        major, minor = (1, 0), (0, sy)
    err = dx - (dy + dy)
    plus_delta, minus_delta = dx + dx, -(dy + dy)
    x, y = x1, y1
    for _ in range(dx + 1):
        img[y, x] = color
        step_minor = err < 0
        err += minus_delta + (plus_delta if step_minor else 0)
        x += major[0] + (minor[0] if step_minor else 0)
        y += major[1] + (minor[1] if step_minor else 0)


def collect_poly_edges(img, pts, edges, color=1):
    """CollectPolyEdges (LINE_8, shift 0, offset 0): draws every edge and appends the non-horizontal
    ones as [y0, y1, x (XY_SHIFT fixed point at y0), dx per row]."""
    h, w = img.shape
    n = len(pts)
    pt0 = (int(pts[n - 1][0]) << XY_SHIFT, int(pts[n - 1][1]))
    for i in range(n):
        pt1 = (int(pts[i][0]) << XY_SHIFT, int(pts[i][1]))
        t0 = ((pt0[0] + (XY_ONE >> 1)) >> XY_SHIFT, pt0[1])
        t1 = ((pt1[0] + (XY_ONE >> 1)) >> XY_SHIFT, pt1[1])
        line8(img, t0, t1, color)
        p0c, p1c = list(pt0), list(pt1)
        if not (0 <= t0[0] < w and 0 <= t1[0] < w and 0 <= t0[1] < h and 0 <= t1[1] < h):
            _, c0, c1 = clip_line(w, h, t0, t1)  # the clipped copies feed the edge even when invisible
            if c0[1] != c1[1]:
                p0c = [c0[0] << XY_SHIFT, c0[1]]
                p1c = [c1[0] << XY_SHIFT, c1[1]]
        else:
            p0c[0] += XY_ONE >> 1
            p1c[0] += XY_ONE >> 1
        if pt0[1] != pt1[1]:
            dx = _cdiv(p1c[0] - p0c[0], p1c[1] - p0c[1])
            if pt0[1] < pt1[1]:
                edges.append([pt0[1], pt1[1], p0c[0] + (pt0[1] - p0c[1]) * dx, dx])
            else:
                edges.append([pt1[1], pt0[1], p1c[0] + (pt1[1] - p1c[1]) * dx, dx])
        pt0 = pt1


def fill_edge_collection(img, edges, color=1):
    """FillEdgeCollection (LINE_8: delta 0): rows y0_min .. min(y1_max, rows) - 1; per row the active
    edges (y0 <= y < y1) sorted by x, consecutive pairs filled from (x_a >> 16) to (x_b >> 16), clipped
    to the image; each edge's x advances by dx per row."""
    h, w = img.shape
    if len(edges) < 2:
        return
    y_min = min(e[0] for e in edges)
    y_max = max(e[1] for e in edges)
    xs = [e[2] for e in edges] + [e[2] + (e[1] - e[0]) * e[3] for e in edges]
    if y_max < 0 or y_min >= h or max(xs) < 0 or min(xs) >= (w << XY_SHIFT):
        return
    for y in range(y_min, min(y_max, h)):
        act = sorted(e[2] + (y - e[0]) * e[3] for e in edges if e[0] <= y < e[1])
        if y < 0:
            continue
        for a, b in zip(act[0::2], act[1::2]):
            x1, x2 = a >> XY_SHIFT, b >> XY_SHIFT
            if x1 < w and x2 >= 0:
                img[y, max(x1, 0):min(x2, w - 1) + 1] = color


def fill_poly_u8(pts, h, w):
    """cv2.fillPoly(np.zeros((h, w), np.uint8), [pts], 1) for int32 points pts [n, 2] (x, y)."""
    img = np.zeros((h, w), np.uint8)
    edges = []
    collect_poly_edges(img, np.asarray(pts, np.int64), edges)
    fill_edge_collection(img, edges)
    return img


def rasterize(polys, labels, h, w):
    """dataset.py:184-200: one fillPoly mask per polygon, then semantic[mask > 0] = label in polygon
    order (the last polygon wins)."""
    out = np.zeros((h, w), np.int64)
    for pts, lab in zip(polys, labels):
        out[fill_poly_u8(pts, h, w) > 0] = lab
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
