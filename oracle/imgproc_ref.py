"""CPU restatement of the cv2 operations on the reference's data / evaluation paths
(TEST INFRASTRUCTURE -- only tests/ import it).

Call sites (citations into /root/reference):
  dataset.py:58-131    _apply_cell_specific_preprocessing     -> cell_preprocess
  dataset.py:259-264   HSV saturation augmentation             -> hsv_adjust(sat=)
  dataset.py:267-272   CLAHE(U(1.5, 3)) augmentation           -> clahe_rgb
  dataset.py:287-292   filter2D sharpen augmentation           -> filter3x3
  dataset.py:295-300   HSV jitter augmentation                 -> hsv_adjust(hue=, val=)
  train_eval.py:365-395  Evaluator._prepare_image_tensor       -> chw_to_u8, clahe_rgb, filter3x3

PARITY UNPINNED: cv2 is not importable in this image and the reference holds no cv2
fixtures, so this file restates OpenCV's published algorithms (imgproc color_lab / color_hsv
/ clahe / filter / smooth modules) rather than being checked against cv2 itself.  The
numpy steps around the cv2 calls (the 1.1 / 0.9 / 0.1 / 0.85 / 0.15 fp32 blends, the
fp64 edge normalisation, astype(uint8) truncations) are the reference's own expressions.
RGB<->Lab 8U follows cv2's bit-exact fixed-point tables (OpenCV >= 3.4).  Every fp32 step rounds per operation
(np.float32 arithmetic), matching the kernels, which are compiled without FMA contraction.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def reflect101(i, n):
    i = np.asarray(i)
    if n == 1:
        return np.zeros_like(i)
    while np.any((i < 0) | (i >= n)):
        i = np.where(i < 0, -i, np.where(i >= n, 2 * (n - 1) - i, i))
    return i


def sat_u8(v):
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def rgb2gray(img):
    """cv2 RGB2GRAY 8U fixed point."""
    r, g, b = (img[..., k].astype(np.int32) for k in range(3))
    return ((4899 * r + 9617 * g + 1868 * b + (1 << 13)) >> 14).astype(np.uint8)


# ---- Lab 8U: OpenCV's bit-exact fixed-point conversion (imgproc/src/color_lab.cpp, OpenCV >= 3.4:
#      initLabTabs, RGB2Lab_b, Lab2RGBinteger; every constant "presented through integers", table
#      entries from IEEE float32 (softfloat) / float64 (softdouble) arithmetic, cvRound = half-even) ----
LAB_SHIFT, GAMMA_SHIFT = 12, 3                     # lab_shift (= xyz_shift), gamma_shift
LAB_SHIFT2 = LAB_SHIFT + GAMMA_SHIFT               # 15
CBRT_TAB_B = 256 * 3 // 2 * (1 << GAMMA_SHIFT)     # LAB_CBRT_TAB_SIZE_B = 3072
INV_GAMMA_TAB = 1 << 12                            # INV_GAMMA_TAB_SIZE (inv_gamma_shift 12)
LAB_BASE = 1 << 14                                 # lab_base_shift 14
MIN_AB = -8145                                     # minABvalue
D65 = (0.950456, 1.0, 1.088754)
SRGB2XYZ = (0.412453, 0.357580, 0.180423, 0.212671, 0.715160, 0.072169, 0.019334, 0.119193, 0.950227)
XYZ2SRGB = (3.240479, -1.53715, -0.498535, -0.969256, 1.875991, 0.041556, 0.055648, -0.204043, 1.057311)
# softdouble gamma constants: 809/20000, 7827/2500000, 323/25, 12/5, 11/200
G_THR, G_INV_THR, G_LOW, G_POW, G_XS = 809 / 20000, 7827 / 2500000, 323 / 25, 12 / 5, 11 / 200


def _rne(v):
    """cvRound of a softfloat / softdouble: round half to even."""
    return np.rint(np.asarray(v, np.float64)).astype(np.int64)


def _apply_gamma(x):  # applyGamma(softfloat) in softdouble, result -> softfloat
    xd = x.astype(np.float64)
    return np.where(xd <= G_THR, xd / G_LOW, np.power((xd + G_XS) / (1.0 + G_XS), G_POW)).astype(f32)


def _apply_inv_gamma(x):
    xd = x.astype(np.float64)
    return np.where(xd <= G_INV_THR, xd * G_LOW, np.power(xd, 1.0 / G_POW) * (1.0 + G_XS) - G_XS).astype(f32)


def _trunc_div(a, b):  # C integer division (toward zero)
    return np.sign(a) * (np.abs(a) // b)


def lab_tables():
    """initLabTabs: sRGBGammaTab_b[256], LabCbrtTab_b[3072], LabToYF_b[256][2], sRGBInvGammaTab_b[4096],
    abToXZ_b[36864] and the RGB2Lab_b / Lab2RGBinteger coefficients (RGB channel order)."""
    i = np.arange(256)
    gamma = _rne(f32(255 * (1 << GAMMA_SHIFT)) * _apply_gamma(i.astype(f32) / f32(255)))
    lthresh, lscale, lbias = f32(216) / f32(24389), f32(841) / f32(108), f32(16) / f32(116)
    x = (f32(1) / (f32(255) * f32(1 << GAMMA_SHIFT))) * np.arange(CBRT_TAB_B).astype(f32)
    lin = (x.astype(np.float64) * np.float64(lscale) + np.float64(lbias)).astype(f32)   # mulAdd: one rounding
    cb = np.cbrt(x.astype(np.float64)).astype(f32)
    cbrt = _rne(f32(1 << LAB_SHIFT2) * np.where(x < lthresh, lin, cb).astype(f32))
    yf = np.zeros((256, 2), np.int64)
    for L in range(256):
        if L <= 20:
            y = _rne(f32(L * LAB_BASE * 20 * 9) / f32(17 * 29 * 29 * 29))
            ify = _rne(f32(LAB_BASE) * (f32(16) / f32(116) + f32(L * 5) / f32(3 * 17 * 29)))
        else:
            fy = f32(L * 100 * LAB_BASE) / f32(255 * 116) + f32(16 * LAB_BASE) / f32(116)
            ify = _rne(fy)
            y = _rne(fy * fy * fy / f32(LAB_BASE * LAB_BASE))
        yf[L] = (y, ify)
    invgamma = _rne(f32(255) * _apply_inv_gamma(f32(1) / f32(INV_GAMMA_TAB) * np.arange(INV_GAMMA_TAB).astype(f32)))
    v = np.arange(MIN_AB, LAB_BASE * 9 // 4 + MIN_AB, dtype=np.int64)
    abxz = np.where(v <= 3390, _trunc_div(v * 108, 841) - LAB_BASE * 16 // 116 * 108 // 841,
                    v * v // LAB_BASE * v // LAB_BASE)
    lshift = float(1 << LAB_SHIFT)
    c_fwd = np.array([_rne(lshift * SRGB2XYZ[r * 3 + j] / D65[r]) for r in range(3) for j in range(3)], np.int64)
    c_inv = np.array([_rne(lshift * XYZ2SRGB[r * 3 + j] * D65[j]) for r in range(3) for j in range(3)], np.int64)
    return dict(gamma=gamma, cbrt=cbrt, yf=yf, invgamma=invgamma, abxz=abxz, c_fwd=c_fwd, c_inv=c_inv)


_TABS = None


def _tabs():
    global _TABS
    if _TABS is None:
        _TABS = lab_tables()
    return _TABS


def _descale(x, n):  # CV_DESCALE
    return (x + (1 << (n - 1))) >> n


def rgb2lab(img):
    """cv2.cvtColor(img, COLOR_RGB2LAB) for uint8 (RGB2Lab_b)."""
    T = _tabs()
    R, G, B = (T["gamma"][img[..., k].astype(np.int64)] for k in range(3))
    C = T["c_fwd"]
    fX, fY, fZ = (T["cbrt"][_descale(R * C[3 * r] + G * C[3 * r + 1] + B * C[3 * r + 2], LAB_SHIFT)] for r in range(3))
    Lscale, Lshift = (116 * 255 + 50) // 100, -((16 * 255 * (1 << LAB_SHIFT2) + 50) // 100)
    L = _descale(Lscale * fY + Lshift, LAB_SHIFT2)
    a = _descale(500 * (fX - fY) + 128 * (1 << LAB_SHIFT2), LAB_SHIFT2)
    b = _descale(200 * (fY - fZ) + 128 * (1 << LAB_SHIFT2), LAB_SHIFT2)
    return np.stack([np.clip(t, 0, 255) for t in (L, a, b)], -1).astype(np.uint8)


def lab2rgb(lab):
    """cv2.cvtColor(lab, COLOR_LAB2RGB) for uint8 (Lab2RGB_b -> Lab2RGBinteger, the bit-exact path)."""
    T = _tabs()
    L, a, b = (lab[..., k].astype(np.int64) for k in range(3))
    y, ify = T["yf"][L, 0], T["yf"][L, 1]
    adiv = ((5 * a * 53687 + (1 << 7)) >> 13) - 128 * LAB_BASE // 500
    bdiv = ((b * 41943 + (1 << 4)) >> 9) - 128 * LAB_BASE // 200 + 1
    x = T["abxz"][ify + adiv - MIN_AB]
    z = T["abxz"][ify - bdiv - MIN_AB]
    C = T["c_inv"]
    shift = LAB_SHIFT + (14 - 12)  # lab_shift + (base_shift - inv_gamma_shift)
    out = []
    for r in range(3):
        v = _descale(C[3 * r] * x + C[3 * r + 1] * y + C[3 * r + 2] * z, shift)
        out.append(T["invgamma"][np.clip(v, 0, INV_GAMMA_TAB - 1)])
    return np.stack(out, -1).astype(np.uint8)


# ---- HSV 8U (H in [0, 180)) ----
def rgb2hsv(img):
    SH = 12
    r, g, b = (img[..., k].astype(np.int64) for k in range(3))
    v = np.maximum(r, np.maximum(g, b))
    vmin = np.minimum(r, np.minimum(g, b))
    diff = v - vmin
    vr = np.where(v == r, -1, 0)
    vg = np.where(v == g, -1, 0)
    idx = np.arange(256, dtype=np.float64)
    with np.errstate(divide="ignore"):
        sdiv = np.where(idx == 0, 0, np.rint((255 << SH) / idx)).astype(np.int64)
        hdiv = np.where(idx == 0, 0, np.rint((180 << SH) / (6.0 * idx))).astype(np.int64)
    s = (diff * sdiv[v] + (1 << (SH - 1))) >> SH
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))))
    h = (h * hdiv[diff] + (1 << (SH - 1))) >> SH
    h = h + np.where(h < 0, 180, 0)
    return h, s, v


def hsv2rgb(h8, s8, v8):
    h = np.asarray(h8).astype(f32) * (f32(6.0) / f32(180.0))
    s = np.asarray(s8).astype(f32) * (f32(1.0) / f32(255.0))
    v = np.asarray(v8).astype(f32) * (f32(1.0) / f32(255.0))
    h = np.where(h < 0, h + f32(6.0), h).astype(f32)
    h = np.where(h >= 6, h - f32(6.0), h).astype(f32)
    sector = np.floor(h).astype(np.int64)
    hf = (h - sector.astype(f32)).astype(f32)
    t0 = v
    t1 = v * (f32(1.0) - s)
    t2 = v * (f32(1.0) - s * hf)
    t3 = v * (f32(1.0) - s * (f32(1.0) - hf))
    tab = np.stack([t0, t1, t2, t3], 0)
    rsel = np.array([0, 2, 1, 1, 3, 0])[sector]
    gsel = np.array([3, 0, 0, 2, 1, 1])[sector]
    bsel = np.array([1, 1, 3, 0, 0, 2])[sector]
    pick = lambda sel: np.take_along_axis(tab, sel[None], 0)[0]
    r, g, b = pick(rsel), pick(gsel), pick(bsel)
    gray = s == 0
    r, g, b = (np.where(gray, v, c).astype(f32) for c in (r, g, b))
    return np.stack([sat_u8(r * f32(255.0)), sat_u8(g * f32(255.0)), sat_u8(b * f32(255.0))], -1)


def hsv_adjust(img, sat=None, hue=None, val=None):
    """dataset.py:261-264 (sat) and :297-300 (hue, val): fp32 arrays, astype(uint8)."""
    h, s, v = rgb2hsv(img)
    if sat is not None:
        s = np.clip(s.astype(f32) * f32(sat), 0, 255).astype(np.uint8).astype(np.int64)
    if hue is not None:
        h = ((h.astype(f32) + f32(hue)) % f32(180.0)).astype(np.uint8).astype(np.int64)
        v = np.clip(v.astype(f32) * f32(val), 0, 255).astype(np.uint8).astype(np.int64)
    return hsv2rgb(h, s, v)


# ---- CLAHE (OpenCV CLAHE_Impl) ----
def clahe(src, clip_limit, grid=(8, 8)):
    """src uint8 [h, w] -> uint8 [h, w]; grid = (tiles_x, tiles_y)."""
    h, w = src.shape
    tx_n, ty_n = grid
    # CLAHE_Impl::apply: a grid multiple on both axes -> size / grid; otherwise both axes are padded
    # by tiles - size % tiles (BORDER_REFLECT_101), so each tile is size // tiles + 1
    even = w % tx_n == 0 and h % ty_n == 0
    tw, th = w // tx_n + (0 if even else 1), h // ty_n + (0 if even else 1)
    ys = reflect101(np.arange(th * ty_n), h)
    xs = reflect101(np.arange(tw * tx_n), w)
    ext = src[ys][:, xs]
    area = tw * th
    clip = max(int(clip_limit * area / 256), 1) if clip_limit > 0 else 1 << 30
    scale = f32(255.0) / f32(area)
    luts = np.zeros((ty_n, tx_n, 256), np.uint8)
    for ty in range(ty_n):
        for tx in range(tx_n):
            hist = np.bincount(ext[ty * th:(ty + 1) * th, tx * tw:(tx + 1) * tw].ravel(), minlength=256)
            excess = int(np.maximum(hist - clip, 0).sum())
            hist = np.minimum(hist, clip)
            batch, residual = excess // 256, excess % 256
            hist = hist + batch
            if residual:
                step = max(256 // residual, 1)
                for i in range(0, 256, step):
                    if residual == 0:
                        break
                    hist[i] += 1
                    residual -= 1
            luts[ty, tx] = sat_u8(np.cumsum(hist).astype(f32) * scale)
    inv_tw, inv_th = f32(1.0) / f32(tw), f32(1.0) / f32(th)
    txf = np.arange(w).astype(f32) * inv_tw - f32(0.5)
    tyf = np.arange(h).astype(f32) * inv_th - f32(0.5)
    tx1, ty1 = np.floor(txf).astype(np.int64), np.floor(tyf).astype(np.int64)
    xa, ya = (txf - tx1.astype(f32)).astype(f32), (tyf - ty1.astype(f32)).astype(f32)
    tx2, ty2 = np.minimum(tx1 + 1, tx_n - 1), np.minimum(ty1 + 1, ty_n - 1)
    tx1, ty1 = np.maximum(tx1, 0), np.maximum(ty1, 0)
    v = src.astype(np.int64)
    Y1, Y2, X1, X2 = ty1[:, None], ty2[:, None], tx1[None, :], tx2[None, :]
    l11, l12 = luts[Y1, X1, v].astype(f32), luts[Y1, X2, v].astype(f32)
    l21, l22 = luts[Y2, X1, v].astype(f32), luts[Y2, X2, v].astype(f32)
    XA, YA = xa[None, :], ya[:, None]
    res = (l11 * (f32(1.0) - XA) + l12 * XA) * (f32(1.0) - YA) + (l21 * (f32(1.0) - XA) + l22 * XA) * YA
    return sat_u8(res.astype(f32))


def clahe_rgb(img, clip_limit, grid=(8, 8)):
    lab = rgb2lab(img)
    lab2 = lab.copy()
    lab2[..., 0] = clahe(lab[..., 0], clip_limit, grid)
    return lab2rgb(lab2)


# ---- filters (BORDER_REFLECT_101) ----
def _taps(img):
    h, w = img.shape[:2]
    ys, xs = np.arange(h), np.arange(w)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            yield dy, dx, img[reflect101(ys + dy, h)][:, reflect101(xs + dx, w)]


def filter3x3(img, k9):
    """cv2.filter2D(img, -1, k) with a 3x3 kernel: fp32 taps in row-major order."""
    k = np.asarray(k9, np.float64).astype(f32).reshape(3, 3)
    s = np.zeros(img.shape, f32)
    for dy, dx, t in _taps(img):
        s = s + k[dy + 1, dx + 1] * t.astype(f32)
    return sat_u8(s)


def sharpen(img, strength):
    return filter3x3(img, np.array([[-1, -1, -1], [-1, 9, -1], [-1, -1, -1]]) * strength)


def unsharp(img):
    """GaussianBlur(3x3, 1.0) 8U fixed point (70, 116, 70)/256 + addWeighted(1.3, -0.3)."""
    wk = (70, 116, 70)
    h, w = img.shape[:2]
    ys, xs = np.arange(h), np.arange(w)
    col = np.zeros(img.shape, np.int64)
    for dy in (-1, 0, 1):
        rows = img[reflect101(ys + dy, h)].astype(np.int64)
        row = sum(wk[dx + 1] * rows[:, reflect101(xs + dx, w)] for dx in (-1, 0, 1))
        col += wk[dy + 1] * row
    g = ((col + (1 << 15)) >> 16).astype(f32)
    return sat_u8(img.astype(f32) * f32(1.3) + g * f32(-0.3))


def edge_features(gray):
    """dataset.py:77-88: Sobel magnitude and |Laplacian| (CV_64F), normalised, 0.7 / 0.3."""
    t = {(dy, dx): v.astype(np.float64) for dy, dx, v in _taps(gray)}
    sx = (t[-1, 1] - t[-1, -1]) + 2 * (t[0, 1] - t[0, -1]) + (t[1, 1] - t[1, -1])
    sy = (t[1, -1] - t[-1, -1]) + 2 * (t[1, 0] - t[-1, 0]) + (t[1, 1] - t[-1, 1])
    mag = np.sqrt(sx ** 2 + sy ** 2)
    e = np.clip(mag / (mag.max() + 1e-6) * 255, 0, 255).astype(np.uint8)
    lap = np.abs(t[-1, 0] + t[0, -1] - 4 * t[0, 0] + t[0, 1] + t[1, 0])
    l = np.clip(lap / (lap.max() + 1e-6) * 255, 0, 255).astype(np.uint8)
    return (e.astype(f32) * f32(0.7) + l.astype(f32) * f32(0.3)).astype(np.uint8)


def cell_preprocess(image, live_mask, dead_mask):
    """dataset.py:58-131 with the masks already reduced to (h, w) unions (:93-100)."""
    image_clahe = clahe_rgb(image, 2.5)
    edges = edge_features(rgb2gray(image))
    edges_rgb = np.repeat(edges[..., None], 3, -1)
    if live_mask.sum() > 0:
        live_enh = np.clip(image_clahe.astype(f32) * f32(1.1), 0, 255).astype(np.uint8)
        image_clahe = np.where(live_mask[..., None] > 0, live_enh, image_clahe)
    if dead_mask.sum() > 0:
        dead_clahe = clahe(rgb2gray(image_clahe), 3.0)
        image_clahe = np.where(dead_mask[..., None] > 0, dead_clahe[..., None], image_clahe)
    iwe = np.clip(image_clahe.astype(f32) * f32(0.9) + edges_rgb.astype(f32) * f32(0.1), 0, 255).astype(np.uint8)
    fin = (iwe.astype(f32) * f32(0.85) + image.astype(f32) * f32(0.15)).astype(np.uint8)
    return unsharp(fin)


def chw_to_u8(x):
    """train_eval.py:367-377."""
    x = np.asarray(x, f32)
    hwc = x.transpose(1, 2, 0)
    v = hwc * f32(255.0) if x.max() <= 1.0 else hwc
    return v.astype(np.int64).astype(np.uint8)
