"""CPU checks of the cv2 restatement (oracle/imgproc_ref.py) -- parity unpinned (cv2 absent).

Pins what can be pinned without cv2: textbook colour values (white / black / primaries in
8U Lab and HSV as OpenCV defines the 8U ranges), round trips, CLAHE invariants (a flat
image stays flat, one-tile LUTs are monotone), filter identities.
"""
import numpy as np
import pytest

from oracle import imgproc_ref as O


def _img(seed, h=37, w=53):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def test_gray_weights():
    px = np.array([[[255, 255, 255], [0, 0, 0], [255, 0, 0], [0, 255, 0], [0, 0, 255]]], np.uint8)
    # 0.299 / 0.587 / 0.114 in 14-bit fixed point
    assert O.rgb2gray(px).tolist() == [[255, 0, 76, 150, 29]]


def test_lab_textbook_values():
    px = np.array([[[255, 255, 255], [0, 0, 0], [255, 0, 0], [0, 255, 0], [0, 0, 255]]], np.uint8)
    lab = O.rgb2lab(px)[0].tolist()
    assert lab[0] == [255, 128, 128] and lab[1] == [0, 128, 128]
    # L*, a*, b* of sRGB red / green / blue (53.2, 80.1, 67.2), (87.7, -86.2, 83.2), (32.3, 79.2, -107.9)
    assert lab[2] == [136, 208, 195] and lab[3] == [224, 42, 211] and lab[4] == [82, 207, 20]


def test_lab_round_trip():
    img = _img(1, 64, 64)
    back = O.lab2rgb(O.rgb2lab(img))
    # 8-bit Lab quantises L to 100/255 and a, b to 1: a few levels on dark saturated colours
    assert np.abs(back.astype(int) - img).max() <= 24  # near-zero channels: steep sRGB curve
    assert np.abs(back.astype(int) - img).mean() < 1.0
    for v in (0, 255):  # black and white survive exactly
        px = np.full((1, 1, 3), v, np.uint8)
        assert np.array_equal(O.lab2rgb(O.rgb2lab(px)), px)


def test_lab_tables_match_opencv_source_comments_and_the_library():
    """The fixed-point Lab tables (color_lab.cpp initLabTabs): the value ranges the OpenCV source states
    in its comments (LabToYF_b: 0 <= y <= BASE, 2260 <= ify <= BASE; abToXZ_b: -1335 <= v <= 88231), the
    D65 white point's raw softdouble bits, and the host tables libeunet_hip builds for its kernels
    (eunet_lab_tables: no GPU needed) equal the numpy construction entry for entry."""
    import ctypes
    import struct
    T = O.lab_tables()
    assert T["yf"][:, 0].min() == 0 and T["yf"][:, 0].max() == 1 << 14
    assert T["yf"][:, 1].min() == 2260 and T["yf"][:, 1].max() == 1 << 14
    assert T["abxz"].min() == -1335 and T["abxz"].max() == 88231
    raw = [struct.unpack("<Q", struct.pack("<d", v))[0] for v in (O.D65[0], O.D65[2])]
    assert raw == [0x3fee6a22b3892ee8, 0x3ff16b8950763a19]
    from eunet import _lib
    lib = _lib.load()
    buf = ctypes.create_string_buffer(2 * (256 + 3072 + 512 + 4096) + 4 * 18)
    assert lib.eunet_lab_tables(buf, len(buf)) == 0
    u16 = np.frombuffer(buf.raw, np.uint16, 256 + 3072 + 512 + 4096)
    i32 = np.frombuffer(buf.raw, np.int32, 18, offset=2 * u16.size)
    o = 0
    for key, n in (("gamma", 256), ("cbrt", 3072), ("yf", 512), ("invgamma", 4096)):
        assert np.array_equal(u16[o:o + n], T[key].reshape(-1)), key
        o += n
    assert np.array_equal(i32[:9], T["c_fwd"]) and np.array_equal(i32[9:], T["c_inv"])


def test_hsv_textbook_values_and_round_trip():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [128, 64, 0]]], np.uint8)
    h, s, v = O.rgb2hsv(px)
    assert h.tolist() == [[0, 60, 120, 0, 15]] and s.tolist() == [[255, 255, 255, 0, 255]]
    assert v.tolist() == [[255, 255, 255, 255, 128]]
    img = _img(2, 48, 48)
    back = O.hsv2rgb(*O.rgb2hsv(img))
    assert np.abs(back.astype(int) - img).max() <= 6  # H quantised to 2 degrees


def test_hsv_adjust_identity_and_hue_wrap():
    img = _img(3)
    assert np.array_equal(O.hsv_adjust(img, sat=1.0), O.hsv2rgb(*O.rgb2hsv(img)))
    h0, _, _ = O.rgb2hsv(img)
    h1, _, _ = O.rgb2hsv(O.hsv_adjust(img, hue=-10.0, val=1.0))
    assert h1.min() >= 0 and h1.max() < 180


@pytest.mark.parametrize("h,w", [(64, 64), (37, 53), (8, 8), (100, 9)])
def test_clahe_invariants(h, w):
    flat = np.full((h, w), 97, np.uint8)
    out = O.clahe(flat, 2.0)
    assert (out == out[0, 0]).all()
    g = np.random.default_rng(4).integers(0, 256, (h, w)).astype(np.uint8)
    a, b = O.clahe(g, 2.0), O.clahe(g, 0.0)
    assert a.shape == g.shape and b.shape == g.shape
    # one tile: the transfer function (a clipped CDF) is monotone
    ramp = np.tile(np.arange(256, dtype=np.uint8), (16, 1))[:, :w if w <= 256 else 256]
    r = O.clahe(ramp, 3.0, (1, 1))
    assert (np.diff(r[0].astype(int)) >= 0).all()


def test_clahe_tile_rule_one_axis_uneven():
    """OpenCV's CLAHE_Impl::apply pads BOTH axes by tiles - size % tiles as soon as one axis is
    not a multiple of the grid: with h = 64 (divisible by 8) and w = 60 the tile is 9 x 8,
    not 8 x 8, so the LUTs cover rows reflected past the bottom edge.  Pinned through the
    result on an image whose histogram differs between rows 0..63 and the reflected rows."""
    h, w = 64, 60
    g = np.zeros((h, w), np.uint8)
    g[:, :] = (np.arange(w)[None, :] * 4).astype(np.uint8)
    g[-8:, :] = 250  # bottom band: the reflected padding rows 64..71 repeat rows 62..55
    got = O.clahe(g, 2.0)
    # restate the padded-tile computation directly: tile 9 x 8 -> area 72, clip int(2.0 * 72 / 256) = 0 -> 1
    ext = g[O.reflect101(np.arange(8 * 9), h)][:, O.reflect101(np.arange(8 * 8), w)]
    hist = np.bincount(ext[:9, :8].ravel(), minlength=256)
    clip = 1
    excess = int(np.maximum(hist - clip, 0).sum())
    hist = np.minimum(hist, clip) + excess // 256
    res = excess % 256
    if res:
        for i in range(0, 256, max(256 // res, 1)):
            if res == 0:
                break
            hist[i] += 1
            res -= 1
    lut0 = O.sat_u8(np.cumsum(hist).astype(np.float32) * (np.float32(255.0) / np.float32(72)))
    # pixel (0, 0) sits in the top-left quarter of tile (0, 0): its value is tile (0, 0)'s LUT
    assert got[0, 0] == lut0[g[0, 0]]
    even = O.clahe(g[:, :56].copy(), 2.0)  # 64 x 56: both multiples of 8 -> 8 x 7 tiles, no padding
    assert even.shape == (64, 56)


def test_filters_identities():
    img = _img(5)
    ident = [0, 0, 0, 0, 1, 0, 0, 0, 0]
    assert np.array_equal(O.filter3x3(img, ident), img)
    flat = np.full((20, 30, 3), 77, np.uint8)
    # the reference's kernel sums to 1 * strength, so on a flat image it scales brightness:
    # 77 * 0.15 = 11.55 -> 12 (train_eval.py:388-391 darkens as written)
    assert (O.sharpen(flat, 0.15) == 12).all()
    assert np.array_equal(O.unsharp(flat), flat)
    assert (O.edge_features(flat[..., 0]) == 0).all()


def test_cell_preprocess_shapes_and_masks():
    img = _img(6, 64, 80)
    live = np.zeros((64, 80), np.int64)
    live[10:30, 10:40] = 1
    dead = np.zeros((64, 80), np.int64)
    dead[40:60, 50:75] = 1
    out = O.cell_preprocess(img, live, dead)
    assert out.shape == img.shape and out.dtype == np.uint8
    none = O.cell_preprocess(img, np.zeros_like(live), np.zeros_like(dead))
    assert not np.array_equal(out[10:30, 10:40], none[10:30, 10:40])
    assert np.array_equal(out[0:5, 0:5], none[0:5, 0:5])  # far from both masks nothing changes


def test_chw_to_u8_branches():
    x = np.random.default_rng(7).random((3, 5, 6)).astype(np.float32)
    assert np.array_equal(O.chw_to_u8(x), (x.transpose(1, 2, 0) * np.float32(255)).astype(np.uint8))
    y = x * 200
    assert np.array_equal(O.chw_to_u8(y), y.transpose(1, 2, 0).astype(np.uint8))
