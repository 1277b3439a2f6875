"""cv2 image operations in HIP (imgproc.hip) vs the numpy restatement (oracle/imgproc_ref.py).

Parity unpinned against cv2 itself (absent from this image); against the restatement every
integer / fixed-point / per-operation fp32 step is bit-exact -- RGB<->Lab included since round 4
(cv2's bit-exact 8U tables: RGB2Lab_b / Lab2RGBinteger), checked over all 2^24 inputs -- and so
are the chains through Lab (cell preprocessing, the evaluator's CLAHE + sharpen).
"""
import numpy as np
import pytest
import torch

from oracle import imgproc_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
SIZES = [(37, 53), (64, 64), (256, 256), (8, 8), (100, 9), (64, 60), (60, 64)]


def _img(seed, h=37, w=53):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def _cells(seed, h, w):
    """A smooth image with bright blobs (cell-like), where CLAHE / edges do real work."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    base = 60 + 40 * np.sin(xx / 17.0) * np.cos(yy / 23.0)
    for _ in range(8):
        cy, cx, r = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(4, 14)
        base = base + 120 * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * r * r))
    rgb = np.stack([base * 0.9, base, base * 0.7], -1) + rng.normal(0, 6, (h, w, 3))
    return np.clip(rgb, 0, 255).astype(np.uint8)


def _d(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("h,w", SIZES)
def test_gray_and_hsv_bit_exact(h, w):
    from eunet import ops
    img = _img(h * 1000 + w, h, w)
    assert np.array_equal(ops.rgb2gray_u8(_d(img)).cpu().numpy(), O.rgb2gray(img))
    for sat in (0.0, 0.8, 1.0, 1.27):  # 0.0: fully desaturated (not read as 'unset')
        t = _d(img)
        ops.hsv_adjust_u8(t, sat=sat)
        assert np.array_equal(t.cpu().numpy(), O.hsv_adjust(img, sat=sat)), sat
    for hue, val in ((-9.7, 0.93), (0.0, 1.0), (9.99, 1.1), (-10.0, 1.05), (3.0, 0.0)):
        t = _d(img)
        ops.hsv_adjust_u8(t, hue=hue, val=val)
        assert np.array_equal(t.cpu().numpy(), O.hsv_adjust(img, hue=hue, val=val)), (hue, val)


@pytest.mark.parametrize("h,w", SIZES)
def test_filters_bit_exact(h, w):
    from eunet import ops
    img = _img(h + 7 * w, h, w)
    for s in (0.1, 0.15, 0.3):
        assert np.array_equal(ops.sharpen_u8(_d(img), s).cpu().numpy(), O.sharpen(img, s)), s
    k = np.random.default_rng(1).normal(0, 0.4, 9)
    assert np.array_equal(ops.filter3x3_u8(_d(img), k).cpu().numpy(), O.filter3x3(img, k))
    assert np.array_equal(ops.unsharp_u8(_d(img)).cpu().numpy(), O.unsharp(img))
    g = img[..., 1].copy()
    assert np.array_equal(ops.edge_features_u8(_d(g)).cpu().numpy(), O.edge_features(g))


@pytest.mark.parametrize("h,w", SIZES)
@pytest.mark.parametrize("clip", [0.0, 1.0, 2.5, 3.0, 40.0])
def test_clahe_gray_bit_exact(h, w, clip):
    """Integer histograms, clip + redistribution, fp32 LUT scale and bilinear blend; the
    padded-tile (BORDER_REFLECT_101) case when h, w are not multiples of the grid."""
    from eunet import ops
    g = _cells(h * 31 + w, h, w)[..., 1].copy()
    assert np.array_equal(ops.clahe_u8(_d(g), clip).cpu().numpy(), O.clahe(g, clip)), (h, w, clip)
    assert np.array_equal(ops.clahe_u8(_d(g), clip, grid=(3, 5)).cpu().numpy(), O.clahe(g, clip, (3, 5)))


def test_lab_conversions_exhaustive():
    """COLOR_RGB2LAB over every 8-bit RGB triple and COLOR_LAB2RGB over every 8-bit Lab triple."""
    from eunet import ops
    allc = np.arange(1 << 24, dtype=np.uint32)
    img = np.stack([(allc >> 16) & 255, (allc >> 8) & 255, allc & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
    assert np.array_equal(ops.rgb2lab_u8(_d(img)).cpu().numpy(), O.rgb2lab(img))
    assert np.array_equal(ops.lab2rgb_u8(_d(img)).cpu().numpy(), O.lab2rgb(img))


@pytest.mark.parametrize("h,w", [(64, 64), (37, 53), (256, 256)])
def test_clahe_on_lab_fused_lab2rgb(h, w):
    """CLAHE on L of a Lab image with the LAB2RGB fused in: bit-exact."""
    from eunet import ops
    lab = O.rgb2lab(_cells(h + w, h, w))
    want = lab.copy()
    want[..., 0] = O.clahe(lab[..., 0], 2.0)
    assert np.array_equal(ops.clahe_u8(_d(lab), 2.0, lab_to_rgb=True).cpu().numpy(), O.lab2rgb(want))


@pytest.mark.parametrize("h,w", [(64, 64), (96, 128), (256, 256)])
def test_cell_preprocess_chain(h, w):
    """dataset.py:58-131 end to end (Lab CLAHE, edge features, live / dead blends, unsharp): bit-exact."""
    from eunet import ops
    img = _cells(h * 5 + w, h, w)
    live = np.zeros((h, w), np.int64)
    live[h // 8:h // 2, w // 8:w // 2] = 1
    dead = np.zeros((h, w), np.int64)
    dead[h // 2:h - 4, w // 2:w - 3] = 1
    want = O.cell_preprocess(img, live, dead)
    got = ops.cell_preprocess_u8(_d(img), _d(live), _d(dead)).cpu().numpy()
    assert np.array_equal(got, want)
    # no dead instance: the dead-CLAHE branch is skipped
    want0 = O.cell_preprocess(img, live, np.zeros_like(dead))
    got0 = ops.cell_preprocess_u8(_d(img), _d(live), None).cpu().numpy()
    assert np.array_equal(got0, want0)


def test_cell_mix_and_live_boost_bit_exact():
    """The numpy blend steps of dataset.py:103-124 with identical inputs: bit-exact."""
    from eunet import _lib, ops
    h, w = 48, 64
    img, cl = _img(11, h, w), _img(12, h, w)
    edges = _img(13, h, w)[..., 0].copy()
    live = (np.random.default_rng(14).random((h, w)) > 0.5).astype(np.int64)
    dead = (np.random.default_rng(15).random((h, w)) > 0.6).astype(np.int64)
    dg = _img(16, h, w)[..., 2].copy()
    t, d_live, d_img, d_edges, d_dead, d_dg = _d(cl), _d(live), _d(img), _d(edges), _d(dead), _d(dg)  # kept alive
    _lib.call("eunet_live_boost_u8", ops._ptr(t), ops._ptr(d_live), h * w, ops._stream())
    boosted = np.where(live[..., None] > 0, np.clip(cl.astype(np.float32) * np.float32(1.1), 0, 255).astype(np.uint8), cl)
    assert np.array_equal(t.cpu().numpy(), boosted)
    out = torch.empty_like(t)
    _lib.call("eunet_cell_mix_u8", ops._ptr(d_img), ops._ptr(t), ops._ptr(d_edges), ops._ptr(d_dead),
              ops._ptr(d_dg), h * w, ops._ptr(out), ops._stream())
    c = np.where(dead[..., None] > 0, dg[..., None], boosted)
    f32 = np.float32
    iwe = np.clip(c.astype(f32) * f32(0.9) + edges[..., None].astype(f32) * f32(0.1), 0, 255).astype(np.uint8)
    want = (iwe.astype(f32) * f32(0.85) + img.astype(f32) * f32(0.15)).astype(np.uint8)
    assert np.array_equal(out.cpu().numpy(), want)


def test_evaluator_prepare_image_tensor():
    """train_eval.py:365-395: both input scalings, CLAHE(2.0) + sharpen(0.15), /255."""
    from eunet import ops
    from eunet.evaluator import reference_preprocess
    rng = np.random.default_rng(21)
    x = rng.random((3, 40, 56)).astype(np.float32)
    u8 = O.chw_to_u8(x)
    assert np.array_equal(ops.chw_to_u8(_d(x)).cpu().numpy(), u8)
    assert np.array_equal(ops.chw_to_u8(_d(x * 200)).cpu().numpy(), O.chw_to_u8(x * 200))
    got = reference_preprocess(_d(x)).cpu().numpy()
    want = (O.sharpen(O.clahe_rgb(u8, 2.0), 0.15).astype(np.float32) / np.float32(255.0)).transpose(2, 0, 1)
    assert got.shape == (3, 40, 56)
    assert np.array_equal(got, want)


def test_dataset_applies_preprocessing(tmp_path):
    """CellDataset items carry the cell-specific preprocessing (val split: no augmentation), and
    the cv2 augmentations run when their draws fire (train split, several seeds)."""
    import json
    import random
    from PIL import Image
    from eunet.data import CellDataset, load_labelme, reference_sizes
    rng = np.random.default_rng(22)
    shapes = [{"label": "live", "points": [[10, 10], [40, 12], [35, 40], [12, 35]]},
              {"label": "dead", "points": [[60, 50], [95, 55], [70, 85]]}]
    for i in range(10):
        Image.fromarray(_cells(100 + i, 96, 128)).save(tmp_path / f"c{i:02d}.png")
        (tmp_path / f"c{i:02d}.jpg").write_bytes((tmp_path / f"c{i:02d}.png").read_bytes())
        (tmp_path / f"c{i:02d}.json").write_text(json.dumps({"shapes": shapes}))
    val = CellDataset(str(tmp_path), split="val", max_size=640, device=DEV)
    item = val[0]
    img = np.array(Image.open(tmp_path / "c07.jpg").convert("RGB"))
    h, w = reference_sizes(96, 128, 640)
    polys, labels, _ = load_labelme(str(tmp_path / "c07.json"), h / 96, w / 128)
    from oracle import data_ref as D
    live = (D.rasterize([polys[0]], [1], h, w) > 0).astype(np.int64)
    dead = (D.rasterize([polys[1]], [1], h, w) > 0).astype(np.int64)
    want = O.cell_preprocess(img, live, dead).astype(np.float32) / np.float32(255.0)
    assert np.array_equal(item["image"].cpu().numpy().transpose(1, 2, 0), want)
    raw = CellDataset(str(tmp_path), split="val", max_size=640, device=DEV, cell_preprocess=False)[0]
    assert not torch.equal(raw["image"], item["image"])
    tr = CellDataset(str(tmp_path), split="train", max_size=640, device=DEV)
    for seed in range(6):
        random.seed(seed)
        np.random.seed(seed)
        t = tr[seed]["image"]
        assert t.shape == (3, h, w) and float(t.min()) >= 0 and float(t.max()) <= 1
