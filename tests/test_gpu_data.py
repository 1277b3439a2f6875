"""Device-side data path (datapath.hip) vs the reference loader's numpy expressions (oracle/data_ref.py).

Pixel ops, flips, ToTensor, cv2.resize INTER_LINEAR (OpenCV's fixed-point algorithm, restated) and
cv2.fillPoly (OpenCV 4.x's Bresenham outline + fixed-point scanline fill, restated in
oracle/data_ref.py fill_poly_u8) are bit-exact against the restatements; cv2 itself is absent, so
parity with cv2 is unpinned.
"""
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import data_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _img(seed, h=37, w=53):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("alpha,beta,sigma,g", [(1.13, 17.4, 6.0, 0.8), (0.61, -25.0, 9.5, 1.27), (1.3, 39.9, 3.1, 1.0)])
def test_pixel_augmentations_bit_exact(alpha, beta, sigma, g):
    from eunet import data, ops
    img = _img(1)
    noise = np.random.default_rng(2).normal(0, sigma, img.shape).astype(np.float32)
    ref = O.gamma(O.add_noise(O.contrast(O.brightness(img, alpha), beta), noise), g)
    d = torch.from_numpy(img).to(DEV)
    ops.augment_u8(d, alpha=alpha)
    ops.augment_u8(d, beta=beta)
    ops.augment_u8(d, noise=torch.from_numpy(noise).to(DEV))
    ops.augment_u8(d, lut=torch.from_numpy(data.gamma_lut(g)).to(DEV))
    assert np.array_equal(d.cpu().numpy(), ref)


@pytest.mark.parametrize("hi,wi,ho,wo,c", [
    (960, 1280, 480, 640, 3),   # exact 2x: cv2's INTER_AREA switch
    (768, 1024, 480, 640, 3),   # the reference's max_size = 640 downscale (scale 1.6)
    (375, 500, 352, 480, 3),    # /32 crop without a max_size scale (dataset.py:154-158)
    (100, 130, 96, 128, 3),
    (37, 53, 96, 160, 3),       # upscale: clamped borders, unclamped row coefficients
    (61, 29, 20, 37, 1),        # 1 channel, a row of 37 elements: vector body + scalar tail
    (50, 21, 13, 5, 3),         # 15 elements per row: 8-element step + scalar tail
])
def test_resize_u8_bit_exact(hi, wi, ho, wo, c):
    """cv2.resize(image, (wo, ho), INTER_LINEAR) for uint8 (dataset.py:151, 158) vs the restatement of
    OpenCV's fixed-point path (oracle/data_ref.py resize_linear_u8)."""
    from eunet import ops
    img = np.random.default_rng(hi * wi + c).integers(0, 256, (hi, wi, c), dtype=np.uint8)
    got = ops.resize_u8(torch.from_numpy(img).to(DEV), ho, wo).cpu().numpy()
    assert np.array_equal(got, O.resize_linear_u8(img, ho, wo))
    same = ops.resize_u8(torch.from_numpy(img).to(DEV), hi, wi).cpu().numpy()
    assert np.array_equal(same, img)


def test_flips_and_to_tensor_exact():
    from eunet import ops
    img = _img(3)
    d = torch.from_numpy(img).to(DEV)
    assert np.array_equal(ops.flip_u8(d, 1).cpu().numpy(), img[:, ::-1])
    assert np.array_equal(ops.flip_u8(d, 0).cpu().numpy(), img[::-1])
    m = torch.randint(0, 3, (37, 53), dtype=torch.int64)
    assert torch.equal(ops.flip_mask(m.to(DEV), 1).cpu(), m.flip(1))
    assert np.array_equal(ops.to_tensor(d).cpu().numpy(), O.to_tensor(img))


def test_rasterize_matches_rule():
    from eunet import ops
    rng = np.random.default_rng(4)
    polys, labels = [], []
    for i in range(12):
        c = rng.uniform(5, 60, 2)
        ang = np.sort(rng.uniform(0, 2 * np.pi, rng.integers(3, 12)))
        r = rng.uniform(2, 14, len(ang))
        pts = np.stack([c[0] + r * np.cos(ang), c[1] + r * np.sin(ang)], 1).astype(np.float32).astype(np.int32)
        polys.append(pts)
        labels.append(1 + (i % 2))
    polys.append(np.array([[10, 10], [20, 10], [20, 20], [10, 20]], np.int32))  # axis-aligned square
    labels.append(1)
    m = ops.rasterize_polygons(polys, labels, 64, 72, DEV).cpu().numpy()
    ref = O.rasterize(polys, labels, 64, 72)
    assert np.array_equal(m, ref)
    assert (m[10:21, 10:21] == 1).all()  # a square's outline and interior are filled


def _random_polys(rng, n, h, w):
    polys = []
    for i in range(n):
        c = rng.uniform(-10, [w + 10, h + 10])  # some straddle or leave the image
        ang = np.sort(rng.uniform(0, 2 * np.pi, rng.integers(1, 16)))  # 1-2 vertices: points / segments
        r = rng.uniform(0, 25, len(ang))
        pts = np.stack([c[0] + r * np.cos(ang), c[1] + r * np.sin(ang)], 1).astype(np.float32).astype(np.int32)
        polys.append(pts)
    return polys


@pytest.mark.parametrize("n,h,w", [(300, 61, 77), (40, 480, 640), (1, 17, 3)])
def test_rasterize_culling_matches_rule(n, h, w):  # noqa: C901
    """The bounding-box culled rasterisers (16x16 tiles with per-chunk polygon lists, > 256
    polygons = several LDS chunks; per-polygon instance masks in 4-byte runs, ragged tails, flips)
    against the oracle's per-pixel rule over every polygon."""
    from eunet import ops
    rng = np.random.default_rng(n + h)
    polys = _random_polys(rng, n, h, w)
    labels = [1 + int(v) for v in rng.integers(0, 2, n)]
    m = ops.rasterize_polygons(polys, labels, h, w, DEV).cpu().numpy()
    assert np.array_equal(m, O.rasterize(polys, labels, h, w))
    k = min(n, 24)
    refs = [(O.rasterize([polys[i]], [1], h, w) > 0).astype(np.uint8) for i in range(k)]
    for fh, fv in ((False, False), (True, False), (False, True), (True, True)):
        inst = ops.rasterize_instances(polys[:k], h, w, DEV, flip_h=fh, flip_v=fv).cpu().numpy()
        for i in range(k):
            ref = refs[i]
            if fh:
                ref = ref[:, ::-1]
            if fv:
                ref = ref[::-1]
            assert np.array_equal(inst[i], ref), (i, fh, fv)


def test_cell_dataset_end_to_end(tmp_path):
    """LabelMe directory -> device batches; same split, sizes and seeded augmentation decisions."""
    from PIL import Image
    from eunet.data import CellDataset, DataLoader, reference_sizes
    rng = np.random.default_rng(5)
    for i in range(10):
        im = rng.integers(0, 256, (100, 130, 3), dtype=np.uint8)
        Image.fromarray(im).save(tmp_path / f"img{i:02d}.jpg", quality=95)
        shapes = [{"label": "Live", "points": [[10, 10], [40, 12], [35, 40], [12, 35]]},
                  {"label": "dead", "points": [[60, 50], [90, 55], [70, 80]]},
                  {"label": "debris", "points": [[0, 0], [5, 0], [5, 5]]}]
        (tmp_path / f"img{i:02d}.json").write_text(json.dumps({"shapes": shapes}))
    ds = CellDataset(str(tmp_path), split="train", max_size=640, device=DEV)
    assert len(ds) == 7 and len(CellDataset(str(tmp_path), "val", device=DEV)) == 1
    random.seed(11)
    np.random.seed(11)
    item = ds[0]
    h, w = reference_sizes(100, 130, 640)
    assert item["image"].shape == (3, h, w) and item["semantic_mask"].shape == (h, w)
    assert item["instance_labels"] == [0, 1]
    assert set(torch.unique(item["semantic_mask"]).tolist()) <= {0, 1, 2}
    assert float(item["image"].min()) >= 0.0 and float(item["image"].max()) <= 1.0
    batch = next(iter(DataLoader(CellDataset(str(tmp_path), "val", device=DEV), batch_size=1)))
    assert batch["images"].shape == (1, 3, h, w) and batch["images"].is_cuda


def test_instance_masks_follow_the_flips(tmp_path):
    """'instance_masks' (dataset.py:313-321) are flipped with the image and the semantic mask
    (dataset.py:209-222): re-painting them in order (later instances win, :197-201) gives back the
    returned semantic mask exactly, flipped or not; an unflipped val item matches the direct fill."""
    from PIL import Image
    from eunet import ops
    from eunet.data import CellDataset, load_labelme, reference_sizes
    rng = np.random.default_rng(6)
    shapes = [{"label": "live", "points": [[10, 10], [40, 12], [35, 40], [12, 35]]},
              {"label": "dead", "points": [[60, 50], [95, 55], [70, 85]]},
              {"label": "live", "points": [[30, 30], [70, 28], [66, 66]]}]  # overlaps both
    for i in range(10):
        Image.fromarray(rng.integers(0, 256, (100, 130, 3), dtype=np.uint8)).save(tmp_path / f"i{i:02d}.jpg")
        (tmp_path / f"i{i:02d}.json").write_text(json.dumps({"shapes": shapes}))
    ds = CellDataset(str(tmp_path), split="train", max_size=640, device=DEV)
    h, w = reference_sizes(100, 130, 640)
    seen = set()
    for seed in range(8):
        random.seed(seed)
        np.random.seed(seed)
        r = random.Random(seed)
        flips = (r.random() > 0.5, r.random() > 0.5)  # the dataset's first two draws
        seen.add(flips)
        item = ds[0]
        inst = item["instance_masks"]
        assert len(inst) == 3 and all(m.dtype == torch.uint8 and m.shape == (h, w) for m in inst)
        sem = torch.zeros(h, w, dtype=torch.int64, device=DEV)
        for m, lab in zip(inst, item["instance_labels"]):
            sem[m > 0] = lab + 1
        assert torch.equal(sem, item["semantic_mask"]), (seed, flips)
        polys, labels, _ = load_labelme(str(tmp_path / "i00.json"), h / 100, w / 130)
        direct = ops.rasterize_instances(polys, h, w, DEV)
        want = direct
        if flips[0]:
            want = want.flip(2)
        if flips[1]:
            want = want.flip(1)
        assert torch.equal(torch.stack(inst), want), (seed, flips)
    assert len(seen) >= 3, seen  # flipped and unflipped cases were exercised
    val = CellDataset(str(tmp_path), split="val", max_size=640, device=DEV)[0]
    polys, labels, _ = load_labelme(str(tmp_path / "i07.json"), h / 100, w / 130)
    ref = O.rasterize(polys, [l + 1 for l in labels], h, w)
    assert np.array_equal(val["semantic_mask"].cpu().numpy(), ref)


def _write_cells(tmp_path, n=12, h=100, w=130, seed=7):
    from PIL import Image
    rng = np.random.default_rng(seed)
    for i in range(n):
        im = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        Image.fromarray(im).save(tmp_path / f"c{i:02d}.jpg", quality=95)
        k = int(rng.integers(1, 4))
        shapes = [{"label": "live", "points": [[10, 10], [40, 12], [35, 40], [12, 35]]},
                  {"label": "dead", "points": [[60, 50], [90, 55], [70, 80]]},
                  {"label": "live", "points": [[80, 10], [120, 14], [110, 40]]}][:k]
        if i % 4 == 3:  # dead-dominated (live ratio < 0.4) and cell-free (ratio 0.5) items
            shapes = [{"label": "dead", "points": [[5, 5], [120, 8], [115, 90], [8, 85]]},
                      {"label": "live", "points": [[50, 40], [60, 40], [55, 50]]}]
        if i % 6 == 5:
            shapes = []
        (tmp_path / f"c{i:02d}.json").write_text(json.dumps({"shapes": shapes}))


def test_sync_free_augmentation_matches_host_ratio(tmp_path):
    """The live ratio read on the device (eunet_augment_ratio_u8, the host drawing the same
    random.random() values random.uniform would) gives the same images as round 2's host read-back
    (dataset.py:225-257), for seeds that reach every ratio branch; the noise is the reference's
    numpy draw here (host_noise=True), so the whole item is compared bit for bit."""
    from eunet.data import CellDataset
    _write_cells(tmp_path)
    a = CellDataset(str(tmp_path), split="train", max_size=640, device=DEV, host_noise=True, host_ratio=True)
    b = CellDataset(str(tmp_path), split="train", max_size=640, device=DEV, host_noise=True, host_ratio=False)
    for seed in range(6):
        for idx in range(len(a)):
            out = []
            for ds in (a, b):
                random.seed(seed)
                np.random.seed(seed)
                out.append(ds[idx])
            assert torch.equal(out[0]["image"], out[1]["image"]), (seed, idx)
            assert torch.equal(out[0]["semantic_mask"], out[1]["semantic_mask"]), (seed, idx)


def test_prefetching_loader_same_batches(tmp_path):
    """DataLoader(workers=3, prefetch=2) -- decode in worker processes, device work of the next
    batches on a side stream, from the calling thread or from one producer thread -- yields the
    batches the plain loop yields for the same seeds (device noise included: its generator is
    reseeded from np.random in item order)."""
    from eunet.data import CellDataset, DataLoader
    _write_cells(tmp_path, n=14)
    ds = CellDataset(str(tmp_path), split="train", max_size=640, device=DEV)
    runs = []
    for workers, prefetch, thread in ((0, 0, False), (3, 2, False), (3, 2, True), (0, 1, True)):
        random.seed(3)
        np.random.seed(3)
        torch.manual_seed(3)
        loader = DataLoader(ds, batch_size=2, shuffle=True, workers=workers, prefetch=prefetch, thread=thread)
        got = [(b["images"].clone(), torch.stack([it["semantic_mask"] for it in b["batch_items"]]).clone())
               for b in loader]
        torch.cuda.synchronize()
        loader.close()
        runs.append(got)
    assert all(len(r) == 5 for r in runs)
    for other in runs[1:]:
        for (xa, ma), (xb, mb) in zip(runs[0], other):
            assert torch.equal(xa, xb) and torch.equal(ma, mb)


def test_threaded_loader_stops_early(tmp_path):
    """Abandoning a threaded loader's epoch mid-way (break) stops its producer thread."""
    import threading
    from eunet.data import CellDataset, DataLoader
    _write_cells(tmp_path, n=14)
    ds = CellDataset(str(tmp_path), split="train", max_size=640, device=DEV)
    loader = DataLoader(ds, batch_size=1, shuffle=False, prefetch=1, thread=True)
    it = iter(loader)
    next(it)
    it.close()  # GeneratorExit at the yield -> the finally block stops and joins the producer
    assert not any(t.name == "eunet-loader" and t.is_alive() for t in threading.enumerate())


def test_train_model_default_fast_path_is_exact(tmp_path):
    """train_model from a LabelMe directory with its cuda fast path -- decode workers (opt-in:
    loader_workers=3) + prefetch and the step replayed from HIP graphs (an odd train split, so every epoch ends on a 1-image batch,
    with an LR step per epoch) -- ends with the parameters of the plain in-loop eager run, bit for bit."""
    from eunet.models import EnhancedUNet
    from eunet.train_eval import train_model
    _write_cells(tmp_path, n=14)
    finals = []
    for graph, workers in ((True, 3), (False, None)):
        random.seed(5)
        np.random.seed(5)
        torch.manual_seed(5)
        model = EnhancedUNet(num_classes=3, in_channels=3, base_ch=16).to(DEV)
        train_model("enhanced_unet", data_dir=str(tmp_path), device=DEV, num_epochs=2, model=model,
                    save_dir=str(tmp_path / f"ck{int(graph)}"), verbose=False,
                    step_graph=None if graph else False, loader_workers=workers)
        finals.append({k: v.detach().clone() for k, v in model.state_dict().items()})
    for k in finals[0]:
        assert torch.equal(finals[0][k], finals[1][k]), k


def _shape_polys(h, w):
    """Concave, self-touching, self-intersecting, rectilinear, degenerate and clipped polygons."""
    rng = np.random.default_rng(17)
    polys = []
    for i in range(10):  # concave stars: alternating radii
        c = rng.uniform(8, [w - 8, h - 8])
        k = int(rng.integers(4, 9))
        ang = np.arange(2 * k) * np.pi / k + rng.uniform(0, 1)
        r = np.where(np.arange(2 * k) % 2 == 0, rng.uniform(8, 20), rng.uniform(2, 6))
        polys.append(np.stack([c[0] + r * np.cos(ang), c[1] + r * np.sin(ang)], 1).astype(np.float32).astype(np.int32))
    polys += [np.array(p, np.int32) for p in (
        [[5, 5], [25, 5], [25, 15], [15, 15], [15, 25], [5, 25]],            # L shape: horizontal / vertical edges
        [[30, 5], [50, 25], [50, 5], [30, 25]],                             # bow tie (self-intersecting)
        [[5, 30], [15, 30], [10, 40], [15, 50], [5, 50], [10, 40]],         # two triangles touching at a vertex
        [[20, 30], [40, 30], [40, 50], [30, 40], [20, 50]],                 # concave notch
        [[44, 44], [44, 44], [60, 44]],                                     # repeated vertex, horizontal segment
        [[3, 60], [3, 70]],                                                 # two points: vertical segment
        [[7, 7]],                                                           # one point
        [[-5, -5], [w + 4, 3], [w // 2, h + 6]],                             # clipped on every side
        [[w - 1, 0], [w, h // 2], [w - 3, h]],                               # x == w: the reference's scaled edge case
        [[0, h], [w // 3, h - 9], [w // 2, h]],                               # y == h
        [[-40, 20], [-10, 30], [-20, 60]],                                  # entirely left of the image
        [[10, 10], [11, 60], [12, 10]],                                     # thin steep sliver
        [[0, 20], [w - 1, 21], [0, 22]])]                                   # thin shallow sliver
    return polys


@pytest.mark.parametrize("h,w", [(64, 72), (63, 65)])
def test_rasterize_fillpoly_shapes_bit_exact(h, w):
    """cv2.fillPoly cases that separate it from a centre-sampled even-odd rule: Bresenham outline pixels
    on slanted edges, concave vertices, self-touching / self-intersecting outlines, horizontal and
    vertical edges, 1-2 point polygons and clipping at (and beyond) every image border -- semantic mask
    (last polygon wins) and the per-instance masks, bit-exact vs oracle/data_ref.py fill_poly_u8."""
    from eunet import ops
    polys = _shape_polys(h, w)
    labels = [1 + (i % 2) for i in range(len(polys))]
    m = ops.rasterize_polygons(polys, labels, h, w, DEV).cpu().numpy()
    assert np.array_equal(m, O.rasterize(polys, labels, h, w))
    inst = ops.rasterize_instances(polys, h, w, DEV).cpu().numpy()
    for i, p in enumerate(polys):
        assert np.array_equal(inst[i], O.fill_poly_u8(p, h, w)), (i, p.tolist())
