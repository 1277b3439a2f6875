"""Pin the CPU oracle (oracle/eunet_ref.py) against reference-generated fixtures.

The fixtures in tests/golden were produced by running the reference itself
(tests/golden/gen_golden.py); this test needs neither the reference nor a GPU.
"""
import os

import numpy as np
import pytest
import torch

from oracle import eunet_ref as R
from oracle.weights import uniform01
from oracle import data_ref as O  # noqa: E402


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("fname,K", [("fwd_c3k3.npz", 3), ("fwd_c3k2.npz", 2)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_forward_matches_reference(golden_dir, fname, K, dtype):
    g = _load(golden_dir, fname)
    S = R.formula_weights(64, 3, K, dtype=dtype)
    x = torch.from_numpy(g["x"]).to(dtype)
    with torch.no_grad():
        out = R.forward(S, x, training=True)
    tol = 1e-5 if dtype == torch.float32 else 2e-5
    assert _rel(out.numpy(), g["out_train"]) < tol
    for k in g.files:
        if k.startswith("bn:"):
            assert _rel(S[k[3:]].numpy(), g[k]) < 1e-4, k
    with torch.no_grad():
        out_e = R.forward(S, x, training=False)
    assert _rel(out_e.numpy(), g["out_eval"]) < tol


def test_in_ch1_equivalence(golden_dir):
    """1-ch input == reference 3-ch model on (x,0,0) with weight[:, :1]."""
    g = _load(golden_dir, "in1_equiv.npz")
    S3 = R.formula_weights(64, 3, 2, dtype=torch.float64)
    S1 = dict(S3)
    S1["model.enc1.0.weight"] = S3["model.enc1.0.weight"][:, :1].contiguous()
    with torch.no_grad():
        out = R.forward(S1, torch.from_numpy(g["x1"]).double(), training=True)
    assert _rel(out.numpy(), g["out_train"]) < 2e-5


@pytest.mark.parametrize("fname", ["loss_k3.npz", "loss_k2.npz"])
def test_loss_matches_reference(golden_dir, fname):
    g = _load(golden_dir, fname)
    logits = torch.from_numpy(g["logits"]).double().requires_grad_(True)
    target = torch.from_numpy(g["target"])
    total, parts = R.combined_loss(logits, target, parts=True)
    total.backward()
    assert abs(total.item() - float(g["total"])) < 1e-5 * abs(float(g["total"]))
    for k in ("focal", "dice", "tversky"):
        assert abs(parts[k].item() - float(g[k])) <= 1e-5 * max(abs(float(g[k])), 1e-6), k
    assert _rel(logits.grad.numpy(), g["grad"]) < 1e-4


FOCAL_CFGS = [  # tests/golden/gen_golden.py LOSS_API_FOCAL
    ([1.0, 8.0, 5.0], 5.0, None, [1.0, 20.0, 10.0]),
    (None, 2.0, None, None),
    (0.25, 2.0, 1, None),
    ([1.0, 2.0], 3.0, None, [1.0, 4.0, 2.0]),
    ([0.5, 1.0, 2.0], 1.5, 255, [2.0, 1.0, 3.0]),
]


def test_loss_api_restatements_match_reference(golden_dir):
    """Generalised FocalLoss / dice_loss / tversky_loss restatements vs the reference modules."""
    g = _load(golden_dir, "loss_api.npz")
    x0 = torch.from_numpy(g["x"]).double()
    t, t_ign = torch.from_numpy(g["t"]), torch.from_numpy(g["t_ign"])

    def check(name, fn, tt):
        x = x0.clone().requires_grad_(True)
        v = fn(x, tt)
        v.backward()
        assert abs(v.item() - float(g[f"{name}_val"])) < 1e-5 * abs(float(g[f"{name}_val"])), name
        assert _rel(x.grad.numpy(), g[f"{name}_grad"]) < 1e-4, name

    for i, (a, gm, ii, cw) in enumerate(FOCAL_CFGS):
        w = None if cw is None else torch.tensor(cw, dtype=torch.float64)
        check(f"focal{i}", lambda x, tt: R.focal_loss(x, tt, a, gm, ii, w), t_ign if ii == 255 else t)
    check("ce", lambda x, tt: torch.nn.functional.cross_entropy(x, tt, weight=torch.tensor(R.CE_WEIGHT).double()), t)
    for nc in (2, 3):
        check(f"dice_nc{nc}", lambda x, tt: R.dice_loss(x, tt, nc), t)
        check(f"tversky_nc{nc}", lambda x, tt: R.tversky_loss(x, tt, nc), t)
    check("tversky_a05", lambda x, tt: R.tversky_loss(x, tt, 3, 0.5), t)


@pytest.mark.parametrize("fname", ["step_c3k3.npz", "step_pad_c3k3.npz"])
def test_train_step_matches_reference(golden_dir, fname):
    """One train_epoch step; step_pad_c3k3 is a 40x56 batch, so the reference's reflect pad of the
    images and zero pad of the masks to /32 (train_eval.py:248-253, 276-296) are in the fixture."""
    g = _load(golden_dir, fname)
    S = R.formula_weights(64, 3, 3, dtype=torch.float32)
    tr = R.OracleTrainer(S, total_epochs=50)
    lr = tr.epoch_lr_step(0)
    assert abs(lr - float(g["lr"])) < 1e-12
    loss = tr.step(torch.from_numpy(g["x"]), torch.from_numpy(g["m"]))
    assert abs(loss - float(g["loss"])) < 1e-5 * abs(float(g["loss"]))
    for k in tr.keys:
        grad = S[k].grad.detach().numpy().astype(np.float64)
        post = S[k].detach().numpy().astype(np.float64)
        for tag, arr in (("grad", grad), ("post", post)):
            if f"{tag}:{k}" in g.files:
                ref = g[f"{tag}:{k}"]
                # conv biases feeding a BatchNorm have an exactly-zero true gradient:
                # their reference values are rounding noise, hence the absolute floor
                # (and AdamW turns that noise into steps of up to ~lr after one update)
                scale = max(np.abs(ref).max(), 1e-12)
                floor = 1e-6
                if tag == "post" and _feeds_bn(k):
                    floor = 2.0 * lr
                assert np.abs(arr.reshape(ref.shape) - ref).max() < 2e-3 * scale + floor, (tag, k)
            else:
                flat = arr.reshape(-1)
                ref_norm = float(g[f"{tag}_norm:{k}"])
                assert abs(np.sqrt((flat ** 2).sum()) - ref_norm) < 1e-3 * ref_norm, (tag, k)
                idx = g[f"{tag}_idx:{k}"]
                ref_v = g[f"{tag}_val:{k}"]
                assert np.abs(flat[idx] - ref_v).max() < 2e-3 * max(np.abs(ref_v).max(), 1e-12), (tag, k)
    for k in S:
        if k.endswith("running_mean") or k.endswith("running_var"):
            ref = g.get(f"post:{k}")
            if ref is not None:
                assert _rel(S[k].numpy(), ref) < 1e-4, k


def _feeds_bn(key):
    return key.endswith((".0.bias", ".3.bias")) and (key.startswith("model.enc") or key.startswith(
        "model.dec") or key.startswith("enhance.0")) and not key.startswith("enhance.3")


def test_lr_trajectory_matches_reference(golden_dir):
    g = _load(golden_dir, "lr_traj.npz")
    for E in (6, 50):
        np.testing.assert_allclose(R.lr_trajectory(E), g[f"E{E}"], rtol=1e-12, atol=1e-15)


def test_bilinear_half_resize_is_avgpool():
    x = torch.randn(2, 3, 16, 12, dtype=torch.float64)
    assert R.avgpool_equals_resize(x) < 1e-12


def test_flops_formula():
    assert R.flops_per_pixel(64, 3, 3) == 3928320.0
    assert R.flops_per_pixel(64, 1, 2) == 3906816.0


def test_formula_weights_deterministic():
    a = uniform01("k", 10)
    b = uniform01("k", 10)
    assert np.array_equal(a, b) and (a >= 0).all() and (a < 1).all()
    spec = R.state_spec(64, 3, 3)
    assert len(spec) == 109


# ---- evaluation path (oracle/evalpath_ref.py) vs the reference's own outputs ----------
def test_semantic_metrics_match_reference(golden_dir):
    from oracle import evalpath_ref as E
    g = _load(golden_dir, "metrics.npz")
    for i in range(int(g["n"])):
        m = E.calculate_semantic_metrics(g[f"pred{i}"], g[f"gt{i}"])
        for k, v in zip(g[f"keys{i}"], g[f"vals{i}"]):
            assert m[str(k)] == v, (i, k)
        assert E.calculate_iou(g[f"pred{i}"], g[f"gt{i}"]) == g[f"iou{i}"]
        assert E.calculate_dice(g[f"pred{i}"], g[f"gt{i}"]) == g[f"dice{i}"]


def test_probs_to_mask_matches_reference_all_regimes(golden_dir):
    from oracle import evalpath_ref as E
    g = _load(golden_dir, "probs_mask.npz")
    regimes = set()
    for i in range(int(g["n"])):
        assert np.array_equal(E.convert_probs_to_mask(g[f"probs{i}"]), g[f"mask{i}"]), i
        lr, dr = E.mask_regime(g[f"probs{i}"])
        regimes.add(("live" if lr > 0.5 else "-", 3 if dr > 0.4 else 2 if dr > 0.25 else 1 if dr > 0.15 else 0))
    # every refinement branch of train_eval.py:533-563 is reached by some case
    assert {r[1] for r in regimes} >= {1, 2, 3} and any(r[0] == "live" for r in regimes)


def test_tta_matches_reference(golden_dir):
    from oracle import evalpath_ref as E
    g = _load(golden_dir, "tta_c3k3.npz")
    S = R.formula_weights(64, 3, 3, dtype=torch.float32)
    for k in g.files:
        if k.startswith("bn:"):
            S[k[3:]] = torch.from_numpy(g[k])
    img = torch.from_numpy(g["img"])
    with torch.no_grad():
        assert _rel(E.run_model_single(S, img).numpy(), g["single"]) < 1e-5
        p = E.run_tta(S, img)
    assert _rel(p.numpy(), g["tta"]) < 1e-5
    assert np.array_equal(E.convert_probs_to_mask(g["tta"]), g["mask"])


# ---- dual-branch (SMP-path) EnhancedUNet: oracle/dual_ref.py vs the reference module ----
def _dual_setup(golden_dir):
    from oracle import dual_ref as D
    g = _load(golden_dir, "dual_c3k3.npz")
    S = D.dual_formula_weights(64, 3, 3, dtype=torch.float32)
    masks = (torch.from_numpy(g["drop0"]), torch.from_numpy(g["drop1"]))
    return D, g, S, masks


def test_dual_forward_matches_reference(golden_dir):
    D, g, S, masks = _dual_setup(golden_dir)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        fused, aux = D.dual_forward(S, x, training=True, drop_masks=masks)
    assert _rel(fused.numpy(), g["out_train"]) < 1e-5
    assert _rel(aux["unetpp"].numpy(), g["aux_unetpp"]) < 1e-5
    assert _rel(aux["deeplab"].numpy(), g["aux_deeplab"]) < 1e-5
    for k in g.files:
        if k.startswith("bn:"):
            assert _rel(S[k[3:]].numpy(), g[k]) < 1e-4, k
    with torch.no_grad():
        out_e, _ = D.dual_forward(S, x, training=False)
    assert _rel(out_e.numpy(), g["out_eval"]) < 1e-5


def test_dual_train_step_matches_reference(golden_dir):
    D, g, S, masks = _dual_setup(golden_dir)
    tr = D.DualOracleTrainer(S, total_epochs=50, drop_masks=masks)
    lr = tr.epoch_lr_step(0)
    loss = tr.step(torch.from_numpy(g["x"]), torch.from_numpy(g["m"]))
    assert abs(loss - float(g["loss"])) < 1e-5 * abs(float(g["loss"]))
    for k in tr.keys:
        for tag, arr in (("grad", S[k].grad.detach().numpy().astype(np.float64)),
                         ("post", S[k].detach().numpy().astype(np.float64))):
            if f"{tag}:{k}" in g.files:
                ref = g[f"{tag}:{k}"]
                floor = 2.0 * lr if (tag == "post" and k.endswith((".0.bias", ".3.bias"))) else 1e-6
                assert np.abs(arr.reshape(ref.shape) - ref).max() < 2e-3 * max(np.abs(ref).max(), 1e-12) + floor, \
                    (tag, k)
            else:
                flat = arr.reshape(-1)
                ref_norm = float(g[f"{tag}_norm:{k}"])
                assert abs(np.sqrt((flat ** 2).sum()) - ref_norm) < 1e-3 * ref_norm, (tag, k)


def test_data_oracle_rules():
    """oracle/data_ref.py: the reference's numpy pixel lines and cv2.fillPoly's square."""
    from oracle import data_ref as O
    img = np.arange(256, dtype=np.uint8).reshape(16, 16, 1)
    assert O.brightness(img, 2.0)[15, 15, 0] == 255 and O.brightness(img, 0.5)[0, 3, 0] == 1
    assert O.contrast(img, -10.0)[0, 5, 0] == 0
    assert (O.gamma(img, 1.0) == img).all()
    sq = O.rasterize([np.array([[2, 2], [5, 2], [5, 5], [2, 5]])], [2], 8, 8)
    assert sq.sum() == 2 * 16 and (sq[2:6, 2:6] == 2).all()


def test_branch_pinned_oracle_at_its_own_branches_is_the_oracle():
    """The branch-pinned forward (eunet_ref._relu / _pool; the GPU gradient tests feed it the kernels'
    ReLU masks and max-pool argmax, tests/_pins.py) evaluated on the oracle's OWN branch configuration
    is the plain oracle bit for bit -- logits, loss and every gradient -- and a pin is really used
    (one flipped mask element changes the logits).  The pins are formed with the same helpers the GPU
    tests use (_pins.relu_mask / pool_argmax on NHWC tensors with an identity affine)."""
    import _pins
    x = torch.rand(2, 1, 32, 32, generator=torch.Generator().manual_seed(1))
    msk = (x[:, 0] > 0.5).long()

    def run(pins=None, rec=None):
        S = R.formula_weights(16, 1, 2, dtype=torch.float32)
        for k in S:
            if S[k].is_floating_point() and "running" not in k:
                S[k].requires_grad_(True)
        d2, _ = R.trunk(S, x, True, pins, record=rec)
        u = torch.nn.functional.conv2d(R._up2(d2), S["model.dec1.weight"], S["model.dec1.bias"])
        loss = R.batch_loss(u, msk)
        loss.backward()
        return u.detach(), loss.detach(), {k: v.grad for k, v in S.items() if getattr(v, "grad", None) is not None}

    rec = {}
    u0, l0, g0 = run(rec=rec)
    nhwc = lambda t: t.permute(0, 2, 3, 1)  # noqa: E731
    one, zero = torch.ones(1), torch.zeros(1)
    pins = {k: _pins.relu_mask(nhwc(v), one, zero) for k, v in rec.items()}
    for i, nm in enumerate(_pins.POOLED, 1):
        pins[f"pool{i}"] = _pins.pool_argmax(nhwc(rec[nm + ".4"]), one, zero, torch.float32)
    u1, l1, g1 = run(pins)
    assert torch.equal(u0, u1) and torch.equal(l0, l1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
    flip = dict(pins)
    m = flip["dec2.4"].clone()
    m.view(-1)[int(m.view(-1).nonzero()[0])] = False
    flip["dec2.4"] = m
    assert not torch.equal(run(flip)[0], u0)


def test_pin_audit_accepts_rounding_and_catches_branch_bugs():
    """tests/_pins.audit: pins taken from an fp32 run of the oracle (an implementation whose branches
    differ from fp64 only by rounding) pass the fp32 audit against the fp64 oracle's own branches; pins
    with one ReLU mask flipped far from its kink, with a 2x2 pool index moved off a clear maximum, or
    formed with the BN shift of the wrong channel are rejected."""
    import _pins
    x = torch.rand(2, 1, 64, 64, generator=torch.Generator().manual_seed(3))
    nhwc = lambda t: t.permute(0, 2, 3, 1)  # noqa: E731
    one, zero = torch.ones(1), torch.zeros(1)

    def pins_of(S, xx):
        rec = {}
        with torch.no_grad():
            R.trunk(S, xx, True, record=rec)
        pins = {k: _pins.relu_mask(nhwc(v), one, zero) for k, v in rec.items()}
        for i, nm in enumerate(_pins.POOLED, 1):
            pins[f"pool{i}"] = _pins.pool_argmax(nhwc(rec[nm + ".4"]), one, zero, torch.float32)
        return pins, rec

    p32, rec32 = pins_of(R.formula_weights(16, 1, 2, dtype=torch.float32), x)
    rec64 = {}
    with torch.no_grad():
        R.trunk(R.formula_weights(16, 1, 2), x.double(), True, pins=p32, record=rec64)
    out = _pins.audit(p32, rec64, torch.float32, label="fp32 oracle vs fp64")
    assert set(out) == set(p32)

    h = rec64["enc2.1"]
    i = int(h.abs().argmax())  # the element farthest from its kink
    bad = dict(p32)
    m = bad["enc2.1"].clone()
    m.view(-1)[i] = ~m.view(-1)[i]
    bad["enc2.1"] = m
    with pytest.raises(AssertionError):
        _pins.audit(bad, rec64, torch.float32)

    v = rec64["enc1.4"].clamp_min(0)
    B, C, H, W = v.shape
    w = v.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    gap = w.max(-1).values - w.min(-1).values
    j = int(gap.argmax())
    bad = dict(p32)
    pl = bad["pool1"].clone()
    pl.view(-1)[j] = int(w.reshape(-1, 4)[j].argmin())
    bad["pool1"] = pl
    with pytest.raises(AssertionError):
        _pins.audit(bad, rec64, torch.float32)

    # a wrong shift channel: the masks of enc3.4 formed with the channels' shifts rolled by one
    hh = nhwc(rec32["enc3.4"])
    shift = torch.linspace(-0.5, 0.5, hh.shape[-1])
    bad = dict(p32)
    bad["enc3.4"] = _pins.relu_mask(hh - shift + shift.roll(1), one, zero)
    with pytest.raises(AssertionError):
        _pins.audit(bad, rec64, torch.float32)


def _fillpoly_per_pixel(pts, h, w):
    """The HIP kernels' per-pixel statement of cv2.fillPoly (csrc/datapath.hip cv_fillpoly_covers):
    closed-form Bresenham membership per edge + the span count over the row's active edges.  An
    independent formulation of the same algorithm, checked against the literal scanline restatement."""
    def cdiv(a, b):
        q = abs(a) // abs(b)
        return q if (a >= 0) == (b >= 0) else -q
    P = [(int(a), int(b)) for a, b in pts]
    out = np.zeros((h, w), np.uint8)
    for y in range(h):
        for x in range(w):
            on, clt, cle = False, 0, 0
            for k in range(len(P)):
                (X0, Y0), (X1, Y1) = P[k - 1], P[k]
                inimg = 0 <= X0 < w and 0 <= X1 < w and 0 <= Y0 < h and 0 <= Y1 < h
                vis, (cx0, cy0), (cx1, cy1) = (True, (X0, Y0), (X1, Y1)) if inimg else \
                    O.clip_line(w, h, (X0, Y0), (X1, Y1))
                if vis:
                    (lx1, ly1), (lx2, ly2) = sorted([(cx0, cy0), (cx1, cy1)], key=lambda q: q[0]) \
                        if cx1 < cx0 else ((cx0, cy0), (cx1, cy1))
                    ddx, ddy = lx2 - lx1, ly2 - ly1
                    ady = abs(ddy)
                    if ady > ddx:
                        i = ly1 - y if ddy < 0 else y - ly1
                        on |= 0 <= i <= ady and x == lx1 + (2 * ddx * i + ady - 1) // (2 * ady)
                    else:
                        i = x - lx1
                        if 0 <= i <= ddx:
                            mm = (2 * ady * i + ddx - 1) // (2 * ddx) if ddx else 0
                            on |= y == (ly1 - mm if ddy < 0 else ly1 + mm)
                if Y0 != Y1:
                    if inimg:
                        c0, c1 = ((X0 << 16) + 32768, Y0), ((X1 << 16) + 32768, Y1)
                    elif cy0 != cy1:
                        c0, c1 = (cx0 << 16, cy0), (cx1 << 16, cy1)
                    else:
                        c0, c1 = (X0 << 16, Y0), (X1 << 16, Y1)
                    dx = cdiv(c1[0] - c0[0], c1[1] - c0[1])
                    y0, y1, x0 = (Y0, Y1, c0[0] + (Y0 - c0[1]) * dx) if Y0 < Y1 else (Y1, Y0, c1[0] + (Y1 - c1[1]) * dx)
                    if y0 <= y < y1:
                        a = (x0 + (y - y0) * dx) >> 16
                        clt += a < x
                        cle += a <= x
            out[y, x] = on or (clt & 1) or cle > clt
    return out


def test_fillpoly_restatement_known_answers_and_per_pixel_form():
    """oracle/data_ref.py fill_poly_u8 (cv2.fillPoly, OpenCV 4.x drawing.cpp restated; cv2 absent, so
    parity with cv2 itself is unpinned): hand-derived answers of the algorithm -- a right triangle's
    staircase (Bresenham diagonal from the left endpoint, x + 1/2 spans), a square's outline + interior,
    one point, a clipped triangle -- and agreement with the per-pixel form the HIP kernels evaluate on
    300 random polygons, a third of them crossing the image border."""
    tri = O.fill_poly_u8([[0, 0], [4, 0], [0, 4]], 6, 6)
    exp = np.zeros((6, 6), np.uint8)
    for r in range(5):
        exp[r, :5 - r] = 1
    assert np.array_equal(tri, exp)
    sq = O.fill_poly_u8([[2, 2], [5, 2], [5, 5], [2, 5]], 8, 8)
    assert sq.sum() == 16 and (sq[2:6, 2:6] == 1).all()
    pt = O.fill_poly_u8([[3, 4]], 6, 6)
    assert pt.sum() == 1 and pt[4, 3] == 1
    assert O.fill_poly_u8([[-9, -9], [-1, -3], [-5, -1]], 6, 6).sum() == 0
    # border-crossing polygons (clipLine + the re-projected PolyEdge path), answers derived by hand from
    # the geometry: exact-integer edges leave no rounding choice, so any OpenCV >= 4.5.2 (requirements.txt:
    # opencv-python>=4.5.0) fills these pixels
    rect = O.fill_poly_u8([[-3, 1], [3, 1], [3, 4], [-3, 4]], 6, 6)  # left half outside
    exp = np.zeros((6, 6), np.uint8)
    exp[1:5, 0:4] = 1
    assert np.array_equal(rect, exp)
    diag = O.fill_poly_u8([[2, 0], [9, 0], [2, 7]], 6, 6)  # hypotenuse x + y = 9 leaves right and bottom
    exp = np.zeros((6, 6), np.uint8)
    for r in range(6):
        exp[r, 2:min(5, 9 - r) + 1] = 1
    assert np.array_equal(diag, exp)
    top = O.fill_poly_u8([[1, -4], [4, -4], [4, 2], [1, 2]], 6, 6)  # top edge above the image
    exp = np.zeros((6, 6), np.uint8)
    exp[0:3, 1:5] = 1
    assert np.array_equal(top, exp)
    rng = np.random.default_rng(0)
    for t in range(300):
        h, w = int(rng.integers(4, 20)), int(rng.integers(4, 20))
        n = int(rng.integers(1, 9))
        lo, hi = (-3, 3) if t % 3 == 0 else (0, 1)
        pts = np.stack([rng.integers(lo, w + hi, n), rng.integers(lo, h + hi, n)], 1)
        assert np.array_equal(O.fill_poly_u8(pts, h, w), _fillpoly_per_pixel(pts, h, w)), (pts.tolist(), h, w)
