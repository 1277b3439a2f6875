"""Evaluation path through the C-ABI (evalpath.hip) vs the reference fixtures / oracle.

Integer work (semantic counts, binary overlap, probability -> mask) is bit-exact;
resampling / softmax / TTA probabilities are fp32 within 1e-5 of the fp32 CPU
reference (PyTorch's own CPU kernels order their fp32 sums differently).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def test_semantic_metrics_bit_exact(golden_dir):
    from eunet import metrics
    g = _load(golden_dir, "metrics.npz")
    for i in range(int(g["n"])):
        m = metrics.calculate_semantic_metrics(g[f"pred{i}"], g[f"gt{i}"])
        for k, v in zip(g[f"keys{i}"], g[f"vals{i}"]):
            assert m[str(k)] == v, (i, k)
        assert metrics.calculate_iou(g[f"pred{i}"], g[f"gt{i}"]) == g[f"iou{i}"]
        assert metrics.calculate_dice(g[f"pred{i}"], g[f"gt{i}"]) == g[f"dice{i}"]


def test_semantic_counts_batched_large():
    from eunet import ops
    from oracle import evalpath_ref as E
    gen = torch.Generator().manual_seed(3)
    p = torch.randint(0, 3, (3, 1024, 1024), generator=gen)
    t = torch.randint(0, 3, (3, 1024, 1024), generator=gen)
    c = ops.semantic_counts(p.to(DEV).reshape(3, -1), t.to(DEV).reshape(3, -1)).cpu()
    for n in range(3):
        for k in range(3):
            assert int(c[n, k, 0]) == int((p[n] == k).sum())
            assert int(c[n, k, 1]) == int((t[n] == k).sum())
            assert int(c[n, k, 2]) == int(((p[n] == k) & (t[n] == k)).sum())
    from eunet.metrics import metrics_from_counts
    assert metrics_from_counts(c[1].numpy()) == E.calculate_semantic_metrics(p[1].numpy(), t[1].numpy())


def test_probs_to_mask_bit_exact(golden_dir):
    from eunet import ops
    g = _load(golden_dir, "probs_mask.npz")
    for i in range(int(g["n"])):
        m = ops.probs_to_mask(torch.from_numpy(g[f"probs{i}"]).to(DEV)).cpu().numpy()
        assert np.array_equal(m, g[f"mask{i}"]), i


def test_probs_to_mask_k2_generalisation():
    from eunet import ops
    from oracle import evalpath_ref as E
    gen = torch.Generator().manual_seed(5)
    probs = F.softmax(torch.randn(2, 33, 47, generator=gen) * 2 + torch.tensor([0.0, 0.8]).view(2, 1, 1), 0)
    m = ops.probs_to_mask(probs.to(DEV)).cpu().numpy()
    assert np.array_equal(m, E.convert_probs_to_mask(probs.numpy()))


@pytest.mark.parametrize("hin,win,scale", [(40, 56, 0.75), (40, 56, 1.25), (37, 23, 0.5), (30, 42, None)])
def test_resize_bilinear_matches_torch(hin, win, scale):
    from eunet import ops
    gen = torch.Generator().manual_seed(7)
    x = torch.rand(3, hin, win, generator=gen)
    if scale is None:  # size= form (train_eval.py:449)
        ref = F.interpolate(x.unsqueeze(0), size=(40, 56), mode="bilinear", align_corners=False)[0]
        y = ops.resize_bilinear(x.to(DEV), 40, 56)
    else:  # scale_factor= form (train_eval.py:441-444)
        ref = F.interpolate(x.unsqueeze(0), scale_factor=scale, mode="bilinear", align_corners=False)[0]
        y = ops.resize_bilinear(x.to(DEV), ref.shape[1], ref.shape[2], 1.0 / scale, 1.0 / scale)
    assert y.shape == ref.shape
    assert float((y.cpu() - ref).abs().max()) < 1e-6


def test_flip_and_softmax_crop():
    from eunet import ops
    gen = torch.Generator().manual_seed(9)
    x = torch.rand(3, 21, 30, generator=gen)
    for fh, fw, dims in ((False, True, [2]), (True, False, [1])):
        y = ops.resize_bilinear(x.to(DEV), 21, 30, 1.0, 1.0, flip_h=fh, flip_w=fw).cpu()
        assert torch.equal(y, torch.flip(x, dims=dims))
    lg = torch.randn(3, 32, 64, generator=gen) * 3
    for fh, fw in ((False, False), (True, False), (False, True)):
        p = ops.softmax_crop(lg.to(DEV), 21, 30, flip_h=fh, flip_w=fw).cpu()
        ref = F.softmax(lg, 0)[:, :21, :30]
        dims = [1] if fh else [2] if fw else []
        if dims:
            ref = ref.flip(dims=dims)
        assert float((p - ref).abs().max()) < 1e-6


def test_tta_inference_matches_reference(golden_dir):
    from eunet.evaluator import Evaluator
    from eunet.models import EnhancedUNet
    from oracle import eunet_ref as R
    g = _load(golden_dir, "tta_c3k3.npz")
    S = R.formula_weights(64, 3, 3, dtype=torch.float32)
    for k in g.files:
        if k.startswith("bn:"):
            S[k[3:]] = torch.from_numpy(g[k])
    m = EnhancedUNet(num_classes=3)
    m.load_state_dict(S)
    m = m.to(DEV).eval()
    ev = Evaluator(m, DEV, "enhanced_unet")
    img = torch.from_numpy(g["img"]).to(DEV)
    with torch.no_grad():
        single = ev._run_model_single(img).cpu().numpy()
        tta = ev._run_tta_inference(img).cpu().numpy()
    assert np.abs(single - g["single"]).max() < 1e-5
    assert np.abs(tta - g["tta"]).max() < 1e-5
    assert np.array_equal(ev._convert_probs_to_mask(torch.from_numpy(g["tta"])), g["mask"])
    pred = ev.predict_semantic_mask(img)
    assert pred.shape == (40, 56) and pred.dtype == np.int64
