"""Generate golden fixtures by running the REFERENCE implementation (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Imports /root/reference/{models,train_eval}.py (read-only, never copied) with inert
stub modules for the CPU/data/plot libraries it imports at module level but never
uses on the training path (cv2, skimage, pycocotools, torchvision, seaborn).  The
stubs fetch nothing.  Outputs small .npz fixtures next to this script; the GPU box
and the product never read /root/reference.

Fixtures (all with formula weights, oracle/weights.py):
  fwd_c3k3.npz     reference EnhancedUNet (SMP-absent fallback, base 64, in 3, K 3):
                   train-mode logits, BN running stats after, eval-mode logits
  fwd_c3k2.npz     same with num_classes=2
  in1_equiv.npz    1-channel input via the (x,0,0) equivalence (in 3 model, K 2)
  loss_k3.npz      Trainer._compute_combined_loss (+parts) and d loss / d logits, K=3
  loss_k2.npz      K=2 via a -inf third logit fed to the reference loss
  step_c3k3.npz    one Trainer.train_epoch (warmup-stepped LR, clip, AdamW) on a B=2 batch
  step_pad_c3k3.npz  the same on a 40x56 batch: train_epoch's reflect pad of the images and zero
                   pad of the masks to /32 (train_eval.py:248-253, 276-296) exercised
  lr_traj.npz      train_model's per-epoch LR for E in {6, 50}
  metrics.npz      metrics.calculate_semantic_metrics / calculate_iou / calculate_dice on
                   mask pairs incl. empty classes and out-of-range labels
  probs_mask.npz   Evaluator._convert_probs_to_mask on probability maps that reach every
                   branch (argmax filters, background promotions, all pixel-ratio regimes)
  dual_c3k3.npz    SMP-path EnhancedUNet (attention gate, fusion head, residual, aux outputs)
                   with stand-in branches + one train_epoch with auxiliary supervision
  loss_api.npz     the reference loss modules as API: FocalLoss(alpha, gamma, ignore_index,
                   class_weights) over several configurations (list / scalar / short alpha,
                   ignore_index in and out of range, non-integer gamma), Trainer.ce_loss,
                   Trainer.dice_loss / tversky_loss with num_classes 2 and 3 -- values and
                   d loss / d logits
  tta_c3k3.npz     Evaluator._run_model_single / _run_tta_inference (flips + 0.75/1.25
                   rescales) of the reference model (eval mode, BN stats from one train
                   forward) on a 40x56 image (reflect pad to /32 and crop exercised)
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)

from oracle.weights import formula_state_dict  # noqa: E402
from oracle.eunet_ref import state_spec  # noqa: E402


def _install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    class _Any:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, item):
            return _Any()

        def __call__(self, *a, **k):
            return _Any()

    mod("cv2")
    sk = mod("skimage")
    sk.measure = mod("skimage.measure")
    sk.feature = mod("skimage.feature", peak_local_max=lambda *a, **k: None)
    pc = mod("pycocotools")
    pc.mask = mod("pycocotools.mask")
    pc.coco = mod("pycocotools.coco", COCO=_Any)
    pc.cocoeval = mod("pycocotools.cocoeval", COCOeval=_Any)
    tv = mod("torchvision")
    tv.transforms = mod("torchvision.transforms", Compose=_Any, ToTensor=_Any, Normalize=_Any)
    mod("seaborn")


def _import_reference():
    _install_stubs()
    sys.path.insert(0, REF)
    import models as ref_models  # noqa
    import train_eval as ref_te  # noqa
    assert not ref_models.SMP_AVAILABLE, "fixtures pin the SMP-absent fallback"
    return ref_models, ref_te


def _load_formula(model, base, in_ch, K, dtype=torch.float32):
    sd = formula_state_dict(state_spec(base, in_ch, K))
    ref_sd = model.state_dict()
    assert list(ref_sd.keys()) == list(sd.keys()), "state_dict schema mismatch"
    new = {}
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            new[k] = torch.tensor(0, dtype=torch.long)
        else:
            new[k] = torch.from_numpy(np.asarray(v)).to(dtype).reshape(ref_sd[k].shape)
    model.load_state_dict(new)


def _inputs(B, C, H, W, K, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, C, H, W, generator=g)
    m = torch.randint(0, K, (B, H, W), generator=g)
    return x, m


def _bn_stats(model):
    return {k: v.detach().numpy().copy() for k, v in model.state_dict().items()
            if k.endswith("running_mean") or k.endswith("running_var")}


def gen_forward(ref_models, K, fname):
    torch.manual_seed(0)
    model = ref_models.get_model("enhanced_unet", num_classes=K, device="cpu")
    _load_formula(model, 64, 3, K)
    x, _ = _inputs(2, 3, 32, 32, K, seed=11)
    model.train()
    with torch.no_grad():
        out_train = model(x)
    stats = _bn_stats(model)
    model.eval()
    with torch.no_grad():
        out_eval = model(x)
    np.savez_compressed(os.path.join(HERE, fname), x=x.numpy(), out_train=out_train.numpy(),
                        out_eval=out_eval.numpy(),
                        **{"bn:" + k: v for k, v in stats.items()})


def gen_in1(ref_models):
    model = ref_models.get_model("enhanced_unet", num_classes=2, device="cpu")
    _load_formula(model, 64, 3, 2)
    g = torch.Generator().manual_seed(21)
    x1 = torch.rand(2, 1, 32, 32, generator=g)
    x3 = torch.cat([x1, torch.zeros_like(x1), torch.zeros_like(x1)], 1)
    model.train()
    with torch.no_grad():
        out = model(x3)
    np.savez_compressed(os.path.join(HERE, "in1_equiv.npz"), x1=x1.numpy(), out_train=out.numpy())


def gen_loss(ref_te, K, fname):
    tr = ref_te.Trainer(torch.nn.Linear(1, 1), "cpu", "enhanced_unet", total_epochs=50)
    g = torch.Generator().manual_seed(31 + K)
    logits = (torch.randn(K, 24, 20, generator=g) * 2.0).requires_grad_(True)
    target = torch.randint(0, K, (24, 20), generator=g)
    if K == 3:
        feed = logits
    else:  # K=2 semantics: third logit at -inf
        feed = torch.cat([logits, torch.full((1, 24, 20), float("-inf"))], 0)
    lg = feed.unsqueeze(0)
    tg = target.unsqueeze(0)
    focal = tr.focal_loss(lg, tg)
    dice = tr.dice_loss(lg, tg, num_classes=3)
    tv = tr.tversky_loss(lg, tg, num_classes=3)
    total = tr._compute_combined_loss(feed, target)
    total.backward()
    np.savez_compressed(os.path.join(HERE, fname), logits=logits.detach().numpy(),
                        target=target.numpy(), total=total.item(), focal=focal.item(),
                        dice=dice.item(), tversky=tv.item(), grad=logits.grad.numpy())


LOSS_API_FOCAL = [  # (alpha, gamma, ignore_index, class_weights)
    ([1.0, 8.0, 5.0], 5.0, None, [1.0, 20.0, 10.0]),
    (None, 2.0, None, None),
    (0.25, 2.0, 1, None),
    ([1.0, 2.0], 3.0, None, [1.0, 4.0, 2.0]),
    ([0.5, 1.0, 2.0], 1.5, 255, [2.0, 1.0, 3.0]),
]


def gen_loss_api(ref_te):
    """loss_api.npz: the reference's FocalLoss / CrossEntropyLoss / dice_loss / tversky_loss."""
    tr = ref_te.Trainer(torch.nn.Linear(1, 1), "cpu", "enhanced_unet", total_epochs=50)
    g = torch.Generator().manual_seed(91)
    x = torch.randn(2, 3, 12, 10, generator=g) * 2.0
    t = torch.randint(0, 3, (2, 12, 10), generator=g)
    t_ign = t.clone()
    t_ign[:, ::3, ::4] = 255
    out = {"x": x.numpy(), "t": t.numpy(), "t_ign": t_ign.numpy()}

    def run(name, fn, tt):
        xx = x.clone().requires_grad_(True)
        v = fn(xx, tt)
        v.backward()
        out[f"{name}_val"] = v.item()
        out[f"{name}_grad"] = xx.grad.numpy()

    for i, (a, gm, ii, cw) in enumerate(LOSS_API_FOCAL):
        fl = ref_te.FocalLoss(alpha=a, gamma=gm, ignore_index=ii,
                              class_weights=None if cw is None else torch.tensor(cw))
        run(f"focal{i}", fl, t_ign if ii == 255 else t)
    run("ce", tr.ce_loss, t)
    for nc in (2, 3):
        run(f"dice_nc{nc}", lambda xx, tt: tr.dice_loss(xx, tt, num_classes=nc), t)
        run(f"tversky_nc{nc}", lambda xx, tt: tr.tversky_loss(xx, tt, num_classes=nc), t)
    run("tversky_a05", lambda xx, tt: tr.tversky_loss(xx, tt, num_classes=3, alpha=0.5), t)
    np.savez_compressed(os.path.join(HERE, "loss_api.npz"), **out)


def gen_step(ref_models, ref_te, H=32, W=32, fname="step_c3k3.npz", seed=41):
    model = ref_models.get_model("enhanced_unet", num_classes=3, device="cpu")
    _load_formula(model, 64, 3, 3)
    x, m = _inputs(2, 3, H, W, 3, seed=seed)
    batch = {"images": x, "batch_items": [{"semantic_mask": m[i]} for i in range(2)]}
    tr = ref_te.Trainer(model, "cpu", "enhanced_unet", total_epochs=50)
    tr.warmup_scheduler.step()  # train_model epoch 0 (train_eval.py:1104-1105)
    lr = tr.optimizer.param_groups[0]["lr"]
    loss = tr.train_epoch([batch])
    sd = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    grads = {k: p.grad.detach().numpy().copy() for k, p in model.named_parameters()}
    np.savez_compressed(os.path.join(HERE, fname), x=x.numpy(), m=m.numpy(), lr=lr,
                        loss=loss, **_summaries("post", sd), **_summaries("grad", grads))


def _summaries(tag, tensors, full_below=8192, n_sample=64):
    """Full tensor when small; else sum / L2 norm / 64 samples at fixed indices."""
    out = {}
    for k, v in tensors.items():
        v = np.asarray(v, dtype=np.float64)
        if v.size <= full_below:
            out[f"{tag}:{k}"] = v
        else:
            flat = v.reshape(-1)
            idx = sample_indices(k, flat.size, n_sample)
            out[f"{tag}_sum:{k}"] = flat.sum()
            out[f"{tag}_norm:{k}"] = np.sqrt((flat * flat).sum())
            out[f"{tag}_idx:{k}"] = idx
            out[f"{tag}_val:{k}"] = flat[idx]
    return out


def sample_indices(key, n, k):
    from oracle.weights import uniform01
    return np.unique((uniform01("idx:" + key, k) * n).astype(np.int64))


def gen_lr(ref_te):
    out = {}
    for E in (6, 50):
        tr = ref_te.Trainer(torch.nn.Linear(1, 1), "cpu", "enhanced_unet", total_epochs=E)
        lrs = []
        for epoch in range(E):
            if epoch < tr.warmup_epochs:
                tr.warmup_scheduler.step()
            else:
                tr.scheduler.step()
            lrs.append(tr.optimizer.param_groups[0]["lr"])
        out[f"E{E}"] = np.array(lrs)
    np.savez_compressed(os.path.join(HERE, "lr_traj.npz"), **out)


def gen_metrics():
    import metrics as ref_metrics  # /root/reference/metrics.py (imported after the stubs)
    g = np.random.default_rng(51)
    cases = [
        (g.integers(0, 3, (37, 53)), g.integers(0, 3, (37, 53))),
        (np.zeros((16, 16), np.int64), g.integers(0, 3, (16, 16))),
        (g.integers(0, 2, (20, 24)), g.integers(0, 2, (20, 24))),          # class 2 absent in both
        (g.integers(0, 4, (19, 23)), g.integers(0, 4, (19, 23))),          # label 3 is ignored
        (np.full((1, 1), 2, np.int64), np.full((1, 1), 2, np.int64)),
        (np.zeros((8, 8), np.int64), np.zeros((8, 8), np.int64)),
    ]
    out = {}
    for i, (p, t) in enumerate(cases):
        p, t = p.astype(np.int64), t.astype(np.int64)
        out[f"pred{i}"], out[f"gt{i}"] = p, t
        m = ref_metrics.calculate_semantic_metrics(p, t)
        out[f"keys{i}"] = np.array(sorted(m))
        out[f"vals{i}"] = np.array([float(m[k]) for k in sorted(m)])
        out[f"iou{i}"] = float(ref_metrics.calculate_iou(p, t))
        out[f"dice{i}"] = float(ref_metrics.calculate_dice(p, t))
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), n=len(cases), **out)


def _probs(g, h, w, bias, spread):
    lg = torch.from_numpy(g.normal(0.0, spread, (3, h, w))) + torch.tensor(bias).view(3, 1, 1)
    return F.softmax(lg.float(), dim=0)


def gen_probs_mask(ref_te):
    ev = ref_te.Evaluator(torch.nn.Identity(), "cpu", "enhanced_unet")
    g = np.random.default_rng(61)
    biases = [(0.0, 0.0, 0.0), (0.0, 1.5, -1.0), (-1.0, 2.5, 0.0), (0.0, -1.0, 1.2),
              (-0.5, -0.5, 1.6), (-1.5, -1.0, 2.0), (-2.5, -1.5, 2.8), (-3.0, -1.0, 3.5),
              (0.5, 0.0, 0.5), (-2.0, 1.0, 1.0)]
    out = {}
    for i, b in enumerate(biases):
        probs = _probs(g, 48, 56, b, 1.5)
        mask = ev._convert_probs_to_mask(probs)
        out[f"probs{i}"], out[f"mask{i}"] = probs.numpy(), np.asarray(mask, np.int64)
    np.savez_compressed(os.path.join(HERE, "probs_mask.npz"), n=len(biases), **out)


def gen_tta(ref_models, ref_te):
    model = ref_models.get_model("enhanced_unet", num_classes=3, device="cpu")
    _load_formula(model, 64, 3, 3)
    g = torch.Generator().manual_seed(71)
    xw = torch.rand(2, 3, 64, 64, generator=g)
    model.train()
    with torch.no_grad():
        model(xw)  # one train forward: BN running stats away from (0, 1)
    stats = _bn_stats(model)
    model.eval()
    img = torch.rand(3, 40, 56, generator=g)
    ev = ref_te.Evaluator(model, "cpu", "enhanced_unet")
    with torch.no_grad():
        single = ev._run_model_single(img)
        tta = ev._run_tta_inference(img)
    mask = ev._convert_probs_to_mask(tta)
    np.savez_compressed(os.path.join(HERE, "tta_c3k3.npz"), xw=xw.numpy(), img=img.numpy(),
                        single=single.numpy(), tta=tta.numpy(), mask=np.asarray(mask, np.int64),
                        **{"bn:" + k: v for k, v in stats.items()})


def _fake_smp(ref_models):
    """Stand-in for segmentation_models_pytorch (absent here, and its backbones need ImageNet
    weights): UnetPlusPlus / DeepLabV3Plus return the reference's own BasicUNet trunk ending at
    input resolution (dec1 on d2, no final upsample), the build's branch definition."""
    def trunk_forward(self, x):
        e1 = self.enc1(x)
        e2 = self.enc2(self.pool(e1))
        e3 = self.enc3(self.pool(e2))
        e4 = self.enc4(self.pool(e3))
        d4 = self.dec4(torch.cat([self.upsample(e4), e3], dim=1))
        d3 = self.dec3(torch.cat([self.upsample(d4), e2], dim=1))
        d2 = self.dec2(torch.cat([self.upsample(d3), e1], dim=1))
        return self.dec1(d2)

    def branch(**kw):
        prev, ref_models.SMP_AVAILABLE = ref_models.SMP_AVAILABLE, False  # -> BasicUNet
        try:
            net = ref_models.UNet(kw["classes"]).model
        finally:
            ref_models.SMP_AVAILABLE = prev
        net.forward = types.MethodType(trunk_forward, net)
        return net

    return types.SimpleNamespace(UnetPlusPlus=branch, DeepLabV3Plus=branch)


def gen_dual(ref_models, ref_te, K=3):
    """dual_c3k3.npz: the reference SMP-path EnhancedUNet (models.py:253-339) with stand-in
    branches: train forward (fused + aux outputs, gate/fusion BN stats), eval forward and one
    Trainer.train_epoch with auxiliary supervision (train_eval.py:199-234).  The two Dropout2d
    use seeded keep-masks that are saved with the fixture."""
    from oracle.dual_ref import dual_state_spec
    smp = _fake_smp(ref_models)
    g = torch.Generator().manual_seed(81)
    B, H = 2, 32
    masks = [(torch.rand(B, 256, generator=g) > 0.2).float(), (torch.rand(B, 128, generator=g) > 0.15).float()]

    def build():
        ref_models.smp, ref_models.SMP_AVAILABLE = smp, True
        try:
            model = ref_models.EnhancedUNet(num_classes=K)
        finally:
            ref_models.SMP_AVAILABLE = False
        sd = formula_state_dict(dual_state_spec(64, 3, K))
        ref_sd = model.state_dict()
        assert list(ref_sd.keys()) == list(sd.keys()), "dual state_dict schema mismatch"
        model.load_state_dict({k: (torch.tensor(0, dtype=torch.long) if k.endswith("num_batches_tracked") else
                                   torch.from_numpy(np.asarray(v)).float().reshape(ref_sd[k].shape))
                               for k, v in sd.items()})
        for idx, (mi, p) in zip((3, 7), zip(masks, (0.2, 0.15))):
            mod = model.fusion_head[idx]
            mod.forward = (lambda mod_, m_, p_: (lambda h: h * m_[:, :, None, None] / (1 - p_) if mod_.training
                                                 else h))(mod, mi, p)
        return model

    def run(model, x, training):
        ref_models.SMP_AVAILABLE = True
        try:
            model.train(training)
            with torch.no_grad():
                out = model(x)
            aux = model.get_aux_outputs()
        finally:
            ref_models.SMP_AVAILABLE = False
        return out, aux

    x, m = _inputs(B, 3, H, H, K, seed=83)
    model = build()
    out, aux = run(model, x, True)
    stats = _bn_stats(model)
    out_eval, _ = run(model, x, False)
    model = build()
    tr = ref_te.Trainer(model, "cpu", "enhanced_unet", total_epochs=50)
    tr.warmup_scheduler.step()
    batch = {"images": x, "batch_items": [{"semantic_mask": m[i]} for i in range(B)]}
    ref_models.SMP_AVAILABLE = True
    try:
        loss = tr.train_epoch([batch])
    finally:
        ref_models.SMP_AVAILABLE = False
    sd = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    grads = {k: p.grad.detach().numpy().copy() for k, p in model.named_parameters()}
    np.savez_compressed(os.path.join(HERE, f"dual_c3k{K}.npz"), x=x.numpy(), m=m.numpy(),
                        drop0=masks[0].numpy(), drop1=masks[1].numpy(), out_train=out.numpy(),
                        aux_unetpp=aux["unetpp"].numpy(), aux_deeplab=aux["deeplab"].numpy(),
                        out_eval=out_eval.numpy(), loss=loss, lr=tr.optimizer.param_groups[0]["lr"],
                        **{"bn:" + k: v for k, v in stats.items() if not k.startswith(("unetpp", "deeplab"))},
                        **_summaries("post", sd), **_summaries("grad", grads))


def main(only=()):
    """python gen_golden.py [name ...]: regenerate all fixtures, or only the named ones."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref_models, ref_te = _import_reference()
    jobs = {
        "fwd_c3k3": lambda: gen_forward(ref_models, 3, "fwd_c3k3.npz"),
        "fwd_c3k2": lambda: gen_forward(ref_models, 2, "fwd_c3k2.npz"),
        "in1_equiv": lambda: gen_in1(ref_models),
        "loss_k3": lambda: gen_loss(ref_te, 3, "loss_k3.npz"),
        "loss_k2": lambda: gen_loss(ref_te, 2, "loss_k2.npz"),
        "loss_api": lambda: gen_loss_api(ref_te),
        "step_c3k3": lambda: gen_step(ref_models, ref_te),
        "step_pad_c3k3": lambda: gen_step(ref_models, ref_te, 40, 56, "step_pad_c3k3.npz", seed=43),
        "lr_traj": lambda: gen_lr(ref_te),
        "metrics": gen_metrics,
        "probs_mask": lambda: gen_probs_mask(ref_te),
        "tta_c3k3": lambda: gen_tta(ref_models, ref_te),
        "dual_c3k3": lambda: gen_dual(ref_models, ref_te, 3),
    }
    for name, job in jobs.items():
        if not only or name in only:
            job()
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
