"""The reference's loss modules as API on the fused HIP loss kernel (loss.hip) vs the reference.

loss_api.npz holds the reference's own FocalLoss(alpha, gamma, ignore_index, class_weights)
over five configurations, Trainer.ce_loss, and Trainer.dice_loss / tversky_loss with
num_classes 2 and 3 (tests/golden/gen_golden.py gen_loss_api): values and d loss / d logits.
fp32 kernel vs fp64-generated fixture: values within 1e-5 relative, gradients within 1e-4
(max-normalised) and 1e-3 per element with a floor of 1e-3 of the largest gradient.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

FOCAL_CFGS = [  # tests/golden/gen_golden.py LOSS_API_FOCAL
    ([1.0, 8.0, 5.0], 5.0, None, [1.0, 20.0, 10.0]),
    (None, 2.0, None, None),
    (0.25, 2.0, 1, None),
    ([1.0, 2.0], 3.0, None, [1.0, 4.0, 2.0]),
    ([0.5, 1.0, 2.0], 1.5, 255, [2.0, 1.0, 3.0]),
]


def _check(g, name, fn, target):
    x = torch.from_numpy(g["x"]).float().to(DEV).requires_grad_(True)
    v = fn(x, target.to(DEV))
    v.backward()
    ref_v, ref_g = float(g[f"{name}_val"]), torch.from_numpy(g[f"{name}_grad"]).double()
    got = x.grad.double().cpu()
    assert abs(v.item() - ref_v) < 1e-5 * abs(ref_v), (name, v.item(), ref_v)
    scale = float(ref_g.abs().max())
    assert float((got - ref_g).abs().max()) < 1e-4 * scale, name
    per_px = (got - ref_g).abs() / ref_g.abs().clamp_min(1e-3 * scale)
    assert float(per_px.max()) < 1e-3, (name, float(per_px.max()))


def test_loss_api_matches_reference_fixture(golden_dir):
    from eunet.models import EnhancedUNet
    from eunet.train_eval import FocalLoss, Trainer
    g = np.load(os.path.join(golden_dir, "loss_api.npz"), allow_pickle=False)
    t, t_ign = torch.from_numpy(g["t"]), torch.from_numpy(g["t_ign"])
    for i, (a, gm, ii, cw) in enumerate(FOCAL_CFGS):
        fl = FocalLoss(alpha=a, gamma=gm, ignore_index=ii,
                       class_weights=None if cw is None else torch.tensor(cw, device=DEV))
        _check(g, f"focal{i}", fl, t_ign if ii == 255 else t)
    tr = Trainer(EnhancedUNet(num_classes=3, base_ch=16).to(DEV), DEV, "enhanced_unet")
    _check(g, "focal0", tr.focal_loss, t)  # the Trainer's own module is configuration 0
    _check(g, "ce", tr.ce_loss, t)
    for nc in (2, 3):
        _check(g, f"dice_nc{nc}", lambda x, tt: tr.dice_loss(x, tt, num_classes=nc), t)
        _check(g, f"tversky_nc{nc}", lambda x, tt: tr.tversky_loss(x, tt, num_classes=nc), t)
    _check(g, "tversky_a05", lambda x, tt: tr.tversky_loss(x, tt, num_classes=3, alpha=0.5), t)


def test_combined_loss_is_the_weighted_sum_of_the_terms(golden_dir):
    """_compute_combined_loss = 2.5 focal + 2.5 dice + 1.0 tversky, each term differentiable."""
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    g = np.load(os.path.join(golden_dir, "loss_k3.npz"), allow_pickle=False)
    tr = Trainer(EnhancedUNet(num_classes=3, base_ch=16).to(DEV), DEV, "enhanced_unet")
    lg = torch.from_numpy(g["logits"]).float().to(DEV)
    tg = torch.from_numpy(g["target"]).to(DEV)
    grads = []
    for fn in (lambda x: tr.focal_loss(x[None], tg[None]), lambda x: tr.dice_loss(x[None], tg[None]),
               lambda x: tr.tversky_loss(x[None], tg[None]), lambda x: tr._compute_combined_loss(x, tg)):
        x = lg.clone().requires_grad_(True)
        v = fn(x)
        v.backward()
        grads.append((v.item(), x.grad.double().cpu()))
    (f, gf), (d, gd), (tv, gt), (tot, gtot) = grads
    for val, key in ((f, "focal"), (d, "dice"), (tv, "tversky"), (tot, "total")):
        assert abs(val - float(g[key])) < 1e-5 * abs(float(g[key])), key
    assert abs(tot - (2.5 * f + 2.5 * d + 1.0 * tv)) < 1e-5 * abs(tot)
    comb = 2.5 * gf + 2.5 * gd + 1.0 * gt
    assert float((gtot - comb).abs().max()) < 1e-5 * float(gtot.abs().max())
    assert float((gtot - torch.from_numpy(g["grad"])).abs().max()) < 1e-4 * float(gtot.abs().max())


def test_out_of_range_target_is_reported():
    """A K=2 model fed a mask holding label 2 (dead, as CellDataset emits for LabelMe 'dead'):
    the reference's F.cross_entropy raises; here the kernel counts the bad targets and the
    training loop raises ValueError at its next sync.  A clean step afterwards is unaffected."""
    from eunet import synth
    from eunet.losses import combined_loss, check_targets
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    x, m = synth.batch(2, 64, 64, start_index=1, num_classes=2, in_channels=1, device=DEV)
    bad = m.clone()
    bad[0, :3, :5] = 2
    lg = torch.randn(2, 2, 64, 64, device=DEV)
    with pytest.raises(ValueError, match="outside"):
        combined_loss(lg, bad, validate=True)
    combined_loss(lg, m, validate=True)  # the counter was reset by the raise; clean input passes
    tr = Trainer(EnhancedUNet(num_classes=2, in_channels=1, base_ch=16).to(DEV), DEV, "enhanced_unet")
    before = {k: v.detach().clone() for k, v in tr.model.state_dict().items()}
    with pytest.raises(ValueError, match="15 target"):
        tr.step(x, bad)
    # raised before backward / AdamW: the parameters are untouched (BN running stats, updated by
    # the forward, are buffers the reference's forward updates too before its loss raises)
    for k, v in tr.model.named_parameters():
        assert torch.equal(v.detach(), before[k]), k
    assert np.isfinite(tr.step(x, m))
    with pytest.raises(ValueError):
        tr.train_epoch([{"images": x.cpu(), "batch_items": [{"semantic_mask": bad[i].cpu()} for i in range(2)]}])
    check_targets()  # nothing pending


@pytest.mark.parametrize("graph", [False, True])
def test_train_epoch_bad_target_leaves_reference_state(graph):
    """train_eval.py:325 -> FocalLoss:39: the reference raises inside the offending batch's loss, after
    its forward (BN running statistics updated) and before its backward / optimizer.step(); later
    batches never run.  A deferred train_epoch (the update guard holds the state from that loss on, the
    error is raised at the epoch's sync) must leave parameters, BN buffers and the AdamW state exactly
    as a trainer that ran the earlier batches and then that batch's forward."""
    from eunet import synth
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    xs, ms = [], []
    for i in range(4):
        x, m = synth.batch(2, 64, 64, start_index=10 + 2 * i, num_classes=2, in_channels=1, device=DEV)
        xs.append(x)
        ms.append(m)
    ms[2] = ms[2].clone()
    ms[2][1, 7, 9] = 5
    batches = [{"images": x, "batch_items": [{"semantic_mask": mm} for mm in m]} for x, m in zip(xs, ms)]

    def trainer():
        torch.manual_seed(3)
        return Trainer(EnhancedUNet(num_classes=2, in_channels=1, base_ch=16).to(DEV), DEV, "enhanced_unet",
                       total_epochs=12)

    ta, tb = trainer(), trainer()
    ta.step_graph = graph
    ta.graph_warmup = 1
    ta.epoch_lr_step(0)
    tb.epoch_lr_step(0)
    with pytest.raises(ValueError, match="1 target"):
        ta.train_epoch(batches)
    tb.step(xs[0], ms[0])
    tb.step(xs[1], ms[1])
    with pytest.raises(ValueError, match="1 target"):
        tb.step(xs[2], ms[2])  # forward (BN running stats) then the raise, before backward / update
    sa, sb = ta.model.state_dict(), tb.model.state_dict()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    for pa, pb in zip(ta.model.parameters(), tb.model.parameters()):
        for key in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(ta.optimizer.state[pa][key], tb.optimizer.state[pb][key]), key
    # the guard drops with the raise: the next epoch trains again (both trainers step alike)
    ta.train_epoch(batches[:2])
    tb.step(xs[0], ms[0])
    tb.step(xs[1], ms[1])
    for (k, pa), pb in zip(ta.model.named_parameters(), tb.model.parameters()):
        assert torch.equal(pa, pb), k
