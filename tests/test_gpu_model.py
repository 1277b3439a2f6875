"""Whole-network parity on the GPU: the HIP path vs the reference fixtures and the oracle.

Gate (BASELINE.json north_star): logits within 1e-3 relative (fp32) of the CPU
reference on identical inputs, PER PIXEL: max over elements of |a - b| / max(|b|, floor)
with floor = PX_FLOOR x max|b| = 1e-2 of the largest logit magnitude, against the fp64
oracle (the fixture-pinned restatement: the exact values the fp32 reference approximates);
the max-normalised max|a - b| / max|b| is checked against the fixtures as well.  Why the
floor: the reference's own fp32 CPU output misses a 1e-3 per-pixel gate at a 1e-3 floor
(2.5e-3 / 3.0e-3 on fwd_c3k3 / fwd_c3k2 vs fp64: logits that cross zero carry the
absolute rounding of the whole network) and meets it at 1e-2 (2.8e-4 / 3.3e-4); each test
prints both floors for our output and, where a fixture exists, for the reference's.  bf16 runs are gated by argmax-mask Dice vs
the fp32 CPU path plus a loose relative L2 bound (bf16 rounding of activations
cannot meet 1e-3; SURVEY.md §7 'bf16 vs 1e-3').
"""
import os

import numpy as np
import pytest
import torch

from oracle import eunet_ref as R

pytestmark = pytest.mark.gpu
BF16_RES = 2.0 ** -8  # bf16 unit roundoff
DEV = "cuda"


def _model(base, cin, K, dtype="fp32"):
    from eunet.models import EnhancedUNet
    m = EnhancedUNet(num_classes=K, in_channels=cin, base_ch=base, dtype=dtype)
    sd = {k: (v.float() if v.is_floating_point() else v) for k, v in R.formula_weights(base, cin, K).items()}
    m.load_state_dict(sd)
    return m.to(DEV)


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


PX_FLOOR = 1e-2


def _rel_px(a, b, floor=PX_FLOOR):
    """Per-pixel relative error with the floor stated above."""
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    den = b.abs().clamp_min(floor * float(b.abs().max()))
    return float(((a - b).abs() / den).max())


def _rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


@pytest.mark.parametrize("fname,K", [("fwd_c3k3.npz", 3), ("fwd_c3k2.npz", 2)])
def test_forward_matches_reference_fixture(golden_dir, fname, K):
    g = _load(golden_dir, fname)
    m = _model(64, 3, K)
    x = torch.from_numpy(g["x"]).to(DEV)
    m.train()
    with torch.no_grad():
        out = m(x)
    assert out.shape == g["out_train"].shape
    assert _rel(out, g["out_train"]) < 1e-3
    with torch.no_grad():
        S64 = R.formula_weights(64, 3, K)
        ref64 = R.forward(S64, torch.from_numpy(g["x"]).double(), training=True)
        ref64_eval = R.forward(S64, torch.from_numpy(g["x"]).double(), training=False)
    print(fname, "ours vs fp64 per-pixel (floor 1e-2, 1e-3):", _rel_px(out, ref64), _rel_px(out, ref64, 1e-3),
          "| reference fp32 vs fp64:", _rel_px(g["out_train"], ref64), _rel_px(g["out_train"], ref64, 1e-3),
          "| max-normalised vs fixture", _rel(out, g["out_train"]))
    assert _rel_px(out, ref64) < 1e-3
    sd = m.state_dict()
    for k in g.files:
        if k.startswith("bn:"):
            assert _rel(sd[k[3:]], g[k]) < 1e-3, k
    m.eval()
    with torch.no_grad():
        out_e = m(x)
    assert _rel(out_e, g["out_eval"]) < 1e-3
    assert _rel_px(out_e, ref64_eval) < 1e-3


def test_in1_matches_reference_fixture(golden_dir):
    g = _load(golden_dir, "in1_equiv.npz")
    from eunet.models import EnhancedUNet
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64)
    sd = {k: v.float() if v.is_floating_point() else v for k, v in R.formula_weights(64, 3, 2).items()}
    sd["model.enc1.0.weight"] = sd["model.enc1.0.weight"][:, :1].contiguous()
    m.load_state_dict(sd)
    m = m.to(DEV).train()
    with torch.no_grad():
        out = m(torch.from_numpy(g["x1"]).to(DEV))
    assert _rel(out, g["out_train"]) < 1e-3
    S1 = R.formula_weights(64, 3, 2)
    S1["model.enc1.0.weight"] = S1["model.enc1.0.weight"][:, :1].contiguous()
    with torch.no_grad():
        ref64 = R.forward(S1, torch.from_numpy(g["x1"]).double(), training=True)
    print("in1 ours vs fp64 per-pixel (floor 1e-2, 1e-3):", _rel_px(out, ref64), _rel_px(out, ref64, 1e-3))
    assert _rel_px(out, ref64) < 1e-3


def _pre_bn_bias(k):
    return k.endswith((".0.bias", ".3.bias")) and not k.startswith("enhance.3")


def _oracle_grads(base, cin, K, x, msk, dtype, pins=None, gpu_dtype="fp32"):
    """Oracle step; pinned fp64 runs also audit the pins against the oracle's own branches (every
    disputed ReLU / pool branch within rounding of its kink / tie: tests/_pins.audit)."""
    import _pins
    S = R.formula_weights(base, cin, K, dtype=dtype)
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    rec = {} if pins is not None and dtype == torch.float64 else None
    loss = R.batch_loss(R.forward(S, x.to(dtype), training=True, pins=pins, record=rec), msk)
    if rec is not None:
        _pins.audit(pins, rec, gpu_dtype, label=f"b{base} c{cin} K{K} {tuple(x.shape[-2:])} {gpu_dtype}")
    loss.backward()
    return S, loss


def _gpu_step_with_pins(m, x, msk):
    """One training forward + backward on the GPU; returns (loss, the branch configuration the
    kernels took: tests/_pins.py)."""
    from eunet.losses import combined_loss
    import _pins
    _pins.keep(m)
    m.train()
    logits = m.forward_lowres(x.to(DEV))
    loss = combined_loss(logits, msk.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    pins = _pins.model_pins(m)
    _pins.keep(m, False)
    m._engine.last_state = None
    return logits.detach(), loss, pins


@pytest.mark.parametrize("base,cin,K,H", [(16, 1, 2, 64), (64, 3, 3, 32), (64, 1, 2, 64), (16, 1, 2, 256)])
def test_train_grads_match_oracle(base, cin, K, H):
    """Loss + every parameter gradient of one train step vs the fp64 oracle, evaluated on the
    branch configuration the GPU took (ReLU masks, max-pool argmax: tests/_pins.py).

    The step is discontinuous at ReLU kinks and max-pool ties; with the oracle pinned to the
    kernels' branches its backward is the exact derivative of the function the GPU computed, so the
    gate is the fp32 one with no kink allowance: relative L2 per tensor <= max(1e-3, 3x the error
    of the same pinned oracle run in fp32).  (16, 1, 2, 256) is BASELINE configs[0]'s shape
    (base 16, 1-ch, 2 classes, 256^2, batch 2)."""
    from eunet import synth
    x, msk = synth.batch(2, H, H, start_index=7, num_classes=K, in_channels=cin)
    m = _model(base, cin, K)
    _, loss, pins = _gpu_step_with_pins(m, x, msk)
    S, loss_ref = _oracle_grads(base, cin, K, x, msk, torch.float64, pins)
    S32, _ = _oracle_grads(base, cin, K, x, msk, torch.float32, pins)
    assert abs(loss.item() - loss_ref.item()) < 1e-4 * abs(loss_ref.item())
    scale = max(float(S[k].grad.abs().max()) for k in S if S[k].grad is not None)
    rows = []
    for k, p in m.named_parameters():
        ref = S[k].grad
        if _pre_bn_bias(k):  # exactly-zero true gradient: compare against the global grad scale
            assert float((p.grad.double().cpu() - ref).abs().max()) < 1e-4 * scale, k
            continue
        tol = max(1e-3, 3.0 * _rel_l2(S32[k].grad, ref))
        rows.append((_rel_l2(p.grad, ref) / tol, k, _rel_l2(p.grad, ref), tol))
    for r in sorted(rows, reverse=True)[:4]:
        print(f"grads b{base} c{cin} K{K} {H}^2 (ratio, name, err, tol):", r)
    assert all(r[0] < 1.0 for r in rows), sorted(rows, reverse=True)[:3]
    for k, v in m.state_dict().items():
        if "running" in k:
            assert _rel(v, S[k]) < 1e-3, k


@pytest.mark.parametrize("fname", ["step_c3k3.npz", "step_pad_c3k3.npz"])
def test_trainer_step_matches_reference_fixture(golden_dir, fname):
    """Trainer.step on the fixture batch: loss and the post-AdamW parameters.  step_pad_c3k3 is a
    40x56 batch: the Trainer's reflect pad of the images and zero pad of the masks to 64x64
    (train_eval.py:248-253, 276-296) is part of what the reference's step pins."""
    from eunet.train_eval import Trainer
    g = _load(golden_dir, fname)
    m = _model(64, 3, 3)
    tr = Trainer(m, DEV, "enhanced_unet", total_epochs=50)
    lr = tr.epoch_lr_step(0)
    assert abs(lr - float(g["lr"])) < 1e-12
    loss = tr.step(torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["m"]).to(DEV))
    assert abs(loss - float(g["loss"])) < 1e-4 * abs(float(g["loss"]))
    sd = m.state_dict()
    for k in sd:
        if "num_batches" in k:
            continue
        post = sd[k].double().cpu().reshape(-1)
        if f"post:{k}" in g.files:
            ref = torch.from_numpy(np.asarray(g[f"post:{k}"])).reshape(-1)
            gref = torch.from_numpy(np.asarray(g[f"grad:{k}"])).reshape(-1) if f"grad:{k}" in g.files else None
        else:
            idx = torch.from_numpy(g[f"post_idx:{k}"])
            post, ref = post[idx], torch.from_numpy(g[f"post_val:{k}"])
            gref = torch.from_numpy(g[f"grad_val:{k}"]).reshape(-1) if f"grad_val:{k}" in g.files else None
        if _pre_bn_bias(k):
            assert float((post - ref).abs().max()) < 2.0 * lr, k
            continue
        # AdamW's first step is lr * g / (|g| + eps): parameters agree to a small fraction
        # of lr.  With dg = the fp32 gradient accuracy (2e-3 of the tensor's scale, a
        # cancelling sum over ~10^6 pixels), elements whose reference |g| <= dg may take
        # either sign (any update in [-lr, lr]); above that the update moves by at most
        # lr*eps*dg/(|g|-dg+eps)^2.
        tol = 0.05 * lr + 1e-6 * ref.abs().max()
        if gref is not None:
            eps = 1e-8
            ga = gref.double().abs()
            dg = 2e-3 * float(ga.max())
            lin = lr * eps * dg / ((ga - dg).clamp_min(0) + eps) ** 2
            tol = tol + torch.where(ga <= dg, torch.full_like(ga, 2.0 * lr), lin)
        assert bool(((post - ref).abs() < tol).all()), (k, float((post - ref).abs().max()))


@pytest.mark.parametrize("H", [128])
def test_bf16_forward_dice_vs_fp32_cpu(H):
    """bf16 path vs the fp32 CPU reference, judged against what bf16 autocast of the
    reference itself achieves on the same input (1e-3 is fp32-only)."""
    from eunet import synth
    x, _ = synth.batch(2, H, H, start_index=3, num_classes=2, in_channels=1)
    S = R.formula_weights(64, 1, 2, dtype=torch.float32)
    pool = torch.nn.functional.avg_pool2d
    with torch.no_grad():
        ref = pool(R.forward(dict(S), x, training=True), 2).double()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            ac = pool(R.forward(R.formula_weights(64, 1, 2, dtype=torch.float32), x, training=True).float(), 2)
    m = _model(64, 1, 2, dtype="bf16").train()
    with torch.no_grad():
        out = m.forward_lowres(x.to(DEV)).double().cpu()

    def metrics(o):
        o = o.double()
        rel_l2 = float((o - ref).norm() / ref.norm())
        a, b = o.argmax(1), ref.argmax(1)
        inter = ((a == 1) & (b == 1)).sum().item()
        dice = 2 * inter / max(1, (a == 1).sum().item() + (b == 1).sum().item())
        return rel_l2, (a == b).double().mean().item(), dice

    ours, auto = metrics(out), metrics(ac)
    print("bf16 ours (relL2, agree, dice):", ours, "autocast:", auto)
    assert ours[0] < max(2.0 * auto[0], 0.02), (ours, auto)
    assert ours[1] > min(0.97, auto[1] - 0.02), (ours, auto)


def test_fp32_large_forward_vs_oracle():
    """256^2 x B=2 (b=64, c=1, K=2) fp32 forward vs the fp64 and the fp32 CPU oracle."""
    from eunet import synth
    x, _ = synth.batch(2, 256, 256, start_index=5, num_classes=2, in_channels=1)
    with torch.no_grad():
        ref = R.forward(R.formula_weights(64, 1, 2, dtype=torch.float32), x, training=True)
        ref64 = R.forward(R.formula_weights(64, 1, 2), x.double(), training=True)
    m = _model(64, 1, 2).train()
    with torch.no_grad():
        out = m(x.to(DEV))
    assert _rel(out, ref) < 1e-3
    print("256^2 fwd per-pixel vs fp64 (floor 1e-2, 1e-3): ours", _rel_px(out, ref64), _rel_px(out, ref64, 1e-3),
          "| CPU fp32 oracle", _rel_px(ref, ref64), _rel_px(ref, ref64, 1e-3))
    assert _rel_px(out, ref64) < 1e-3


def test_train_step_multitile_256_vs_fp64_oracle():
    """Full fp32 train step at 256^2, B=2, base 64, c=1, K=2 against the branch-pinned fp64 oracle:
    every level is multi-tile (L3 = 32^2 = 2 x 1 tiles of 16 x 32 per sample), so the split-K wgrad
    over many tiles, the fused BN-backward reduction rows and the capped reduction grids all run.
    Loss, logits (per pixel) and every parameter gradient (gate as test_train_grads_match_oracle)."""
    from eunet import synth
    x, msk = synth.batch(2, 256, 256, start_index=9, num_classes=2, in_channels=1)
    m = _model(64, 1, 2)
    logits, loss, pins = _gpu_step_with_pins(m, x, msk)
    S, loss_ref = _oracle_grads(64, 1, 2, x, msk, torch.float64, pins)
    S32, _ = _oracle_grads(64, 1, 2, x, msk, torch.float32, pins)
    with torch.no_grad():
        ref_logits = torch.nn.functional.avg_pool2d(R.forward(R.formula_weights(64, 1, 2), x.double(), True), 2)
    print("256^2 step: loss", loss.item(), loss_ref.item(), "logits per-pixel rel", _rel_px(logits, ref_logits))
    assert _rel_px(logits, ref_logits) < 1e-3
    assert abs(loss.item() - loss_ref.item()) < 1e-4 * abs(loss_ref.item())
    scale = max(float(S[k].grad.abs().max()) for k in S if S[k].grad is not None)
    rows = []
    for k, p in m.named_parameters():
        ref = S[k].grad
        if _pre_bn_bias(k):
            assert float((p.grad.double().cpu() - ref).abs().max()) < 1e-4 * scale, k
            continue
        tol = max(1e-3, 3.0 * _rel_l2(S32[k].grad, ref))
        rows.append((_rel_l2(p.grad, ref) / tol, k, _rel_l2(p.grad, ref), tol))
    for r in sorted(rows, reverse=True)[:5]:
        print("256^2 grad (ratio, name, err, tol):", r)
    assert all(r[0] < 1.0 for r in rows), sorted(rows, reverse=True)[:3]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_materialised_activation_is_exact(dtype, monkeypatch):
    """The BN+ReLU applied inside conv .3's forward / wgrad operand staging (the default,
    UNetEngine.materialize_za = False) and the DoubleConv activation materialised once
    (eunet_bnrelu, materialize_za = True) round identically, so the logits, the loss and
    every gradient agree bit for bit."""
    from eunet import engine, synth
    from eunet.losses import combined_loss
    x, msk = synth.batch(2, 64, 64, start_index=3, num_classes=2, in_channels=1)
    out = {}
    for mat in (True, False):
        monkeypatch.setattr(engine.UNetEngine, "materialize_za", mat)
        m = _model(16, 1, 2, dtype)
        m.train()
        logits = m.forward_lowres(x.to(DEV))
        loss = combined_loss(logits, msk.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        out[mat] = (logits.detach().clone(), loss.item(),
                    {k: p.grad.detach().clone() for k, p in m.named_parameters()})
    assert torch.equal(out[True][0], out[False][0])
    assert out[True][1] == out[False][1]
    for k, g in out[True][2].items():
        assert torch.equal(g, out[False][2][k]), k


def test_backward_stream_schedules_are_exact(monkeypatch):
    """The weight gradients on the side stream (conv .3's enqueued early or after the block's BN-a
    backward, UNetEngine.wg3_late; conv .0's data gradient issued before or after them,
    UNetEngine.dgrad_first) or all on the launch stream run the same kernels on the same operands:
    every gradient agrees bit for bit."""
    from eunet import engine, synth
    from eunet.losses import combined_loss
    x, msk = synth.batch(2, 64, 64, start_index=5, num_classes=2, in_channels=1)
    out = {}
    for overlap, late, first in ((True, True, True), (True, True, False), (True, False, True), (False, True, True)):
        monkeypatch.setattr(engine.UNetEngine, "wg3_late", late)
        monkeypatch.setattr(engine.UNetEngine, "overlap_wgrad", overlap)
        monkeypatch.setattr(engine.UNetEngine, "dgrad_first", first)
        m = _model(16, 1, 2, "bf16")
        m.train()
        loss = combined_loss(m.forward_lowres(x.to(DEV)), msk.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        out[(overlap, late, first)] = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    ref = out[(True, True, True)]
    for key, grads in out.items():
        for k, g in grads.items():
            assert torch.equal(g, ref[k]), (key, k)


@pytest.mark.parametrize("dt,base", [("bf16", 16), ("fp32", 16), ("bf16", 64)])
def test_recomputed_block_gradients_are_exact(monkeypatch, dt, base):
    """Block output gradients recomputed inside their BatchNorm's backward apply instead of stored: dec1's
    W^T g_z (UNetEngine.dec1_recompute, eunet_bn_bwd_apply_1x1) and the encoders' gskip + maxpool-adjoint
    (UNetEngine.pool_recompute, eunet_bn_bwd_apply_pool), each producer reducing without storing -- against
    the stored-gradient path: every gradient bit for bit, each switch alone and both (base 64: the bench's
    channel counts; base 16: C = 16 / 32 / 64)."""
    from eunet import engine, synth
    from eunet.losses import combined_loss
    x, msk = synth.batch(2, 64, 96, start_index=9, num_classes=2, in_channels=1)
    out = {}
    for dec1, pool in ((False, False), (True, False), (False, True), (True, True)):
        monkeypatch.setattr(engine.UNetEngine, "dec1_recompute", dec1)
        monkeypatch.setattr(engine.UNetEngine, "pool_recompute", pool)
        m = _model(base, 1, 2, dt)
        m.train()
        loss = combined_loss(m.forward_lowres(x.to(DEV)), msk.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        out[(dec1, pool)] = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    ref = out[(False, False)]
    for key, grads in out.items():
        for k, g in grads.items():
            assert torch.equal(g, ref[k]), (key, k)


def test_train_epoch_device_loss_sum():
    """Trainer.train_epoch keeps the running loss on the device (one sync per epoch) and returns
    what the reference's per-step `total += loss.item()` loop returns (train_eval.py train_epoch),
    with the same parameters afterwards (the kernels reduce in a fixed order)."""
    from eunet import synth
    from eunet.train_eval import Trainer
    batches = []
    for i in range(3):
        x, msk = synth.batch(2, 64, 64, start_index=2 * i, num_classes=2, in_channels=1)
        batches.append({"images": x, "batch_items": [{"semantic_mask": mm} for mm in msk]})
    ta = Trainer(_model(16, 1, 2, "bf16"), DEV, "enhanced_unet", total_epochs=50)
    tb = Trainer(_model(16, 1, 2, "bf16"), DEV, "enhanced_unet", total_epochs=50)
    avg = ta.train_epoch(batches)
    tot = 0.0
    for b in batches:
        tot += tb.step(b["images"].to(DEV), tb._masks(b, DEV, 0, 0))
    assert avg == tot / len(batches)
    for (k, p), q in zip(ta.model.named_parameters(), tb.model.parameters()):
        assert torch.equal(p, q), k


def _oracle_grads_autocast(base, cin, K, x, msk):
    """The oracle's train step with its convolutions under CPU bf16 autocast (the reference run in
    bf16 the way torch.autocast would run it): loss and every parameter gradient."""
    S = R.formula_weights(base, cin, K, dtype=torch.float32)
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        out = R.forward(S, x.float(), training=True)
    loss = R.batch_loss(out.float(), msk)
    loss.backward()
    return S, loss


BF16_GRAD_FLOOR = 3e-2  # relative L2: ~15 bf16 unit roundoffs (2^-9) compounded over 15 layers
HEAD_BF16_GRAD_TOL = 3e-2  # explicit bound on the 2H head's parameter gradients (bf16 MFMA sums; measured <= 1.7e-2)


def test_bf16_train_grads_vs_fp64_oracle():
    """bf16 whole-network gradient parity (models.py:217-238, train_eval.py:337-338): base 64, c 1,
    K 2, 128^2, B 2.  Every parameter gradient of one train step vs the fp64 oracle, relative L2
    <= max(2 x the error of the oracle's own step under CPU bf16 autocast, BF16_GRAD_FLOOR) --
    the gate the bf16 forward uses.  bf16 storage of the activations and gradients is itself
    ill-conditioned for the deep encoder's weight gradients (the BN backward subtracts two means
    from g'; measured on the first GPU run: 0.3-0.5 relative L2 for enc1-enc3 weights, ours and
    autocast's alike, ours/autocast 0.9-1.2), so the gate is relative to what bf16 does to the
    reference, not absolute.  Conv biases ahead of a BatchNorm have an exactly-zero true gradient
    and are compared with the global gradient scale."""
    from eunet import synth
    from eunet.losses import combined_loss
    x, msk = synth.batch(2, 128, 128, start_index=31, num_classes=2, in_channels=1)
    S, loss_ref = _oracle_grads(64, 1, 2, x, msk, torch.float64)
    Sac, loss_ac = _oracle_grads_autocast(64, 1, 2, x, msk)
    m = _model(64, 1, 2, dtype="bf16")
    _, loss, pins = _gpu_step_with_pins(m, x, msk)
    # the gradients below are compared with the unpinned oracle; the bf16 branch configuration is still
    # audited: every bf16 ReLU / pool branch that differs from the fp64 oracle's is within bf16 rounding
    # of its kink / tie (tests/_pins.audit, TOL_BF16)
    import _pins

    def run_ac(record):
        with torch.autocast("cpu", dtype=torch.bfloat16):
            R.forward(R.formula_weights(64, 1, 2, dtype=torch.float32), x.float(), training=True, record=record)

    def run64(p, record):
        R.forward(R.formula_weights(64, 1, 2), x.double(), training=True, pins=p, record=record)
    ref = _pins.autocast_reference(run_ac, run64)
    rec = {}
    with torch.no_grad():
        run64(pins, rec)
    _pins.audit(pins, rec, "bf16", label="bf16 b64 128^2", ref=ref)
    print("bf16 step loss", loss.item(), "fp64", loss_ref.item(), "autocast", loss_ac.item())
    assert abs(loss.item() - loss_ref.item()) < max(2 * abs(loss_ac.item() - loss_ref.item()), 1e-2 * abs(loss_ref.item()))
    scale = max(float(S[k].grad.abs().max()) for k in S if S[k].grad is not None)
    rows = []
    for k, p in m.named_parameters():
        ref = S[k].grad
        if _pre_bn_bias(k):
            err, err_ac = float((p.grad.double().cpu() - ref).abs().max()), float((Sac[k].grad.double() - ref).abs().max())
            # the true gradient is exactly 0: what remains is rounding noise of a sum of bf16-rounded
            # BN-backward outputs, so the floor is the bf16 resolution of the gradient scale (2^-8; a 1e-3
            # floor sat below it: the dual base-96 unetpp.enc1.0.bias measured 2.6e-3 of the scale after the
            # round-4 conv epilogue changes, the oracle under bf16 autocast 1.1e-3)
            assert err < max(2 * err_ac, BF16_RES * scale), (k, err, err_ac, scale)
            continue
        e, eac = _rel_l2(p.grad, ref), _rel_l2(Sac[k].grad, ref)
        rows.append((e / max(2 * eac, BF16_GRAD_FLOOR), k, e, eac))
    for r in sorted(rows, reverse=True)[:8]:
        print("bf16 grad (ratio to the gate, name, ours, autocast):", r)
    print("bf16 grad ours / autocast, median over tensors:", sorted(r[2] / max(r[3], 1e-30) for r in rows)[len(rows) // 2])
    assert all(r[0] < 1.0 for r in rows), sorted(rows, reverse=True)[:3]
    # the 2H head's parameter gradients carry an explicit bf16-level bound as well: since round 4 gW2, dgamma
    # and dbeta are MFMA sums over bf16 operands (g_o, relu(pre), xhat rounded to bf16; csrc/head.hip
    # head_bwd1t32), gW1 an MFMA over bf16 g_h and im2col(u) -- each operand within 2^-9 relative, the sums
    # over 2 x 256^2 pixels in fp32
    head = {r[1]: r[2] for r in rows if r[1].startswith("enhance.")}
    print("bf16 head parameter gradients, rel L2 vs fp64:", head)
    assert all(e < HEAD_BF16_GRAD_TOL for e in head.values()), head


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_bn_apply_schedule_is_exact(dtype, monkeypatch):
    """UNetEngine.fuse_bn_apply (BN-backward apply inside the data-gradient staging, weight
    gradients reading the gy it stores) against the separate bn_bwd_apply passes: the loss and
    every parameter gradient agree bit for bit, with the weight gradients on the side stream or
    on the launch stream."""
    from eunet import engine, synth
    from eunet.losses import combined_loss
    x, msk = synth.batch(2, 96, 64, start_index=13, num_classes=2, in_channels=1)
    out = {}
    deep = frozenset({"enc3", "enc4", "dec4"})  # per-block fusion (UNetEngine.fuse_bn_apply as a set)
    for fused, fused_a, overlap in ((True, False, True), (True, True, True), (False, False, True),
                                    (True, True, False), (deep, False, True), (deep, deep, True)):
        monkeypatch.setattr(engine.UNetEngine, "fuse_bn_apply", fused)
        monkeypatch.setattr(engine.UNetEngine, "fuse_bn_apply_a", fused_a)
        monkeypatch.setattr(engine.UNetEngine, "overlap_wgrad", overlap)
        m = _model(32, 1, 2, dtype)
        m.train()
        loss = combined_loss(m.forward_lowres(x.to(DEV)), msk.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        out[(fused, fused_a, overlap)] = (loss.item(), {k: p.grad.detach().clone() for k, p in m.named_parameters()})
    ref = out[(False, False, True)]
    for key, (lv, grads) in out.items():
        assert lv == ref[0], key
        for k, g in grads.items():
            assert torch.equal(g, ref[1][k]), (key, k)


@pytest.mark.parametrize("dtype", ["bf16"])
def test_wgrad_schedule_knobs_are_exact(dtype, monkeypatch):
    """UNetEngine.wg3_late / wg3_early_last / dgrad_first / fork_once only move conv .3's weight gradient
    between the launch and side streams, change the issue order or the events the side stream waits on:
    loss and every parameter gradient bit for bit."""
    from eunet import engine, synth
    from eunet.losses import combined_loss
    x, msk = synth.batch(2, 96, 64, start_index=17, num_classes=2, in_channels=1)
    out = {}
    for late, early_last, dfirst, fonce in ((True, True, False, True), (True, False, False, True),
                                            (False, False, False, True), (True, True, True, True),
                                            (True, False, False, False), (True, False, True, False)):
        monkeypatch.setattr(engine.UNetEngine, "wg3_late", late)
        monkeypatch.setattr(engine.UNetEngine, "wg3_early_last", early_last)
        monkeypatch.setattr(engine.UNetEngine, "dgrad_first", dfirst)
        monkeypatch.setattr(engine.UNetEngine, "fork_once", fonce)
        m = _model(32, 1, 2, dtype)
        m.train()
        loss = combined_loss(m.forward_lowres(x.to(DEV)), msk.to(DEV))
        loss.backward()
        torch.cuda.synchronize()
        out[(late, early_last, dfirst, fonce)] = (loss.item(),
                                                  {k: p.grad.detach().clone() for k, p in m.named_parameters()})
    ref = out[(True, False, False, False)]
    for key, (lv, grads) in out.items():
        assert lv == ref[0], key
        for k, g in grads.items():
            assert torch.equal(g, ref[1][k]), (key, k)


def _graph_batches(n, H=64, W=96, B=2):
    from eunet import synth
    out = []
    for i in range(n):
        x, msk = synth.batch(B, H, W, start_index=5 * i + 1, num_classes=3, in_channels=3)
        out.append((x.to(DEV), msk.to(DEV)))
    return out


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_step_graph_replay_is_exact(dtype):
    """Trainer.step_graph (StepGraph: the step captured as a HIP graph, replayed per batch) against
    eager steps from the same weights: every step's loss, the parameters, the AdamW moments and the
    BN running statistics agree bit for bit over 2 eager warm-up steps, a capture, replays, an LR
    change (epoch_lr_step: AdamW runs outside the graph, so no re-capture) and more replays."""
    from eunet.train_eval import Trainer
    batches = _graph_batches(7)
    ta = Trainer(_model(16, 3, 3, dtype), DEV, "enhanced_unet", total_epochs=12)
    tb = Trainer(_model(16, 3, 3, dtype), DEV, "enhanced_unet", total_epochs=12)
    tb.step_graph = True
    for i, (x, m) in enumerate(batches):
        if i == 4:
            ta.epoch_lr_step(1)
            tb.epoch_lr_step(1)
        la = ta.step(x, m, sync_loss=False)
        lb = tb.step(x, m, sync_loss=False)
        assert torch.equal(la, lb), i
    assert tb._graph is not None and tb.graph_captures == 1
    assert ta.optimizer.param_groups[0]["lr"] == tb.optimizer.param_groups[0]["lr"] != 4e-3
    for (k, p), q in zip(ta.model.named_parameters(), tb.model.parameters()):
        assert torch.equal(p, q), k
        sa, sb = ta.optimizer.state[p], tb.optimizer.state[q]
        for s in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(sa[s], sb[s]), (k, s)
    for (k, a), b in zip(ta.model.named_buffers(), tb.model.buffers()):
        assert torch.equal(a, b), k


def test_step_graph_recaptures_after_set_dtype():
    """EnhancedUNet.set_dtype between graph-replayed steps: the compute dtype is part of the
    graph key, so the switch re-captures instead of replaying the bf16 kernels, and the fp32 steps that
    follow equal an eager trainer's that made the same switch."""
    from eunet.train_eval import Trainer
    batches = _graph_batches(7)
    ta = Trainer(_model(16, 3, 3, "bf16"), DEV, "enhanced_unet", total_epochs=12)
    tb = Trainer(_model(16, 3, 3, "bf16"), DEV, "enhanced_unet", total_epochs=12)
    tb.step_graph = True
    for i, (x, m) in enumerate(batches):
        if i == 4:
            ta.model.set_dtype("fp32")
            tb.model.set_dtype("fp32")
            assert tb.graph_captures == 1
        assert torch.equal(ta.step(x, m, sync_loss=False), tb.step(x, m, sync_loss=False)), i
    assert tb.graph_captures == 2 and tb._graph.key[5][-2:] == ("torch.float32", "torch.float32")
    for (k, p), q in zip(ta.model.named_parameters(), tb.model.parameters()):
        assert torch.equal(p, q), k


def test_step_graph_train_epoch_and_bad_targets():
    """train_epoch over a graph-replayed trainer returns the eager epoch's mean loss, and an
    out-of-range target in a replayed batch still raises at the epoch's sync (the loss adds its
    count into the persistent accumulator inside the graph)."""
    from eunet.train_eval import Trainer
    batches = [{"images": x, "batch_items": [{"semantic_mask": mm} for mm in m]} for x, m in _graph_batches(5)]
    ta = Trainer(_model(16, 3, 3, "bf16"), DEV, "enhanced_unet", total_epochs=12)
    tb = Trainer(_model(16, 3, 3, "bf16"), DEV, "enhanced_unet", total_epochs=12)
    tb.step_graph = True
    assert ta.train_epoch(batches) == tb.train_epoch(batches)
    assert tb._graph is not None
    assert ta.train_epoch(batches) == tb.train_epoch(batches)
    bad = [dict(b) for b in batches]
    m = bad[2]["batch_items"][0]["semantic_mask"].clone()
    m[3, 5] = 7
    bad[2] = {"images": bad[2]["images"], "batch_items": [{"semantic_mask": m}, bad[2]["batch_items"][1]]}
    with pytest.raises(ValueError, match="outside"):
        tb.train_epoch(bad)
    tb.train_epoch(batches)  # the accumulator was cleared at the raise: no error carried over


def test_step_graph_ragged_epochs_keep_one_graph_per_shape():
    """An epoch whose last batch is smaller (an odd image count at batch 2) with an LR step between
    epochs: one graph per batch shape, captured once and replayed in every later epoch, and the
    epochs' mean losses and final parameters equal the eager trainer's bit for bit."""
    from eunet.train_eval import Trainer
    full = _graph_batches(4)
    last = _graph_batches(1, B=1)
    batches = [{"images": x, "batch_items": [{"semantic_mask": mm} for mm in m]} for x, m in full + last]
    ta = Trainer(_model(16, 3, 3, "bf16"), DEV, "enhanced_unet", total_epochs=12)
    tb = Trainer(_model(16, 3, 3, "bf16"), DEV, "enhanced_unet", total_epochs=12)
    tb.step_graph = True
    for ep in range(3):
        ta.epoch_lr_step(ep)
        tb.epoch_lr_step(ep)
        assert ta.train_epoch(batches) == tb.train_epoch(batches), ep
    assert tb.graph_captures == 2 and len(tb._graphs) == 2
    for (k, p), q in zip(ta.model.named_parameters(), tb.model.parameters()):
        assert torch.equal(p, q), k
    tb.graph_cache = 1  # a one-graph cache re-captures at every shape change and stays exact
    for ep in range(3, 5):
        ta.epoch_lr_step(ep)
        tb.epoch_lr_step(ep)
        assert ta.train_epoch(batches) == tb.train_epoch(batches), ep
    assert tb.graph_captures == 5 and len(tb._graphs) == 1  # epoch 3: the last batch; epoch 4: both
    for (k, p), q in zip(ta.model.named_parameters(), tb.model.parameters()):
        assert torch.equal(p, q), k


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_dispatcher_path_is_exact_and_visible(dtype, monkeypatch):
    """The network ops run through torch.ops.eunet.* (the default) or directly (ops.USE_DISPATCHER =
    False): two Trainer steps give bit-identical losses and parameters, and torch.profiler records the
    eunet:: ops of a step."""
    from eunet import ops
    from eunet.train_eval import Trainer
    batches = _graph_batches(2)
    ta = Trainer(_model(16, 3, 3, dtype), DEV, "enhanced_unet", total_epochs=12)
    tb = Trainer(_model(16, 3, 3, dtype), DEV, "enhanced_unet", total_epochs=12)
    for x, m in batches:
        monkeypatch.setattr(ops, "USE_DISPATCHER", True)
        la = ta.step(x, m, sync_loss=False)
        monkeypatch.setattr(ops, "USE_DISPATCHER", False)
        lb = tb.step(x, m, sync_loss=False)
        assert torch.equal(la, lb)
    for (k, p), q in zip(ta.model.named_parameters(), tb.model.parameters()):
        assert torch.equal(p, q), k
    monkeypatch.setattr(ops, "USE_DISPATCHER", True)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        ta.step(*batches[0], sync_loss=False)
        torch.cuda.synchronize()
    names = {e.key for e in prof.key_averages()}
    for op in ("eunet::conv3x3_fwd", "eunet::conv3x3_wgrad", "eunet::head_bwd", "eunet::bn_finalize"):
        assert op in names, (op, sorted(n for n in names if n.startswith("eunet::")))


def test_trained_model_logits_per_pixel_north_star_gate():
    """BASELINE north_star: logits within 1e-3 relative of the CPU reference, per pixel, fp32 -- here with the
    strict floor (|a - b| / max(|b|, 1e-3 max|b|)), on a model trained for 60 seeded steps (untimed, as the
    bench's parity model) rather than formula weights: its logits no longer straddle zero wholesale, so the
    1e-3 floor is meaningful (formula-weight logits cross zero everywhere and even the reference's own fp32
    run misses a 1e-3 floor there -- see the module docstring).  Eval mode, held-out 256^2 tile vs the fp64
    oracle (forward + the 2H -> H bilinear resize of train_eval.py:306-310)."""
    from eunet import synth
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    torch.manual_seed(1)
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=32, dtype="fp32").to(DEV)
    tr = Trainer(m, DEV, "enhanced_unet", total_epochs=50)
    for s in range(60):
        for g in tr.optimizer.param_groups:
            g["lr"] = 4e-3 * min(1.0, (s + 1) / 12)
        x, msk = synth.batch(4, 128, 128, start_index=5000 + 4 * s, num_classes=2, in_channels=1, device=DEV)
        tr.step(x, msk, sync_loss=False)
    torch.cuda.synchronize()
    x, _ = synth.batch(1, 256, 256, start_index=90000, num_classes=2, in_channels=1)
    S = {k: (v.detach().double().cpu() if v.is_floating_point() else v.cpu()) for k, v in m.state_dict().items()}
    with torch.no_grad():
        ref = torch.nn.functional.interpolate(R.forward(S, x.double(), training=False), size=(256, 256),
                                              mode="bilinear", align_corners=False)
    m.eval()
    with torch.no_grad():
        got = m.forward_lowres(x.to(DEV)).double().cpu()
    px3, px2 = _rel_px(got, ref, 1e-3), _rel_px(got, ref, 1e-2)
    print(f"trained base-32 model, eval logits per pixel vs fp64: {px3:.2e} (floor 1e-3), {px2:.2e} (floor 1e-2)")
    assert px3 < 1e-3
