"""Dual-branch (SMP-path) Enhanced-UNet on the GPU vs the reference fixture and the oracle.

dual_c3k3.npz was produced by the reference EnhancedUNet (models.py:253-339) built
with stand-in branches (tests/golden/gen_golden.py gen_dual); the Dropout2d keep
masks are part of the fixture and injected here.  fp32 gates: fused / aux outputs
and BN running statistics within 1e-3 relative; gradients within
max(1e-3, 3x the fp32 oracle's own error) relative L2 of the fp64 oracle evaluated on the branch
configuration (ReLU masks, max-pool argmax) the GPU took (tests/_pins.py).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import dual_ref as D

pytestmark = pytest.mark.gpu
BF16_RES = 2.0 ** -8  # bf16 unit roundoff
DEV = "cuda"
BRANCHES = ("unetpp.", "deeplab.")


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _model(base, cin, K, dtype="fp32", keep=None):
    from eunet.models import EnhancedUNet
    m = EnhancedUNet(num_classes=K, in_channels=cin, base_ch=base, dtype=dtype, dual_branch=True)
    sd = {k: (v.float() if v.is_floating_point() else v) for k, v in D.dual_formula_weights(base, cin, K).items()}
    m.load_state_dict(sd)
    m = m.to(DEV)
    if keep is not None:
        m._engine.drop_keep = keep
    return m


def test_dual_forward_matches_reference_fixture(golden_dir):
    g = _load(golden_dir, "dual_c3k3.npz")
    keep = (torch.from_numpy(g["drop0"]), torch.from_numpy(g["drop1"]))
    m = _model(64, 3, 3, keep=keep).train()
    x = torch.from_numpy(g["x"]).to(DEV)
    with torch.no_grad():
        out = m(x)
    aux = m.get_aux_outputs()
    assert out.shape == g["out_train"].shape
    assert _rel(out, g["out_train"]) < 1e-3
    assert _rel(aux["unetpp"], g["aux_unetpp"]) < 1e-3
    assert _rel(aux["deeplab"], g["aux_deeplab"]) < 1e-3
    sd = m.state_dict()
    for k in g.files:
        if k.startswith("bn:"):
            assert _rel(sd[k[3:]], g[k]) < 1e-3, k
    m.eval()
    with torch.no_grad():
        out_e = m(x)
    assert _rel(out_e, g["out_eval"]) < 1e-3


def _oracle(base, cin, K, x, msk, keep, dtype, pins=None, gpu_dtype="fp32"):
    """Oracle step; pinned fp64 runs also audit the pins (tests/_pins.audit; bf16 against 2x the
    bf16-autocast oracle's own disputed branches)."""
    import _pins
    ref = None
    if pins is not None and dtype == torch.float64 and gpu_dtype == "bf16":
        def run_ac(record):
            with torch.autocast("cpu", dtype=torch.bfloat16):
                D.dual_forward(D.dual_formula_weights(base, cin, K, dtype=torch.float32), x.float(), training=True,
                               drop_masks=keep, record=record)

        def run64(p, record):
            D.dual_forward(D.dual_formula_weights(base, cin, K), x.double(), training=True, drop_masks=keep,
                           pins=p, record=record)
        ref = _pins.autocast_reference(run_ac, run64)
    S = D.dual_formula_weights(base, cin, K, dtype=dtype)
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    rec = {} if pins is not None and dtype == torch.float64 else None
    fused, aux = D.dual_forward(S, x.to(dtype), training=True, drop_masks=keep, pins=pins, record=rec)
    if rec is not None:
        _pins.audit(pins, rec, gpu_dtype, label=f"dual b{base} c{cin} K{K} {tuple(x.shape[-2:])} {gpu_dtype}",
                    ref=ref)
    loss = D.dual_batch_loss(fused, aux, msk)
    loss.backward()
    return S, loss


def _gpu_step(m, x, msk):
    """One dual-branch training step (aux supervision) on the GPU; returns (loss, pins)."""
    import _pins
    from eunet.train_eval import Trainer
    _pins.keep(m)
    tr = Trainer(m, DEV, "enhanced_unet")
    out = m(x.to(DEV))
    loss = tr.aux_loss(out, m.get_aux_outputs(), msk.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    pins = _pins.model_pins(m)
    _pins.keep(m, False)
    m._engine.last_state = None
    return loss, pins


def _pre_bn_bias(k):
    return k.startswith(BRANCHES) and k.endswith((".0.bias", ".3.bias"))


def _grad_rows(m, S, S32):
    """(ratio to the gate, name, err, tol) per parameter; conv biases ahead of a BatchNorm (true gradient
    exactly 0) are checked against the global gradient scale instead."""
    scale = max(float(S[k].grad.abs().max()) for k in S if S[k].grad is not None)
    rows = []
    for k, p in m.named_parameters():
        ref = S[k].grad
        if _pre_bn_bias(k):
            assert float((p.grad.double().cpu() - ref).abs().max()) < 1e-4 * scale, k
            continue
        tol = max(1e-3, 3 * _rel_l2(S32[k].grad, ref))
        rows.append((_rel_l2(p.grad, ref) / tol, k, _rel_l2(p.grad, ref), tol))
    return rows


@pytest.mark.parametrize("base,cin,K,H", [(64, 3, 3, 32), (16, 1, 2, 64)])
def test_dual_train_grads_match_oracle(golden_dir, base, cin, K, H):
    """Loss + every parameter gradient of one dual-branch step vs the branch-pinned fp64 oracle
    (gate: max(1e-3, 3x the pinned fp32 oracle's error) relative L2; no kink allowance)."""
    if base == 64:
        g = _load(golden_dir, "dual_c3k3.npz")
        x, msk = torch.from_numpy(g["x"]), torch.from_numpy(g["m"])
        keep = (torch.from_numpy(g["drop0"]), torch.from_numpy(g["drop1"]))
    else:
        from eunet import synth
        x, msk = synth.batch(2, H, H, start_index=11, num_classes=K, in_channels=cin)
        gen = torch.Generator().manual_seed(5)
        keep = ((torch.rand(2, 256, generator=gen) > 0.2).float(), (torch.rand(2, 128, generator=gen) > 0.15).float())
    m = _model(base, cin, K, keep=keep).train()
    loss, pins = _gpu_step(m, x, msk)
    S, loss_ref = _oracle(base, cin, K, x, msk, keep, torch.float64, pins)
    S32, _ = _oracle(base, cin, K, x, msk, keep, torch.float32, pins)
    assert abs(loss.item() - loss_ref.item()) < 1e-4 * abs(loss_ref.item())
    rows = _grad_rows(m, S, S32)
    for r in sorted(rows, reverse=True)[:6]:
        print("dual grad (ratio, name, err, tol):", r)
    assert all(r[0] < 1.0 for r in rows), sorted(rows, reverse=True)[:3]


def test_dual_trainer_step_matches_reference_fixture(golden_dir):
    """One Trainer.step (aux supervision, clip, AdamW) vs the reference train_epoch."""
    from eunet.train_eval import Trainer
    g = _load(golden_dir, "dual_c3k3.npz")
    keep = (torch.from_numpy(g["drop0"]), torch.from_numpy(g["drop1"]))
    m = _model(64, 3, 3, keep=keep)
    tr = Trainer(m, DEV, "enhanced_unet", total_epochs=50)
    lr = tr.epoch_lr_step(0)
    loss = tr.step(torch.from_numpy(g["x"]).to(DEV), torch.from_numpy(g["m"]).to(DEV))
    assert abs(loss - float(g["loss"])) < 1e-4 * abs(float(g["loss"]))
    sd = m.state_dict()
    for k, p in m.named_parameters():
        post = p.detach().double().cpu().numpy()
        if f"post:{k}" in g.files:
            ref = g[f"post:{k}"]
            floor = 2.0 * lr if k.endswith((".0.bias", ".3.bias")) else 1e-6
            # AdamW's first step is ~lr * sign(g): a gradient within noise of 0 may flip it
            assert np.abs(post.reshape(ref.shape) - ref).max() < 2e-3 * np.abs(ref).max() + max(floor, 2.0 * lr), k
        else:
            flat = post.reshape(-1)
            assert abs(np.sqrt((flat ** 2).sum()) - float(g[f"post_norm:{k}"])) < 1e-3 * float(g[f"post_norm:{k}"]), k
    for k in g.files:
        if k.startswith("post:") and ("running" in k):
            assert _rel(sd[k[5:]], g[k]) < 1e-3, k


def test_consistency_loss_matches_torch():
    from eunet.losses import consistency_loss
    gen = torch.Generator().manual_seed(3)
    f, a, b = (torch.randn(2, 3, 17, 23, generator=gen, dtype=torch.float64) * 2 for _ in range(3))
    ts = [t.clone().requires_grad_(True) for t in (f, a, b)]
    pf = F.softmax(ts[0], 1)
    ref = 0.24 * F.mse_loss(F.softmax(ts[1], 1), pf) + 0.2 * F.mse_loss(F.softmax(ts[2], 1), pf)
    ref.backward()
    gs = [t.float().to(DEV).requires_grad_(True) for t in (f, a, b)]
    out = consistency_loss(gs[0], gs[1], gs[2], 0.24, 0.2)
    out.backward()
    assert abs(out.item() - ref.item()) < 1e-5 * abs(ref.item())
    for t, r in zip(gs, ts):
        assert _rel(t.grad, r.grad) < 1e-4


def test_dual_bf16_vs_autocast_reference(golden_dir):
    """bf16 path vs the fp32 reference output, judged against bf16 autocast of the oracle
    (the reference's own reduced-precision behaviour on the same input)."""
    g = _load(golden_dir, "dual_c3k3.npz")
    keep = (torch.from_numpy(g["drop0"]), torch.from_numpy(g["drop1"]))
    x = torch.from_numpy(g["x"])
    ref = torch.from_numpy(g["out_train"]).double()
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        ac = D.dual_forward(D.dual_formula_weights(64, 3, 3, dtype=torch.float32), x, True, keep)[0].float()
    m = _model(64, 3, 3, dtype="bf16", keep=keep).train()
    with torch.no_grad():
        out = m(x.to(DEV)).double().cpu()
    ours, auto = _rel_l2(out, ref), _rel_l2(ac, ref)
    print("dual bf16 relL2 ours", ours, "autocast", auto)
    assert torch.isfinite(out).all()
    assert ours < max(2.0 * auto, 0.02), (ours, auto)


def _keep96(seed=7):
    gen = torch.Generator().manual_seed(seed)
    return ((torch.rand(2, 256, generator=gen) > 0.2).float(), (torch.rand(2, 128, generator=gen) > 0.15).float())


def test_dual_base96_forward_fp32_vs_oracle():
    """configs[4] width: base_ch = 96 (96/192/384/768-channel trunks; every layer runs the partial
    co-block path, cout_pad 128 / 256 / 384 / 768).  fp32 train-mode forward at 64^2, B = 2: fused
    and both aux outputs per pixel (floor 1e-3 of the max) within 1e-3 of the fp64 oracle, BN
    running statistics within 1e-3."""
    from eunet import synth
    x, _ = synth.batch(2, 64, 64, start_index=21, num_classes=2, in_channels=1)
    keep = _keep96()
    S = D.dual_formula_weights(96, 1, 2, dtype=torch.float64)
    with torch.no_grad():
        ref, ref_aux = D.dual_forward(S, x.double(), training=True, drop_masks=keep)
    m = _model(96, 1, 2, keep=keep).train()
    with torch.no_grad():
        out = m(x.to(DEV))
    aux = m.get_aux_outputs()

    def px(a, b, floor=1e-2):  # per-pixel gate of test_gpu_model (floor 1e-2 of the max; see there)
        a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
        return float(((a - b).abs() / b.abs().clamp_min(floor * float(b.abs().max()))).max())

    pairs = ((out, ref), (aux["unetpp"], ref_aux["unetpp"]), (aux["deeplab"], ref_aux["deeplab"]))
    errs = tuple(px(a, b) for a, b in pairs)
    print("dual base96 fp32 per-pixel vs fp64 (fused, unetpp, deeplab), floor 1e-2:", errs, "floor 1e-3:",
          tuple(px(a, b, 1e-3) for a, b in pairs), "max-normalised:", tuple(_rel(a, b) for a, b in pairs))
    assert max(errs) < 1e-3, errs
    sd = m.state_dict()
    for k, v in S.items():
        if "running" in k:
            assert _rel(sd[k], v) < 1e-3, k


def test_dual_base96_train_grads_fp32_vs_oracle():
    """Loss + every parameter gradient of one dual-branch step at base 96 (64^2, B = 2, c = 1,
    K = 2, deep supervision) vs the branch-pinned fp64 oracle, gate as
    test_dual_train_grads_match_oracle."""
    from eunet import synth
    x, msk = synth.batch(2, 64, 64, start_index=23, num_classes=2, in_channels=1)
    keep = _keep96()
    m = _model(96, 1, 2, keep=keep).train()
    loss, pins = _gpu_step(m, x, msk)
    S, loss_ref = _oracle(96, 1, 2, x, msk, keep, torch.float64, pins)
    S32, _ = _oracle(96, 1, 2, x, msk, keep, torch.float32, pins)
    assert abs(loss.item() - loss_ref.item()) < 1e-4 * abs(loss_ref.item())
    rows = _grad_rows(m, S, S32)
    for r in sorted(rows, reverse=True)[:6]:
        print("dual base96 grad (ratio, name, err, tol):", r)
    assert all(r[0] < 1.0 for r in rows), sorted(rows, reverse=True)[:3]


def test_dual_base96_bf16_vs_autocast_reference():
    """bf16 at base 96 vs the fp32 oracle, gated by what bf16 autocast of the oracle achieves."""
    from eunet import synth
    x, _ = synth.batch(2, 64, 64, start_index=25, num_classes=2, in_channels=1)
    keep = _keep96()
    with torch.no_grad():
        ref = D.dual_forward(D.dual_formula_weights(96, 1, 2, dtype=torch.float64), x.double(), True, keep)[0]
        with torch.autocast("cpu", dtype=torch.bfloat16):
            ac = D.dual_forward(D.dual_formula_weights(96, 1, 2, dtype=torch.float32), x, True, keep)[0].float()
    m = _model(96, 1, 2, dtype="bf16", keep=keep).train()
    with torch.no_grad():
        out = m(x.to(DEV)).double().cpu()
    ours, auto = _rel_l2(out, ref), _rel_l2(ac, ref)
    agree = float((out.argmax(1) == ref.argmax(1)).double().mean())
    print("dual base96 bf16 relL2 ours", ours, "autocast", auto, "argmax agreement", agree)
    assert torch.isfinite(out).all()
    assert ours < max(2.0 * auto, 0.02), (ours, auto)


def test_dual_base96_train_grads_bf16_vs_fp64_oracle():
    """bf16 whole-network gradient parity of the dual-branch model at base 96 (64^2, B 2, c 1, K 2,
    deep supervision): every parameter gradient vs the fp64 oracle pinned to the GPU's branch
    configuration (tests/_pins.py) within max(2 x the oracle-under-bf16-autocast error, 3e-2)
    relative L2 (test_gpu_model.test_bf16_train_grads_vs_fp64_oracle's gate).  Pinning removes the
    branch flips between the bf16 run and the fp64 reference; what remains is bf16 rounding, which
    the autocast term measures on the reference itself."""
    from eunet import synth
    x, msk = synth.batch(2, 64, 64, start_index=27, num_classes=2, in_channels=1)
    keep = _keep96()
    m = _model(96, 1, 2, dtype="bf16", keep=keep).train()
    loss, pins = _gpu_step(m, x, msk)
    S, loss_ref = _oracle(96, 1, 2, x, msk, keep, torch.float64, pins, gpu_dtype="bf16")
    Sac = D.dual_formula_weights(96, 1, 2, dtype=torch.float32)
    for k in Sac:
        if Sac[k].is_floating_point() and "running" not in k:
            Sac[k].requires_grad_(True)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        fused, aux = D.dual_forward(Sac, x, training=True, drop_masks=keep)
    D.dual_batch_loss(fused.float(), {n: a.float() for n, a in aux.items()}, msk).backward()
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
        rows.append((e / max(2 * eac, 3e-2), k, e, eac))
    for r in sorted(rows, reverse=True)[:8]:
        print("dual base96 bf16 grad (ratio, name, ours, autocast):", r)
    assert all(r[0] < 1.0 for r in rows), sorted(rows, reverse=True)[:3]
