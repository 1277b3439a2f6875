"""BASELINE.json configs at their own workloads on the GPU (not only in the bench).

configs[1]: base 64, 1 x 512^2 -> 2 classes, batch 8, fp32 (models.py:217-238, train_eval.py:236-353):
  logits per pixel and the loss vs the fp64 oracle, every parameter gradient vs the fp32 CPU oracle --
  both evaluated on the branch configuration the GPU took (tests/_pins.py).
configs[2]: base 64, 1 x 1024^2 -> 2 classes, batch 4, bf16 -- the bench workload: the configs[4] properties
  below at this size (determinism, exact schedules, BN statistics of three layers vs the recomputed conv,
  loss decrease, a 256^2 slice vs the fp64 oracle).
configs[4]: dual-branch base 96 + deep supervision, 2048^2, batch 2, bf16 (models.py:253-333,
  train_eval.py:199-234): an fp64 oracle at this size is out of reach of the host, so full-size
  properties -- finite loss; two runs bit-identical; the side-stream and the serial weight-gradient
  schedules bit-identical; BN running statistics equal to the statistics of the pre-BN conv outputs
  recomputed from the kernels' own operands; the loss decreasing over 3 steps -- plus a 256^2 slice
  of the same model vs the oracle.
"""
import pytest
import torch

from oracle import dual_ref as D
from oracle import eunet_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel_l2(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _rel_px(a, b, floor=1e-2):
    """test_gpu_model's per-pixel gate: |a - b| / max(|b|, floor x max|b|)."""
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float(((a - b).abs() / b.abs().clamp_min(floor * float(b.abs().max()))).max())


def _pre_bn_bias(k):
    return k.endswith((".0.bias", ".3.bias")) and not k.startswith("enhance.3")


def test_configs1_fp32_512_batch8_vs_oracle():
    """BASELINE configs[1] (base 64, c 1, K 2, fp32, 512^2, B 8): one training step.
    Logits [8,2,512,512] per pixel within 1e-3 of the fp64 oracle (floor 1e-2 of max|ref|, as every
    per-pixel gate here), loss within 1e-4; every parameter gradient within 1e-3 relative L2 of the
    pinned fp32 CPU oracle (conv biases ahead of a BatchNorm, whose true gradient is 0, against the
    global gradient scale).  The fp64 backward at this size is left out (host time)."""
    import _pins
    from eunet import synth
    from eunet.losses import combined_loss
    from eunet.models import EnhancedUNet
    x, msk = synth.batch(8, 512, 512, start_index=41, num_classes=2, in_channels=1)
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64, dtype="fp32")
    m.load_state_dict({k: (v.float() if v.is_floating_point() else v) for k, v in R.formula_weights(64, 1, 2).items()})
    m = _pins.keep(m.to(DEV).train())
    logits = m.forward_lowres(x.to(DEV))
    loss = combined_loss(logits, msk.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    pins = _pins.model_pins(m)
    m._engine.last_state = None
    logits = logits.detach().cpu()
    rec = {}
    with torch.no_grad():
        S64 = R.formula_weights(64, 1, 2)
        out64 = R.forward(S64, x.double(), training=True, pins=pins, record=rec)
        loss64 = R.batch_loss(out64, msk)
        ref64 = torch.nn.functional.avg_pool2d(out64, 2)
        del out64
    # the pins are the oracle's own branches up to fp32 rounding (tests/_pins.audit)
    _pins.audit(pins, rec, "fp32", label="configs[1]")
    del rec
    px = _rel_px(logits, ref64)
    print("configs[1] logits per-pixel vs pinned fp64:", px, "loss", loss.item(), float(loss64))
    assert px < 1e-3
    assert abs(loss.item() - float(loss64)) < 1e-4 * abs(float(loss64))
    # UNPINNED: the plain fp64 oracle (its own branches everywhere).  Pixels downstream of a disputed kink
    # are those where the pinned and the unpinned fp64 oracles themselves differ (> 1e-4, same per-pixel
    # measure); outside that reported set the GPU logits meet the 1e-3 per-pixel gate against the plain
    # reference forward.
    with torch.no_grad():
        ref64u = torch.nn.functional.avg_pool2d(R.forward(R.formula_weights(64, 1, 2), x.double(), training=True), 2)
    den = ref64u.abs().clamp_min(1e-2 * float(ref64u.abs().max()))
    near = ((ref64 - ref64u).abs() / den) > 1e-4
    pxu = ((logits.double() - ref64u).abs() / den)
    n_near = int(near.sum())
    pxu_out = float(pxu[~near].max())
    print(f"configs[1] logits per-pixel vs UNPINNED fp64: {pxu_out:.2e} outside {n_near} of {near.numel()} "
          f"logits downstream of disputed kinks (all: {float(pxu.max()):.2e})")
    assert pxu_out < 1e-3
    assert n_near <= 1e-3 * near.numel(), n_near
    del ref64, ref64u, pxu, near, den
    S = R.formula_weights(64, 1, 2, dtype=torch.float32)
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    R.batch_loss(R.forward(S, x, training=True, pins=pins), msk).backward()
    scale = max(float(S[k].grad.abs().max()) for k in S if S[k].grad is not None)
    rows = []
    for k, p in m.named_parameters():
        ref = S[k].grad
        if _pre_bn_bias(k):
            assert float((p.grad.double().cpu() - ref.double()).abs().max()) < 1e-4 * scale, k
            continue
        rows.append((_rel_l2(p.grad, ref), k))
    for r in sorted(rows, reverse=True)[:5]:
        print("configs[1] grad vs pinned fp32 oracle (relL2, name):", r)
    assert all(r[0] < 1e-3 for r in rows), sorted(rows, reverse=True)[:3]
    for k, v in m.state_dict().items():
        if "running" in k:
            assert _rel_l2(v, S[k]) < 1e-4, k


# ---- configs[4]: dual-branch base 96, 2048^2, B 2, bf16 ---------------------------------------------------
B4, H4 = 2, 2048


def _keep(seed=3):
    gen = torch.Generator().manual_seed(seed)
    return ((torch.rand(B4, 256, generator=gen) > 0.2).float(), (torch.rand(B4, 128, generator=gen) > 0.15).float())


def _dual96(dtype="bf16"):
    from eunet.models import EnhancedUNet
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=96, dtype=dtype, dual_branch=True)
    m.load_state_dict({k: (v.float() if v.is_floating_point() else v)
                       for k, v in D.dual_formula_weights(96, 1, 2).items()})
    m = m.to(DEV).train()
    m._engine.drop_keep = _keep()
    return m


@pytest.fixture(scope="module")
def cfg4_batch():
    from eunet import synth
    x, msk = synth.batch(B4, H4, H4, start_index=61, num_classes=2, in_channels=1)
    return x.to(DEV), msk.to(DEV)


def _grads(m, x, msk):
    from eunet.train_eval import Trainer
    tr = Trainer(m, DEV, "enhanced_unet")
    loss = tr.aux_loss(m(x), m.get_aux_outputs(), msk)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}


def test_configs4_dual96_2048_deterministic_and_schedules_exact(cfg4_batch, monkeypatch):
    """configs[4] workload: the loss is finite, two runs from the same weights / dropout masks give
    bit-identical losses and gradients, and so does the serial schedule (weight gradients on the
    launch stream, UNetEngine.overlap_wgrad = False) -- at 2048^2 the grids, split counts and the
    > 2 GiB per-sample conv slices (dec2.0 input: 2048^2 x 288 channels) are the production ones."""
    from eunet import engine
    x, msk = cfg4_batch
    l1, g1 = _grads(_dual96(), x, msk)
    assert torch.isfinite(l1).all()
    assert all(torch.isfinite(g).all() for g in g1.values())
    l2, g2 = _grads(_dual96(), x, msk)
    assert torch.equal(l1, l2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), ("rerun", k)
    del g2
    monkeypatch.setattr(engine.UNetEngine, "overlap_wgrad", False)
    l3, g3 = _grads(_dual96(), x, msk)
    assert torch.equal(l1, l3)
    for k in g1:
        assert torch.equal(g1[k], g3[k]), ("serial schedule", k)


def test_configs4_bn_running_stats_match_recomputed_conv(cfg4_batch):
    """One training forward at the configs[4] size from fresh running statistics (mean 0, var 1):
    running_mean = 0.1 mean, running_var = 0.9 + 0.1 unbiased var of the layer's pre-BN conv output,
    with the output recomputed from the kernels' own operands: unetpp.enc1.1 (enc1.0, the 1 -> 96
    direct conv of the bf16 input, in fp64) and unetpp.enc1.4 (enc1.3, 96 -> 96 on the MFMA kernel, its
    operand bf16(relu(ya * scale + shift)) and bf16 weights, conv in fp32) over 2 x 2048^2 pixels.  The
    kernels reduce their fp32 accumulators before any rounding, so the statistics of the stored bf16
    tensor would NOT do as a reference (rounding adds ~5e-6 (1 + mean^2 / var) to the variance: 1.2e-3
    on enc1.0, whose mean is large against its spread on the bright-field input).  Checked: the batch
    mean and 1/std the step normalised with, and the running statistics they updated."""
    import _pins
    import torch.nn.functional as F
    x, _ = cfg4_batch
    m = _pins.keep(_dual96())
    with torch.enable_grad():
        m(x)
    S = m._engine.last_state["SA"]
    sd = m.state_dict()
    P = dict(m.named_parameters())
    xin = S["xin"].permute(0, 3, 1, 2).double()                          # the kernels' bf16 input
    y1 = F.conv2d(xin, P["unetpp.enc1.0.weight"].double(), P["unetpp.enc1.0.bias"].double(), padding=1)
    ya, bna = S["enc1"]["ya"], S["enc1"]["bna"]
    za = torch.relu(ya.float() * bna["scale"] + bna["shift"]).bfloat16().float().permute(0, 3, 1, 2)
    w3 = P["unetpp.enc1.3.weight"].bfloat16().float()
    y3 = F.conv2d(za, w3, P["unetpp.enc1.3.bias"].float(), padding=1)
    del za
    for key, y, bn in (("unetpp.enc1.1", y1, S["enc1"]["bna"]), ("unetpp.enc1.4", y3, S["enc1"]["bnb"])):
        yd = y.double().transpose(0, 1).reshape(y.shape[1], -1)
        n = yd.shape[1]
        mean, var = yd.mean(1), yd.var(1, unbiased=True)
        std = var.sqrt()
        # the step's batch statistics (bn_finalize's mean / 1/std, fp32) ...
        em = float(((bn["mean"].double() - mean).abs() / std).max())
        ei = float(((bn["invstd"].double() - 1.0 / torch.sqrt(var * (n - 1) / n + 1e-5)).abs()
                    * torch.sqrt(var * (n - 1) / n + 1e-5)).max())
        # ... and the running statistics they updated (momentum 0.1, unbiased variance); these are fp32
        # numbers near 0.9 + 0.1 var, so their own representation (2^-24 relative) is allowed for
        rm, rv = sd[key + ".running_mean"].double(), sd[key + ".running_var"].double()
        ref_rv = 0.9 + 0.1 * var
        erm = float(((rm - 0.1 * mean).abs() / (0.1 * std)).max())
        erv = float(((rv - ref_rv).abs() / (1e-4 * 0.1 * var + 2.0 ** -23 * ref_rv)).max())
        print(f"configs[4] {key} ({n} px): batch mean err / std {em:.2e}, 1/std rel err {ei:.2e}; running mean "
              f"err / std {erm:.2e}, running var err / (1e-4 x 0.1 var + fp32 ulp) {erv:.2f}")
        assert em < 1e-4 and ei < 1e-4 and erm < 1e-4 and erv < 1.0, (key, em, ei, erm, erv)
    m._engine.last_state = None


def test_configs4_loss_decreases_over_three_steps(cfg4_batch):
    """Three Trainer.steps (clip, AdamW at lr 1e-3) on the configs[4] batch with fixed dropout masks:
    the loss decreases at every step."""
    from eunet.train_eval import Trainer
    x, msk = cfg4_batch
    m = _dual96()
    tr = Trainer(m, DEV, "enhanced_unet")
    for g in tr.optimizer.param_groups:
        g["lr"] = 1e-3
    losses = [tr.step(x, msk) for _ in range(4)]
    print("configs[4] losses:", losses)
    assert all(b < a for a, b in zip(losses, losses[1:])), losses


def test_configs4_256_slice_vs_oracle(cfg4_batch):
    """A 256^2 crop of the configs[4] batch through the same bf16 base-96 model (train mode, the same
    dropout masks) vs the fp64 oracle, gated by what bf16 autocast of the oracle achieves on the same
    crop (test_gpu_dual.test_dual_base96_bf16_vs_autocast_reference's gate), plus argmax agreement."""
    x, _ = cfg4_batch
    xs = x[:, :, 768:1024, 1024:1280].contiguous()
    m = _dual96()
    with torch.no_grad():
        out = m(xs).double().cpu()
    keep = _keep()
    xc = xs.cpu()
    with torch.no_grad():
        ref = D.dual_forward(D.dual_formula_weights(96, 1, 2), xc.double(), True, keep)[0]
        with torch.autocast("cpu", dtype=torch.bfloat16):
            ac = D.dual_forward(D.dual_formula_weights(96, 1, 2, dtype=torch.float32), xc, True, keep)[0].float()
    ours, auto = _rel_l2(out, ref), _rel_l2(ac, ref)
    agree = float((out.argmax(1) == ref.argmax(1)).double().mean())
    agree_ac = float((ac.argmax(1) == ref.argmax(1)).double().mean())
    print("configs[4] 256^2 slice bf16 relL2 ours", ours, "autocast", auto, "argmax agreement", agree, agree_ac)
    assert torch.isfinite(out).all()
    assert ours < max(2.0 * auto, 0.02), (ours, auto)
    assert agree > min(0.97, agree_ac - 0.02), (agree, agree_ac)


# ---- configs[2]: base 64, 1 x 1024^2 -> 2 classes, batch 4, bf16 (the bench workload) ----------------------
# The headline config at its own size (models.py:217-238, train_eval.py:236-353).  An fp64 oracle of the full
# step is out of reach of the host here too, so the configs[4] suite's full-size properties are applied to it:
# determinism and the exact schedules, BN statistics against the conv recomputed from the kernels' own bf16
# operands at three layers (64 -> 64 at 1024^2, 512 -> 512 at 128^2, the 192 -> 64 concat input of dec2.0),
# the loss decreasing over three Trainer steps, and a 256^2 slice of the same model against the fp64 oracle.
B2, H2 = 4, 1024


def _base64(dtype="bf16"):
    from eunet.models import EnhancedUNet
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64, dtype=dtype)
    m.load_state_dict({k: (v.float() if v.is_floating_point() else v) for k, v in R.formula_weights(64, 1, 2).items()})
    return m.to(DEV).train()


@pytest.fixture(scope="module")
def cfg2_batch():
    from eunet import synth
    x, msk = synth.batch(B2, H2, H2, start_index=71, num_classes=2, in_channels=1)
    return x.to(DEV), msk.to(DEV)


def _grads2(m, x, msk):
    from eunet.losses import combined_loss
    loss = combined_loss(m.forward_lowres(x), msk)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}


def test_configs2_deterministic_and_schedules_exact(cfg2_batch, monkeypatch):
    """configs[2] workload: finite loss and gradients; a second run from the same weights is bit-identical,
    and so is the serial schedule (weight gradients on the launch stream: UNetEngine.overlap_wgrad = False)."""
    from eunet import engine
    x, msk = cfg2_batch
    l1, g1 = _grads2(_base64(), x, msk)
    assert torch.isfinite(l1).all()
    assert all(torch.isfinite(g).all() for g in g1.values())
    l2, g2 = _grads2(_base64(), x, msk)
    assert torch.equal(l1, l2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), ("rerun", k)
    del g2
    monkeypatch.setattr(engine.UNetEngine, "overlap_wgrad", False)
    l3, g3 = _grads2(_base64(), x, msk)
    assert torch.equal(l1, l3)
    for k in g1:
        assert torch.equal(g1[k], g3[k]), ("serial schedule", k)


def test_configs2_bn_running_stats_match_recomputed_conv(cfg2_batch):
    """One training forward at the configs[2] size from fresh running statistics: the batch mean / 1/std and
    the running statistics of model.enc1.4 (enc1.3: 64 -> 64 at 1024^2), model.enc4.4 (enc4.3: 512 -> 512 at
    128^2) and model.dec2.1 (dec2.0 over the 192-channel concat buffer [skip | upsampled], 1024^2) against the
    statistics of the pre-BN conv output recomputed from the kernels' own operands: the bf16 operand as staged
    (bf16(relu(fmaf(ya, scale, shift))) for a .3 conv, the stored concat buffer for dec2.0) and the bf16
    weights, conv in fp32 (TF32 off) -- the kernels take the statistics from their fp32 accumulators."""
    import _pins
    import torch.nn.functional as F
    x, _ = cfg2_batch
    m = _pins.keep(_base64())
    with torch.enable_grad():
        m.forward_lowres(x)
    S = m._engine.last_state
    sd = m.state_dict()
    P = dict(m.named_parameters())
    tf32 = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = False
    try:
        for key, blk, conv in (("model.enc1.4", "enc1", "model.enc1.3"), ("model.enc4.4", "enc4", "model.enc4.3"),
                               ("model.dec2.1", "dec2", "model.dec2.0")):
            s = S[blk]
            if conv.endswith(".3"):
                ya, bna = s["ya"], s["bna"]
                inp = torch.relu(torch.addcmul(bna["shift"], ya.float(), bna["scale"]))  # fmaf, as the kernels
                inp = inp.bfloat16().float().permute(0, 3, 1, 2)
                bn = s["bnb"]
            else:
                X = s["X"]
                inp = X._keep[..., X.coff:X.coff + X.c].float().permute(0, 3, 1, 2)
                bn = s["bna"]
            y = F.conv2d(inp, P[conv + ".weight"].bfloat16().float(), P[conv + ".bias"].float(), padding=1)
            del inp
            yd = y.transpose(0, 1).reshape(y.shape[1], -1).double()
            del y
            n = yd.shape[1]
            mean, var = yd.mean(1), yd.var(1, unbiased=True)
            del yd
            std = var.sqrt()
            vb = var * (n - 1) / n
            em = float(((bn["mean"].double() - mean).abs() / std).max())
            ei = float(((bn["invstd"].double() - 1.0 / torch.sqrt(vb + 1e-5)).abs() * torch.sqrt(vb + 1e-5)).max())
            rm, rv = sd[key + ".running_mean"].double(), sd[key + ".running_var"].double()
            ref_rv = 0.9 + 0.1 * var
            erm = float(((rm - 0.1 * mean).abs() / (0.1 * std)).max())
            erv = float(((rv - ref_rv).abs() / (1e-4 * 0.1 * var + 2.0 ** -23 * ref_rv)).max())
            print(f"configs[2] {key} ({n} px): batch mean err / std {em:.2e}, 1/std rel err {ei:.2e}; running mean "
                  f"err / std {erm:.2e}, running var err / (1e-4 x 0.1 var + fp32 ulp) {erv:.2f}")
            assert em < 1e-4 and ei < 1e-4 and erm < 1e-4 and erv < 1.0, (key, em, ei, erm, erv)
    finally:
        torch.backends.cudnn.allow_tf32 = tf32
        m._engine.last_state = None


def test_configs2_loss_decreases_bf16_tracks_fp32(cfg2_batch):
    """Five Trainer.steps (clip, native AdamW at lr 3e-4) on the configs[2] batch in bf16 and in fp32 (the
    precision the oracle tests pin at configs[1]): the loss decreases at every step in both, and the bf16 loss
    trajectory stays within 2e-3 relative of the fp32 one (measured 2.6e-4 .. 4.8e-4).  At lr 1e-3 both
    precisions rise after the first step alike (14.30 -> 14.90 bf16, 14.30 -> 14.90 fp32:
    tools/cfg2_loss_probe.py) -- optimisation dynamics, not a precision effect."""
    from eunet.train_eval import Trainer
    x, msk = cfg2_batch
    traj = {}
    for dt in ("bf16", "fp32"):
        tr = Trainer(_base64(dt), DEV, "enhanced_unet")
        for g in tr.optimizer.param_groups:
            g["lr"] = 3e-4
        traj[dt] = [tr.step(x, msk) for _ in range(5)]
        del tr
        torch.cuda.empty_cache()
    print("configs[2] losses bf16:", traj["bf16"], "fp32:", traj["fp32"])
    for dt in traj:
        assert all(b < a for a, b in zip(traj[dt], traj[dt][1:])), (dt, traj[dt])
    rel = max(abs(a - b) / abs(b) for a, b in zip(traj["bf16"], traj["fp32"]))
    assert rel < 2e-3, (rel, traj)


def test_configs2_256_slice_vs_oracle(cfg2_batch):
    """A 256^2 crop of the configs[2] batch through the same bf16 base-64 model (train mode) vs the fp64
    oracle, gated by what CPU bf16 autocast of the oracle achieves on the same crop, plus argmax agreement."""
    x, _ = cfg2_batch
    xs = x[:, :, 512:768, 256:512].contiguous()
    m = _base64()
    with torch.no_grad():
        out = m(xs).double().cpu()
    xc = xs.cpu()
    with torch.no_grad():
        ref = R.forward(R.formula_weights(64, 1, 2), xc.double(), training=True)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            ac = R.forward(R.formula_weights(64, 1, 2, dtype=torch.float32), xc, training=True).float()
    ours, auto = _rel_l2(out, ref), _rel_l2(ac, ref)
    agree = float((out.argmax(1) == ref.argmax(1)).double().mean())
    agree_ac = float((ac.argmax(1) == ref.argmax(1)).double().mean())
    print("configs[2] 256^2 slice bf16 relL2 ours", ours, "autocast", auto, "argmax agreement", agree, agree_ac)
    assert torch.isfinite(out).all()
    assert ours < max(2.0 * auto, 0.02), (ours, auto)
    assert agree > min(0.97, agree_ac - 0.02), (agree, agree_ac)
