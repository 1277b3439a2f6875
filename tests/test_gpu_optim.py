"""Native clip_grad_norm_ + AdamW (eunet.optim.ClipAdamW, csrc/optim.hip) against PyTorch's
clip_grad_norm_(foreach) + AdamW(fused) -- the reference's train_eval.py:341-343 on the optimizer of
:120 -- over several steps with learning-rate changes, clipping active and inactive (GPU only)."""
import copy
import re

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
SHAPES = [(64, 1, 3, 3), (64,), (3,), (1,), (2049,), (128, 64, 3, 3), (70001,), (2, 64), (512, 256, 3, 3)]


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _pair(seed, lr=4e-3, wd=1e-4):
    g = torch.Generator(device="cpu").manual_seed(seed)
    base = [torch.randn(s, generator=g) * 0.1 for s in SHAPES]
    pa = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
    pb = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
    oa = torch.optim.AdamW(pa, lr=lr, weight_decay=wd, betas=(0.9, 0.999), fused=True)
    ob = torch.optim.AdamW(pb, lr=lr, weight_decay=wd, betas=(0.9, 0.999), fused=True)
    return g, pa, pb, oa, ob


@pytest.mark.parametrize("gscale", [1.0, 1e-3])  # total norm >> 1 (clipped) / < 1 (coefficient 1)
def test_clip_adamw_matches_torch(gscale):
    from eunet.optim import ClipAdamW, supported
    g, pa, pb, oa, ob = _pair(3)
    assert supported(ob)
    native = ClipAdamW(ob)
    for it, lr in enumerate([4e-3, 4e-3, 1e-3, 2.5e-4]):
        for o in (oa, ob):
            o.param_groups[0]["lr"] = lr
        grads = [torch.randn(p.shape, generator=g) * gscale for p in pa]
        for p, q, gr in zip(pa, pb, grads):
            p.grad = gr.to(DEV)
            q.grad = gr.to(DEV)
        na = torch.nn.utils.clip_grad_norm_(pa, max_norm=1.0, foreach=True)
        oa.step()
        nb = native.step(1.0)
        torch.cuda.synchronize()
        assert rel(nb, na) < 1e-6, it
        for p, q in zip(pa, pb):
            assert rel(q.grad, p.grad) < 1e-6, (it, p.shape)  # p.grad left clipped
            assert rel(q, p) < 1e-6, (it, p.shape)
            sa, sb = oa.state[p], ob.state[q]
            assert float(sa["step"]) == float(sb["step"]) == it + 1
            assert sb["step"].dtype == torch.float32 and sb["step"].is_cuda
            assert rel(sb["exp_avg"], sa["exp_avg"]) < 1e-6, (it, p.shape)
            assert rel(sb["exp_avg_sq"], sa["exp_avg_sq"]) < 1e-6, (it, p.shape)
    # torch's own step continues from the native state (same layout), and state_dict round-trips
    ob.load_state_dict(copy.deepcopy(oa.state_dict()))  # (shallow: the two would share state tensors)
    for p, q in zip(pa, pb):
        gr = torch.randn(p.shape, generator=g).to(DEV)
        p.grad, q.grad = gr.clone(), gr.clone()
    oa.step()
    ob.step()
    for p, q in zip(pa, pb):
        assert rel(q, p) < 1e-6


def test_clip_adamw_skips_parameters_without_grad():
    from eunet.optim import ClipAdamW
    g, pa, pb, oa, ob = _pair(4)
    native = ClipAdamW(ob)
    for p, q in zip(pa, pb):
        if p.dim() == 1 and p.numel() < 10:
            continue  # no gradient: torch skips the parameter (no state, no update)
        gr = torch.randn(p.shape, generator=g).to(DEV)
        p.grad, q.grad = gr.clone(), gr.clone()
    na = torch.nn.utils.clip_grad_norm_([p for p in pa if p.grad is not None], max_norm=1.0, foreach=True)
    oa.step()
    nb = native.step(1.0)
    assert rel(nb, na) < 1e-6
    for p, q in zip(pa, pb):
        assert (q in ob.state) == (p in oa.state)
        assert rel(q, p) < 1e-6


def test_trainer_native_step_matches_torch_path():
    """Trainer.step with the native optimizer step vs Trainer.native_clip_adamw = False (torch's
    clip_grad_norm_ + fused AdamW), same seeded model and batches: parameters after 3 steps."""
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    torch.manual_seed(0)
    x = torch.rand(2, 1, 64, 64, device=DEV)
    m = torch.randint(0, 2, (2, 64, 64), device=DEV)
    out = []
    for native in (True, False):
        torch.manual_seed(1)
        model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16).to(DEV)
        tr = Trainer(model, DEV, "enhanced_unet", total_epochs=50)
        tr.native_clip_adamw = native
        tr.epoch_lr_step(0)
        for _ in range(3):
            tr.step(x, m, sync_loss=False)
        assert tr._native_opt() == native
        out.append({k: v.detach().clone() for k, v in model.state_dict().items()})
    for k in out[0]:
        # the biases of the convs feeding a BatchNorm get gradients of rounding noise (BN removes
        # them), which AdamW normalises to +-lr steps of arbitrary sign: not comparable
        if out[0][k].is_floating_point() and not re.search(r"\.[03]\.bias$", k):
            assert rel(out[0][k], out[1][k]) < 1e-4, k


def test_plain_foreach_adamw_is_not_taken():
    """The reference's plain optim.AdamW(...) (foreach, not capturable) keeps CPU step counters once torch
    has stepped it: the native path refuses it, and the Trainer then runs torch's clip + step."""
    from eunet.optim import ClipAdamW, supported
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in SHAPES[:4]]
    o = torch.optim.AdamW(ps, lr=1e-3, foreach=True)
    for p in ps:
        p.grad = torch.randn_like(p)
    o.step()
    assert not o.state[ps[0]]["step"].is_cuda  # the hazard the check guards against
    assert not supported(o)
    with pytest.raises(ValueError):
        ClipAdamW(o)


def test_capturable_adamw_after_torch_step_and_cpu_state():
    """A capturable AdamW stepped by torch first, then natively; and a state whose step counter was
    loaded onto the CPU (load_state_dict of a CPU-mapped checkpoint) is moved to the device first."""
    from eunet.optim import ClipAdamW, supported
    g = torch.Generator(device="cpu").manual_seed(7)
    base = [torch.randn(s, generator=g) * 0.1 for s in SHAPES]
    pa = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
    pb = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
    oa = torch.optim.AdamW(pa, lr=4e-3, weight_decay=1e-4, capturable=True)
    ob = torch.optim.AdamW(pb, lr=4e-3, weight_decay=1e-4, capturable=True)
    assert supported(ob)
    for it in range(3):
        grads = [torch.randn(p.shape, generator=g) for p in pa]
        for p, q, gr in zip(pa, pb, grads):
            p.grad, q.grad = gr.to(DEV), gr.to(DEV)
        torch.nn.utils.clip_grad_norm_(pa, max_norm=1.0, foreach=True)
        if it == 1:
            # the native step restates torch's FUSED AdamW (bias corrections and hyper-parameter products in
            # double, narrowed to fp32).  capturable foreach AdamW forms the bias corrections as fp32 tensor
            # ops instead, so it differs from both in the step size's last bits (1.1e-6 relative after two
            # steps, round 5).  The reference therefore continues from the capturable optimizer's state with a
            # fused AdamW, which computes exactly what the native step computes.
            fused = torch.optim.AdamW(pa, lr=4e-3, weight_decay=1e-4, fused=True)
            for p in pa:  # (the state only: load_state_dict would also restore the param-group flags)
                fused.state[p] = {k: v.clone() for k, v in oa.state[p].items()}
            oa = fused
        oa.step()
        if it == 0:  # torch's own first step on ob, then a CPU step counter on one tensor
            torch.nn.utils.clip_grad_norm_(pb, max_norm=1.0, foreach=True)
            ob.step()
            ob.state[pb[1]]["step"] = ob.state[pb[1]]["step"].cpu()
            native = ClipAdamW(ob)
        else:
            native.step(1.0)
        torch.cuda.synchronize()
        for p, q in zip(pa, pb):
            assert rel(q, p) < 1e-6, (it, p.shape)
            assert ob.state[q]["step"].is_cuda or it == 0
            assert float(ob.state[q]["step"]) == it + 1


def test_clip_adamw_nan_gradient_poisons_like_torch():
    """A NaN gradient element: torch's clamp(max=1) keeps the NaN coefficient, so every clipped
    gradient and every updated parameter becomes NaN; the native step does the same."""
    from eunet.optim import ClipAdamW
    g, pa, pb, oa, ob = _pair(5)
    native = ClipAdamW(ob)
    for p, q in zip(pa, pb):
        gr = torch.randn(p.shape, generator=g).to(DEV)
        p.grad, q.grad = gr.clone(), gr.clone()
    pa[3].grad.view(-1)[0] = float("nan")
    pb[3].grad.view(-1)[0] = float("nan")
    torch.nn.utils.clip_grad_norm_(pa, max_norm=1.0, foreach=True)
    oa.step()
    native.step(1.0)
    torch.cuda.synchronize()
    for p, q in zip(pa, pb):
        assert torch.isnan(p).all() and torch.isnan(q).all()
        assert torch.isnan(q.grad).all()
