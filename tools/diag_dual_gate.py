"""Diagnostic (not a test): where the bf16 dual-branch step loses the attention gate's gradient.

Runs the base-96 dual model (64^2, B 2, c 1, K 2; tests/test_gpu_dual.py's bf16 gradient case) in
bf16 on the GPU, the fp64 oracle and the oracle under CPU bf16 autocast, and prints the relative L2
error vs fp64 of: the fused / branch logits, g_f2 (d loss / d gated features, split into the fusion
head's dgrad and the residual's part), and the gate's parameter gradients.

    python tools/diag_dual_gate.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import dual_ref as D  # noqa: E402
from oracle import eunet_ref as R  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def oracle(x, msk, keep, dtype, autocast=False):
    S = D.dual_formula_weights(96, 1, 2, dtype=dtype)
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    ctx = torch.autocast("cpu", dtype=torch.bfloat16) if autocast else torch.autocast("cpu", enabled=False)
    with ctx:
        out_main = D.branch_forward(S, "unetpp", x.to(dtype), True)
        out_aux = D.branch_forward(S, "deeplab", x.to(dtype), True)
        ff = torch.cat([out_main, out_aux], 1)
        a = F.conv2d(ff, S["attention_gate.0.weight"], padding=1)
        a = F.gelu(R._bn(S, "attention_gate.1", a, True))
        a = F.conv2d(a, S["attention_gate.3.weight"])
        att = torch.sigmoid(R._bn(S, "attention_gate.4", a, True))
        f2 = ff * att
        f2.retain_grad()
        h = F.relu(R._bn(S, "fusion_head.1", F.conv2d(f2, S["fusion_head.0.weight"], padding=1), True))
        h = D._drop(h, keep[0], D.DROP_P[0], True)
        h = F.relu(R._bn(S, "fusion_head.5", F.conv2d(h, S["fusion_head.4.weight"], padding=1), True))
        h = D._drop(h, keep[1], D.DROP_P[1], True)
        h = F.relu(R._bn(S, "fusion_head.9", F.conv2d(h, S["fusion_head.8.weight"], padding=1), True))
        fused = F.conv2d(h, S["fusion_head.11.weight"], S["fusion_head.11.bias"])
        fused = fused + F.conv2d(f2, S["fusion_residual.weight"], S["fusion_residual.bias"])
    aux = {"unetpp": out_main.float() if autocast else out_main, "deeplab": out_aux.float() if autocast else out_aux}
    loss = D.dual_batch_loss(fused.float() if autocast else fused, aux, msk)
    loss.backward()
    return S, fused.detach(), aux, f2.grad.detach().float()


def main():
    from eunet import ops, synth
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    x, msk = synth.batch(2, 64, 64, start_index=27, num_classes=2, in_channels=1)
    gen = torch.Generator().manual_seed(7)
    keep = ((torch.rand(2, 256, generator=gen) > 0.2).float(), (torch.rand(2, 128, generator=gen) > 0.15).float())
    S64, f64, aux64, g64 = oracle(x, msk, keep, torch.float64)
    Sac, fac, auxac, gac = oracle(x, msk, keep, torch.float32, autocast=True)
    cap = {}
    orig = ops.gate_bwd1

    def spy(za, zb, k, gf2conv, gf2res, *rest):
        cap["conv"] = gf2conv._keep[..., :2 * k].permute(0, 3, 1, 2).float().clone()
        cap["res"] = gf2res.permute(0, 3, 1, 2).float().clone()
        return orig(za, zb, k, gf2conv, gf2res, *rest)

    ops.gate_bwd1 = spy
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=96, dtype="bf16", dual_branch=True)
    m.load_state_dict({k: (v.float() if v.is_floating_point() else v) for k, v in D.dual_formula_weights(96, 1, 2).items()})
    m = m.cuda().train()
    m._engine.drop_keep = keep
    tr = Trainer(m, "cuda", "enhanced_unet")
    out = m(x.cuda())
    aux = m.get_aux_outputs()
    loss = tr.aux_loss(out, aux, msk.cuda())
    loss.backward()
    torch.cuda.synchronize()
    ops.gate_bwd1 = orig
    g_ours = cap["conv"] + cap["res"]
    print("fused logits   ours", rel(out.detach(), f64), "autocast", rel(fac, f64))
    print("unetpp logits  ours", rel(aux["unetpp"].detach(), aux64["unetpp"]), "autocast", rel(auxac["unetpp"], aux64["unetpp"]))
    print("g_f2 total     ours", rel(g_ours, g64), "autocast", rel(gac, g64), "|g64|", float(g64.norm()))
    print("g_f2 conv part |.|", float(cap["conv"].norm()), "res part |.|", float(cap["res"].norm()))
    for k in ("attention_gate.0.weight", "attention_gate.1.weight", "attention_gate.1.bias", "attention_gate.3.weight",
              "attention_gate.4.weight", "attention_gate.4.bias", "fusion_residual.weight", "fusion_head.0.weight"):
        p = dict(m.named_parameters())[k]
        print(f"{k:28s} ours {rel(p.grad, S64[k].grad):.4f}  autocast {rel(Sac[k].grad, S64[k].grad):.4f}  "
              f"|g| {float(S64[k].grad.norm()):.4e}")


if __name__ == "__main__":
    main()
