"""Diagnostic (GPU box): the enc1.0 bias gradient at 256^2 B=2 (base 64, c 1, K 2, fp32).

Captures the dY the engine hands to conv_small_wgrad (the gradient w.r.t. enc1's pre-BN conv
output y_a) and compares (1) the kernel's bias gradient with an fp64 host column sum of that
same dY, (2) that dY with the fp64 oracle's gradient w.r.t. y_a.  Not part of the product.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import eunet_ref as R  # noqa: E402


def main():
    from eunet import ops, synth
    from eunet.losses import combined_loss
    from eunet.models import EnhancedUNet
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dt = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    x, msk = synth.batch(2, H, H, start_index=9, num_classes=2, in_channels=1)
    # fp64 oracle with a hook on enc1's pre-BN conv output
    S = R.formula_weights(64, 1, 2)
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    cap = {}
    orig_conv = F.conv2d

    def conv_hook(inp, w, b=None, *a, **kw):
        y = orig_conv(inp, w, b, *a, **kw)
        if w is S["model.enc1.0.weight"]:
            y.retain_grad()
            cap["ya"] = y
        return y

    F.conv2d = conv_hook
    try:
        loss = R.batch_loss(R.forward(S, x.double(), training=True), msk)
        loss.backward()
    finally:
        F.conv2d = orig_conv
    g64 = cap["ya"].grad  # [N, 64, H, W]

    got = {}
    orig = ops.conv_small_wgrad

    def spy(xa, dya, dw_part, db_part, nsplit):
        orig(xa, dya, dw_part, db_part, nsplit)
        if "dy" not in got:
            got["dy"] = dya._keep.detach().double().cpu().clone()
            torch.cuda.synchronize()
            got["db_part"] = db_part.detach().double().cpu().clone().view(nsplit, -1)

    ops.conv_small_wgrad = spy
    try:
        m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64, dtype=dt)
        m.load_state_dict({k: v.detach().float() if v.is_floating_point() else v for k, v in S.items()})
        m = m.cuda().train()
        combined_loss(m.forward_lowres(x.cuda()), msk.cuda()).backward()
        torch.cuda.synchronize()
    finally:
        ops.conv_small_wgrad = orig
    dy = got["dy"]  # NHWC [N, H, W, 64]
    host_db = dy.sum((0, 1, 2))
    kern_db = got["db_part"].sum(0)
    ref = g64.permute(0, 2, 3, 1)
    print("kernel db vs host fp64 sum of the same dY: max abs", float((kern_db - host_db).abs().max()),
          "at channel", int((kern_db - host_db).abs().argmax()))
    print("host sum of dY (should be ~0):", [round(float(v), 6) for v in host_db[:8]], "max",
          float(host_db.abs().max()), "argmax", int(host_db.abs().argmax()))
    print("grad bias from model:", float(m.model.enc1[0].bias.grad.abs().max()),
          int(m.model.enc1[0].bias.grad.abs().argmax()))
    d = (dy - ref).abs()
    print("dY vs fp64 oracle dL/dya: max-normalised", float(d.max() / ref.abs().max()))
    per_c = d.amax((0, 1, 2)) / ref.abs().amax((0, 1, 2))
    print("per channel worst (rel to channel max):", [(int(c), float(per_c[c])) for c in per_c.argsort(descending=True)[:5]])
    c = int(host_db.abs().argmax())
    print(f"channel {c}: sum dY ours {float(dy[..., c].sum()):.6g} oracle {float(ref[..., c].sum()):.3g}; "
          f"mean dY ours {float(dy[..., c].mean()):.3g}; |dY| max {float(dy[..., c].abs().max()):.4g}")
    diff = (dy[..., c] - ref[..., c])
    print(f"channel {c}: mean(diff) {float(diff.mean()):.4g} std(diff) {float(diff.std()):.4g}")


if __name__ == "__main__":
    main()
