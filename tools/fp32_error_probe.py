"""Diagnostic (GPU box): where does the fp32 path's error vs the fp64 oracle grow?

For one 256^2 B=2 train-mode forward (base 64, c 1, K 2) prints, per DoubleConv, the
max-normalised error of the pre-BatchNorm conv outputs y_a, y_b of the HIP engine and of the
fp32 CPU oracle, both against the fp64 oracle (same input and formula weights), then z =
dec1(d2) and the logits.  Not part of the product or the tests.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import eunet_ref as R  # noqa: E402


def oracle_levels(S, x):
    """models.py:227-238 with every pre-BN conv output kept (NCHW)."""
    pre = {}

    def dc(name, h):
        p = f"model.{name}"
        ya = F.conv2d(h, S[p + ".0.weight"], S[p + ".0.bias"], padding=1)
        h = F.relu(R._bn(S, p + ".1", ya, True))
        yb = F.conv2d(h, S[p + ".3.weight"], S[p + ".3.bias"], padding=1)
        pre[name] = (ya, yb)
        return F.relu(R._bn(S, p + ".4", yb, True))

    up = R._up2
    e1 = dc("enc1", x)
    e2 = dc("enc2", F.max_pool2d(e1, 2))
    e3 = dc("enc3", F.max_pool2d(e2, 2))
    e4 = dc("enc4", F.max_pool2d(e3, 2))
    d4 = dc("dec4", torch.cat([up(e4), e3], 1))
    d3 = dc("dec3", torch.cat([up(d4), e2], 1))
    d2 = dc("dec2", torch.cat([up(d3), e1], 1))
    z = F.conv2d(d2, S["model.dec1.weight"], S["model.dec1.bias"])
    return pre, z


def err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max())


def main():
    from eunet import synth
    from eunet.models import EnhancedUNet
    x, _ = synth.batch(2, 256, 256, start_index=9, num_classes=2, in_channels=1)
    S64 = R.formula_weights(64, 1, 2)
    S32 = R.formula_weights(64, 1, 2, dtype=torch.float32)
    with torch.no_grad():
        p64, z64 = oracle_levels(S64, x.double())
        p32, z32 = oracle_levels(S32, x)
        out64 = R.forward(R.formula_weights(64, 1, 2), x.double(), True)
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64)
    m.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in R.formula_weights(64, 1, 2).items()})
    m = m.cuda().train()
    with torch.no_grad():
        out, S = m._engine.forward(x.cuda(), training=True, want="out2h")
    print(f"{'block':6s} {'gpu ya':>10s} {'cpu32 ya':>10s} {'gpu yb':>10s} {'cpu32 yb':>10s}   bn-b |mean|/std max")
    for nm in ("enc1", "enc2", "enc3", "enc4", "dec4", "dec3", "dec2"):
        ya = S[nm]["ya"].permute(0, 3, 1, 2)
        yb = S[nm]["yb"].permute(0, 3, 1, 2)
        r64 = p64[nm][1]
        ms = float((r64.mean((0, 2, 3)).abs() / r64.std((0, 2, 3))).max())
        print(f"{nm:6s} {err(ya, p64[nm][0]):10.2e} {err(p32[nm][0], p64[nm][0]):10.2e} "
              f"{err(yb, p64[nm][1]):10.2e} {err(p32[nm][1], p64[nm][1]):10.2e}   {ms:8.2f}")
    print("z     ", f"{err(S['z'].permute(0, 3, 1, 2), z64):10.2e} {err(z32, z64):10.2e}")
    print("out2h ", f"{err(out, out64):10.2e}")


if __name__ == "__main__":
    main()
