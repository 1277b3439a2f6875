"""Per-parameter gradient error of the fp32 HIP path vs the fp64 oracle, next to the
fp32 oracle's own error (diagnostic for parity tolerances).

    python tools/grad_diag.py [--base 64] [--cin 1] [--K 2] [--H 64]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402

from oracle import eunet_ref as R  # noqa: E402


def oracle(base, cin, K, x, m, dt):
    S = R.formula_weights(base, cin, K, dtype=dt)
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    R.batch_loss(R.forward(S, x.to(dt), training=True), m).backward()
    return S


def oracle_bufs(base, cin, K, x, dt):
    S = R.formula_weights(base, cin, K, dtype=dt)
    with torch.no_grad():
        R.forward(S, x.to(dt), training=True)
    return S


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", type=int, default=64)
    ap.add_argument("--cin", type=int, default=1)
    ap.add_argument("--K", type=int, default=2)
    ap.add_argument("--H", type=int, default=64)
    a = ap.parse_args()
    from eunet import synth
    from eunet.losses import combined_loss
    from eunet.models import EnhancedUNet
    x, m = synth.batch(2, a.H, a.H, start_index=7, num_classes=a.K, in_channels=a.cin)
    S64 = oracle(a.base, a.cin, a.K, x, m, torch.float64)
    S32 = oracle(a.base, a.cin, a.K, x, m, torch.float32)
    model = EnhancedUNet(num_classes=a.K, in_channels=a.cin, base_ch=a.base)
    fresh = R.formula_weights(a.base, a.cin, a.K, dtype=torch.float64)  # running stats not yet updated
    model.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in fresh.items()})
    model = model.cuda().train()
    logits = model.forward_lowres(x.cuda())
    combined_loss(logits, m.cuda()).backward()
    r = lambda p, q: float((p.double().cpu() - q.double()).norm() / q.double().norm())
    # BN running stats after the training forward = batch statistics of every layer
    S64r = oracle_bufs(a.base, a.cin, a.K, x, torch.float64)
    S32r = oracle_bufs(a.base, a.cin, a.K, x, torch.float32)
    for k, v in model.state_dict().items():
        if "running" in k:
            ours, o32 = r(v, S64r[k]), r(S32r[k], S64r[k])
            if ours > 3 * o32 + 1e-6:
                print(f"BN {k:32s} ours {ours:.2e}  oracle32 {o32:.2e}")
    rl2 = lambda p, q: float((p.double().cpu() - q).norm() / q.norm().clamp_min(1e-30))
    rows = []
    for k, p in model.named_parameters():
        rows.append((rl2(p.grad, S64[k].grad), rl2(S32[k].grad, S64[k].grad), k))
    rows = [r for r in rows if not (r[2].endswith((".0.bias", ".3.bias")) and not r[2].startswith("enhance.3"))]
    for ours, o32, k in sorted(rows, key=lambda r: -r[0] / max(r[1], 1e-30))[:16]:
        print(f"{k:32s} ours {ours:.2e}   oracle32 {o32:.2e}   ratio {ours / max(o32, 1e-30):.1f}")


if __name__ == "__main__":
    main()
