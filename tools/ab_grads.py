"""A/B two library builds on one train step (fp32): per-parameter gradient rel-L2 vs the
fp64 oracle for each build, and between the builds.

    python tools/ab_grads.py LIB_A LIB_B [--base 64 --cin 1 --K 2 --H 64]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]


def dump(a, out):
    import torch
    from oracle import eunet_ref as R
    from eunet import synth
    from eunet.losses import combined_loss
    from eunet.models import EnhancedUNet
    x, m = synth.batch(2, a.H, a.H, start_index=7, num_classes=a.K, in_channels=a.cin)
    model = EnhancedUNet(num_classes=a.K, in_channels=a.cin, base_ch=a.base)
    fresh = R.formula_weights(a.base, a.cin, a.K, dtype=torch.float64)
    model.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in fresh.items()})
    model = model.cuda().train()
    lg = model.forward_lowres(x.cuda())
    combined_loss(lg, m.cuda()).backward()
    torch.save({"logits": lg.detach().cpu(), **{k: p.grad.cpu() for k, p in model.named_parameters()}}, out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--base", type=int, default=64)
    ap.add_argument("--cin", type=int, default=1)
    ap.add_argument("--K", type=int, default=2)
    ap.add_argument("--H", type=int, default=64)
    ap.add_argument("--dump", default="")
    a = ap.parse_args()
    if a.dump:
        dump(a, a.dump)
        return
    import torch
    from oracle import eunet_ref as R
    from eunet import synth
    outs = []
    for i, lib in enumerate(a.libs):
        out = os.path.join(ROOT, "gpurun_out", f"ab_{i}.pt")
        env = dict(os.environ, EUNET_LIB=os.path.abspath(lib))
        subprocess.run([sys.executable, __file__, "--dump", out, "--base", str(a.base), "--cin", str(a.cin),
                        "--K", str(a.K), "--H", str(a.H)], env=env, check=True, timeout=600)
        outs.append(torch.load(out, weights_only=True))
    x, m = synth.batch(2, a.H, a.H, start_index=7, num_classes=a.K, in_channels=a.cin)
    S = R.formula_weights(a.base, a.cin, a.K, dtype=torch.float64)
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    R.batch_loss(R.forward(S, x.double(), training=True), m).backward()
    r = lambda p, q: float((p.double() - q.double()).norm() / q.double().norm().clamp_min(1e-30))
    print(f"{'param':32s} " + " ".join(f"lib{i}-vs-fp64" for i in range(len(outs))) + "  lib0-vs-lib1")
    for k in outs[0]:
        if k == "logits" or k.endswith((".0.bias", ".3.bias")) and not k.startswith("enhance.3"):
            continue
        errs = [r(o[k], S[k].grad) for o in outs]
        ab = r(outs[0][k], outs[1][k]) if len(outs) > 1 else 0.0
        print(f"{k:32s} " + " ".join(f"{e:12.2e}" for e in errs) + f"  {ab:12.2e}")
    if len(outs) > 1:
        print("logits lib0-vs-lib1", r(outs[0]["logits"], outs[1]["logits"]))


if __name__ == "__main__":
    main()
