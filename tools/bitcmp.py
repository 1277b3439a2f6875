"""Bit-identity check between library builds: two bf16 Trainer steps of the bench model (default: the bench
size), then a SHA-256 over every parameter, gradient and BN running statistic, one line per build.

    python tools/bitcmp.py LIB [LIB ...] [--size 1024 --batch 4]

Each build runs in its own child process (EUNET_LIB); equal digests = bit-identical steps."""
import argparse
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]


def digest(a):
    import torch
    from eunet import synth
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    torch.manual_seed(0)
    model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64, dtype="bf16").cuda()
    tr = Trainer(model, "cuda", "enhanced_unet", total_epochs=50)
    tr.epoch_lr_step(0)
    for i in range(2):
        x, m = synth.batch(a.batch, a.size, a.size, start_index=3 + i, num_classes=2, in_channels=1)
        tr.step(x.cuda(), m.cuda(), sync_loss=False)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for k, t in list(model.state_dict().items()) + [(k + ".grad", p.grad) for k, p in model.named_parameters()]:
        h.update(k.encode())
        h.update(t.detach().contiguous().cpu().numpy().tobytes())
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        print(digest(a), flush=True)
        return
    for lib in a.libs:
        r = subprocess.run([sys.executable, __file__, "--child", "--size", str(a.size), "--batch", str(a.batch)],
                           env=dict(os.environ, EUNET_LIB=lib), capture_output=True, text=True, timeout=300)
        if r.returncode:
            sys.stderr.write(r.stderr[-3000:])
            raise SystemExit(f"{lib}: rc {r.returncode}")
        print(f"bitcmp {lib} {r.stdout.strip().splitlines()[-1]}", flush=True)


if __name__ == "__main__":
    main()
