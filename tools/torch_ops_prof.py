"""List the PyTorch (non-HIP-extension) ops of one cfg3 training step with their Python call
sites: what issues the fills / copies / small torch kernels around the HIP path.
    python tools/torch_ops_prof.py
"""
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from eunet import synth  # noqa: E402
from eunet.models import EnhancedUNet  # noqa: E402
from eunet.train_eval import Trainer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64, dtype="bf16").to(dev)
    tr = Trainer(model, dev, "enhanced_unet", total_epochs=50)
    tr.epoch_lr_step(0)
    x, m = synth.batch(4, 1024, 1024, num_classes=2, in_channels=1, device=dev)
    for _ in range(2):
        tr.step(x, m)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        tr.step(x, m)
        torch.cuda.synchronize()
    sites = Counter()
    for ev in prof.events():
        if ev.name in ("aten::fill_", "aten::zero_", "aten::copy_", "aten::clone", "aten::ones_like", "aten::zeros"):
            stack = [f for f in (ev.stack or []) if "eunet" in f or "train_eval" in f or "torch/autograd" in f
                     or "torch/nn/utils" in f or "torch/optim" in f]
            sites[(ev.name, stack[0] if stack else "?")] += 1
    for (name, site), k in sites.most_common(40):
        print(f"{k:4d}  {name:16s} {site}")
    allops = Counter(ev.name for ev in prof.events())
    print("all ops:", allops.most_common(45))


if __name__ == "__main__":
    main()
