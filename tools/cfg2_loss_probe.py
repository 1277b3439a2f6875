"""configs[2] batch (base 64, 1024^2, B 4): Trainer losses over 4 steps per (dtype, lr) -- is a loss rise after the
first AdamW step optimisation dynamics (fp32 does it too) or a bf16 defect?  Diagnostic only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402

from eunet import synth  # noqa: E402
from eunet.models import EnhancedUNet  # noqa: E402
from eunet.train_eval import Trainer  # noqa: E402
from oracle import eunet_ref as R  # noqa: E402

x, m = synth.batch(4, 1024, 1024, start_index=71, num_classes=2, in_channels=1)
x, m = x.cuda(), m.cuda()
W = {k: (v.float() if v.is_floating_point() else v) for k, v in R.formula_weights(64, 1, 2).items()}
for dt in ("bf16", "fp32"):
    for lr in (1e-3, 3e-4, 1e-4):
        mod = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64, dtype=dt)
        mod.load_state_dict(W)
        tr = Trainer(mod.cuda().train(), "cuda", "enhanced_unet")
        for g in tr.optimizer.param_groups:
            g["lr"] = lr
        print(dt, lr, [round(tr.step(x, m), 4) for _ in range(6)], flush=True)
