"""The dual-branch configs[4] step alone (base 96, 2048^2, batch 2, bf16) for a rocprofv3 kernel trace:

    rocprofv3 --kernel-trace --stats -- python tools/dual_prof.py [--steps 3]

Diagnostic only (synthetic batch, random weights)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    sys.argv = ["bench.py", "--steps", str(a.steps), "--warmup", "2"]
    args = bench.parse()
    from eunet import synth
    tr = bench.build_trainer(args, "cuda", dtype="bf16", base=96, dual=True)
    x, m = synth.batch(2, 2048, 2048, start_index=0, num_classes=2, in_channels=1, device="cuda")
    for _ in range(2 + a.steps):
        tr.step(x, m)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
