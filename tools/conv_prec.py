"""fp32 precision of the conv3x3 kernels (fwd, dgrad, wgrad) vs fp64, next to torch CPU fp32.

    python tools/conv_prec.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from eunet import ops  # noqa: E402


def rl2(a, b):
    return float((a.double().cpu() - b).norm() / b.norm())


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def main():
    g = torch.Generator().manual_seed(0)
    for (N, H, W, ci, co) in [(2, 16, 16, 256, 256), (2, 8, 8, 256, 512), (2, 32, 32, 128, 64), (2, 64, 64, 64, 64)]:
        x = torch.randn(N, H, W, ci, generator=g, dtype=torch.float64)
        w = torch.randn(co, ci, 3, 3, generator=g, dtype=torch.float64) / (3 * ci ** 0.5)
        gy = torch.randn(N, H, W, co, generator=g, dtype=torch.float64)
        ref = nhwc(F.conv2d(nchw(x), w, padding=1))
        cpu32 = nhwc(F.conv2d(nchw(x).float(), w.float(), padding=1))
        y = torch.empty(N, H, W, co, device="cuda")
        wp = ops.conv3x3_pack(w.float().cuda(), torch.float32, flip=False)
        ops.conv3x3_fwd(ops.act(x.float().cuda()), wp, ops.act(y))
        gref = nhwc(F.conv_transpose2d(nchw(gy), w, padding=1))
        gcpu = nhwc(F.conv_transpose2d(nchw(gy).float(), w.float(), padding=1))
        gx = torch.empty(N, H, W, ci, device="cuda")
        wpt = ops.conv3x3_pack(w.float().cuda(), torch.float32, flip=True)
        ops.conv3x3_fwd(ops.act(gy.float().cuda()), wpt, ops.act(gx))
        torch.cuda.synchronize()
        print(f"N{N} H{H} W{W} ci{ci} co{co}: fwd ours {rl2(y, ref):.2e} cpu32 {rl2(cpu32, ref):.2e} | "
              f"dgrad ours {rl2(gx, gref):.2e} cpu32 {rl2(gcpu, gref):.2e}", flush=True)


if __name__ == "__main__":
    main()
