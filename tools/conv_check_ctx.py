"""Check every conv3x3 launch of one fp32 train step against an fp64 recomputation
from the launch's own inputs (in-context precision / correctness of fwd + dgrad).

    python tools/conv_check_ctx.py [--base 64 --cin 1 --K 2 --H 64]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from eunet import ops  # noqa: E402


def view(a):
    """NHWC tensor of an Act (channel slice)."""
    t = a._keep
    return t.reshape(a.n, a.h, a.w, a.ctot)[..., a.coff:a.coff + a.c]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", type=int, default=64)
    ap.add_argument("--cin", type=int, default=1)
    ap.add_argument("--K", type=int, default=2)
    ap.add_argument("--H", type=int, default=64)
    a = ap.parse_args()
    packs = {}
    orig_pack, orig_fwd = ops.conv3x3_pack, ops.conv3x3_fwd

    def pack(w, dtype, flip):
        wp = orig_pack(w, dtype, flip)
        packs[wp.data_ptr()] = (w.detach().clone(), flip)
        return wp

    def fwd(x, wp, y, bias=None, scale=None, shift=None, stats=None):
        xin = view(x).double().cpu().clone()
        orig_fwd(x, wp, y, bias=bias, scale=scale, shift=shift, stats=stats)
        torch.cuda.synchronize()
        w, flip = packs[wp.data_ptr()]
        w = w.double().cpu()
        xi = xin.permute(0, 3, 1, 2)
        if scale is not None:
            xi = torch.relu(xi * scale.double().cpu()[None, :, None, None] + shift.double().cpu()[None, :, None, None])
        if flip:
            ref = F.conv_transpose2d(xi, w, padding=1)
        else:
            ref = F.conv2d(xi, w, None if bias is None else bias.double().cpu(), padding=1)
        ref = ref.permute(0, 2, 3, 1)
        out = view(y).double().cpu()
        err = (out - ref)
        print(f"{'dgrad' if flip else 'fwd  '} x{tuple(xin.shape)} -> y{tuple(out.shape)} coff{y.coff}/{y.ctot} "
              f"rl2 {float(err.norm() / ref.norm()):.2e} maxabs {float(err.abs().max()):.2e} "
              f"meanerr/rms {float(err.mean() / ref.pow(2).mean().sqrt()):.2e} "
              f"border-maxabs {float(torch.cat([err[:, 0].flatten(), err[:, -1].flatten(), err[:, :, 0].flatten(), err[:, :, -1].flatten()]).abs().max()):.2e}",
              flush=True)

    ops.conv3x3_pack, ops.conv3x3_fwd = pack, fwd
    from oracle import eunet_ref as R
    from eunet import synth
    from eunet.losses import combined_loss
    from eunet.models import EnhancedUNet
    x, m = synth.batch(2, a.H, a.H, start_index=7, num_classes=a.K, in_channels=a.cin)
    model = EnhancedUNet(num_classes=a.K, in_channels=a.cin, base_ch=a.base)
    model.load_state_dict({k: v.float() if v.is_floating_point() else v
                           for k, v in R.formula_weights(a.base, a.cin, a.K, dtype=torch.float64).items()})
    model = model.cuda().train()
    combined_loss(model.forward_lowres(x.cuda()), m.cuda()).backward()


if __name__ == "__main__":
    main()
