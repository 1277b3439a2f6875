"""Standalone timing of HBM-bound kernels at the 1024^2 x 4, 64-channel bf16 shape (HIP events).
    python tools/time_memk.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]
import torch  # noqa: E402
from eunet import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


N, H, C = 4, 1024, 64
dev = "cuda"
g = torch.randn(N, H, H, C, device=dev).bfloat16()
y = torch.randn(N, H, H, C, device=dev).bfloat16()
gy = torch.empty_like(g)
v = [torch.rand(C, device=dev) + 0.5 for _ in range(6)]
ms = timeit(lambda: ops.bn_bwd_apply(ops.act(g), ops.act(y), *v, ops.act(gy)))
print(f"bn_bwd_apply        {ms * 1e3:7.1f} us  {3 * g.numel() * 2 / ms / 1e9:5.2f} TB/s")
z = torch.empty(N, H, H, 2, device=dev)
w, b = torch.randn(2, C, device=dev), torch.randn(2, device=dev)
ms = timeit(lambda: ops.bnrelu_conv1x1(ops.act(y), v[0], v[1], w, b, 2, z))
print(f"bnrelu_conv1x1      {ms * 1e3:7.1f} us  {(y.numel() * 2 + z.numel() * 4) / ms / 1e9:5.2f} TB/s")

# BN+ReLU -> x2 upsample into the decoder's concat slots (the bench's three launches: 128^2 x 512, 256^2 x 256,
# 512^2 x 128 channels at N 4 -> 2x into [up | skip] buffers)
tot = 0.0
for h, c in ((128, 512), (256, 256), (512, 128)):
    yu = torch.randn(N, h, h, c, device=dev).bfloat16()
    cat = torch.empty(N, 2 * h, 2 * h, 2 * c, device=dev).bfloat16()
    sc, sh = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.3
    ms = timeit(lambda: ops.bnrelu_upsample(ops.act(yu), sc, sh, ops.act(cat, 0, c)))
    tot += ms
    print(f"bnrelu_upsample {h:4d}^2 x {c:3d} {ms * 1e3:7.1f} us  {yu.numel() * 2 * 5 / ms / 1e9:5.2f} TB/s")
print(f"bnrelu_upsample total {tot * 1e3:7.1f} us")

# x2 upsample adjoint with the fused BN-backward partial sums (the bench's three launches: gradients of the
# decoder's [up | skip] concat inputs at 256^2 / 512^2 / 1024^2 -> 128^2 x 512, 256^2 x 256, 512^2 x 128)
tot = 0.0
for h, c in ((128, 512), (256, 256), (512, 128)):
    gcat = torch.randn(N, 2 * h, 2 * h, 2 * c, device=dev).bfloat16()
    glo = torch.empty(N, h, h, c, device=dev).bfloat16()
    yl = torch.randn(N, h, h, c, device=dev).bfloat16()
    vv = [torch.rand(c, device=dev) + 0.5 for _ in range(4)]
    rows = ops.upsample_bwd_bnr_rows(ops.act(glo))
    part = torch.empty(rows * 2 * c, device=dev)
    ms = timeit(lambda: ops.upsample_bwd_bnr(ops.act(gcat, 0, c), ops.act(glo), ops.act(yl), *vv, part))
    tot += ms
    print(f"upsample_bwd_bnr {h:4d}^2 x {c:3d} {ms * 1e3:7.1f} us  {glo.numel() * 2 * 6 / ms / 1e9:5.2f} TB/s")
print(f"upsample_bwd_bnr total {tot * 1e3:7.1f} us")

# enc1.0: the 1-input-channel direct conv (conv_small_fwd, 1024^2 x 4 -> 64 channels bf16, BN partials), HBM-write-bound
xs1 = torch.randn(N, H, H, 1, device=dev).bfloat16()
w1s, b1s = torch.randn(64, 1, 3, 3, device=dev) * 0.3, torch.randn(64, device=dev) * 0.1
ys1 = torch.empty(N, H, H, 64, device=dev).bfloat16()
tiles1 = N * (H // 16) * (H // 32)
st1 = torch.empty(tiles1 * 2 * 64 + tiles1, device=dev)
ms = timeit(lambda: ops.conv_small_fwd(ops.act(xs1), w1s, b1s, ops.act(ys1), st1))
print(f"conv_small_fwd enc1.0 {ms * 1e3:7.1f} us  {(ys1.numel() * 2 + xs1.numel() * 2) / ms / 1e9:5.2f} TB/s")

# BN+ReLU -> skip activation + 2x2 max-pool (the bench's three launches: 1024^2 x 64, 512^2 x 128, 256^2 x 256)
tot = 0.0
for h, c in ((1024, 64), (512, 128), (256, 256)):
    yp_ = torch.randn(N, h, h, c, device=dev).bfloat16()
    catp = torch.empty(N, h, h, 2 * c, device=dev).bfloat16()
    pooled = torch.empty(N, h // 2, h // 2, c, device=dev).bfloat16()
    sc, sh = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.3
    ms = timeit(lambda: ops.bnrelu_pool(ops.act(yp_), sc, sh, ops.act(catp, c, c), ops.act(pooled)))
    tot += ms
    print(f"bnrelu_pool {h:5d}^2 x {c:3d} {ms * 1e3:7.1f} us  {yp_.numel() * 2 * 2.25 / ms / 1e9:5.2f} TB/s")
print(f"bnrelu_pool total {tot * 1e3:7.1f} us")
