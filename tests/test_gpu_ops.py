"""Per-kernel numerics through the C-ABI vs plain PyTorch fp64 references (GPU only).

fp32 kernels (exact-fp32 MFMA / VALU) are held to 1e-4 relative.  The bf16 conv3x3 / conv_small
kernels (bf16 operands, fp32 accumulation, one rounding of a bf16 output) are held to an
operand-exact bound (gate()): the fp64 reference is evaluated on the kernel's own bf16 operands --
the inputs and weights as rounded, and the BN+ReLU operand transform as the kernels form it
(relu(fmaf(x, scale, shift)) of the fp32 constants, then rounded to bf16: tf()) -- so what remains is
the fp32 accumulation and the output rounding, and every element must satisfy
    |got - ref| <= 2^-8 |ref| + 1e-5 max|ref|
(2^-8 = twice the round-to-nearest bound of a bf16 output).  A dropped K-chunk, a mis-indexed co-block
or a shifted tap moves elements by O(|ref|) and fails it.  The other bf16 kernels (BN+ReLU / pool /
upsample / 1x1 producers, whose references are not operand-exact) keep 2e-2 of the output scale.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from eunet import ops
    return ops


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2}


def gate(got, ref, dt):
    """Worst element's error over its bound (passes at <= 1).  fp32: max|got - ref| <= 1e-4 max|ref|;
    bf16 (operand-exact reference, module docstring): |got - ref| <= 2^-8 |ref| + 1e-5 max|ref| per element."""
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    mx = float(ref.abs().max().clamp_min(1e-30))
    if dt == torch.float32:
        return float((got - ref).abs().max()) / (1e-4 * mx)
    return float(((got - ref).abs() / (2.0 ** -8 * ref.abs() + 1e-5 * mx)).max())


def tf(x, sc, sh, dt):
    """The conv kernels' BN+ReLU operand transform: relu(fmaf(x, sc, sh)) with the fp32 constants (the
    fp64 product and sum of these operands are exact, then rounded once to fp32 as the fused multiply-add
    rounds), rounded to the staged operand's dtype."""
    v = (x * sc.float().double() + sh.float().double()).float().double().clamp_min(0.0)
    return v.to(torch.bfloat16).double() if dt == torch.bfloat16 else v


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("transform", [False, True])
def test_conv3x3_fwd_stats(dt, transform):
    ops = _ops()
    g = torch.Generator().manual_seed(1)
    N, H, W, Cin, Cout, CT, CO = 2, 20, 36, 32, 80, 48, 8
    buf = torch.randn(N, H, W, CT, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / 17.0
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    sc = torch.rand(Cin, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(Cin, generator=g, dtype=torch.float64) * 0.3
    xd = buf.to(DEV, dt)
    xq = xd.double().cpu()[..., CO:CO + Cin]  # rounded input the kernel sees
    xt = nchw(xq)
    if transform:
        xt = tf(xt, sc[None, :, None, None], sh[None, :, None, None], dt)
    wq = w.to(dt).double()
    ref = nhwc(F.conv2d(xt, wq, b.float().double(), padding=1))
    y = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    wp = ops.conv3x3_pack(w.float().to(DEV), dt, flip=False)
    tiles = ops.conv3x3_tiles(ops.act(y))
    st = torch.empty(tiles * (2 * Cout + 1), dtype=torch.float32, device=DEV)
    ops.conv3x3_fwd(ops.act(xd, CO, Cin), wp, ops.act(y), bias=b.float().to(DEV),
                    scale=sc.float().to(DEV) if transform else None,
                    shift=sh.float().to(DEV) if transform else None, stats=st)
    torch.cuda.synchronize()
    assert gate(y, ref, dt) <= 1.0, gate(y, ref, dt)
    # BN statistics via finalize
    gamma = torch.ones(Cout, device=DEV)
    beta = torch.zeros(Cout, device=DEV)
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    mean, inv = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    s1, s2 = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    ops.bn_finalize(st, tiles, Cout, gamma, beta, 1e-5, 0.1, rm, rv, mean, inv, s1, s2)
    torch.cuda.synchronize()
    yr = y.double().cpu() if dt == torch.float32 else ref
    m_ref = yr.mean(dim=(0, 1, 2))
    v_ref = yr.var(dim=(0, 1, 2), unbiased=False)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert rel(mean, m_ref) < tol
    assert rel(1.0 / inv ** 2 - 1e-5, v_ref) < tol * 10
    n = N * H * W
    assert rel(rv, 0.9 + 0.1 * v_ref * n / (n - 1)) < tol * 10


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_fwd_stats_ragged_offset_channels(dt):
    """BN partials of edge tiles when a channel's mean is far larger than its spread (bias 300, unit
    spread; 20 x 36 images: every tile row / column edge is ragged): the per-wave M2 of an edge tile
    takes only the valid pixels (no (0 - mean)^2 terms to cancel afterwards), so the batch variance stays
    at fp32 accuracy relative to the VARIANCE, not to mean^2 (the subtraction form lost ~1e-2
    of the variance here)."""
    ops = _ops()
    g = torch.Generator().manual_seed(2)
    N, H, W, Cin, Cout = 2, 20, 36, 32, 64
    x = torch.randn(N, H, W, Cin, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / 17.0
    b = 300.0 + torch.randn(Cout, generator=g, dtype=torch.float64)
    xd = x.to(DEV, dt)
    y = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    wp = ops.conv3x3_pack(w.float().to(DEV), dt, flip=False)
    tiles = ops.conv3x3_tiles(ops.act(y))
    st = torch.empty(tiles * (2 * Cout + 1), dtype=torch.float32, device=DEV)
    ops.conv3x3_fwd(ops.act(xd), wp, ops.act(y), bias=b.float().to(DEV), stats=st)
    gamma, beta = torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    mean, inv = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    s1, s2 = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    ops.bn_finalize(st, tiles, Cout, gamma, beta, 1e-5, 0.1, rm, rv, mean, inv, s1, s2)
    torch.cuda.synchronize()
    # the fp32 accumulators the partials are taken from: the exact conv of the kernel's operands + bias (fp32)
    ref = nhwc(F.conv2d(nchw(xd.double().cpu()), w.to(dt).double(), b.float().double(), padding=1))
    v_ref = ref.var(dim=(0, 1, 2), unbiased=False)
    v_got = 1.0 / inv.double().cpu() ** 2 - 1e-5
    err = float(((v_got - v_ref).abs() / v_ref).max())
    print(f"{dt} ragged offset-channel variance rel err {err:.2e} (mean ~300, var ~{float(v_ref.mean()):.2f})")
    assert err < 2e-4


def test_conv3x3_fwd_large_sample_slice():
    """One sample's input above 2 GiB (2048^2 x 288 bf16 = 2.4 GB: the dual-branch base-96 dec2.0
    input of BASELINE configs[4]) through the buffer-descriptor staging (unsigned 32-bit offsets, slices
    < 3 GiB): outputs at points whose halo lies beyond the 2 GiB mark vs fp64 dot products."""
    ops = _ops()
    N, H, W, Cin, Cout = 1, 2048, 2048, 288, 96
    g = torch.Generator(device=DEV).manual_seed(21)
    x = torch.randn(N, H, W, Cin, generator=g, device=DEV, dtype=torch.float32).to(torch.bfloat16)
    gc = torch.Generator().manual_seed(22)
    w = (torch.randn(Cout, Cin, 3, 3, generator=gc, dtype=torch.float64) / 50).to(torch.bfloat16).double()
    b = torch.randn(Cout, generator=gc, dtype=torch.float64)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=DEV)
    wp = ops.conv3x3_pack(w.float().to(DEV), torch.bfloat16, flip=False)
    ops.conv3x3_fwd(ops.act(x), wp, ops.act(y), bias=b.float().to(DEV))
    torch.cuda.synchronize()
    pts = [(2047, 2047), (2047, 0), (1900, 1500), (1800, 2047), (0, 0), (1024, 17), (2046, 1023)]
    for yy, xx in pts:
        patch = torch.zeros(3, 3, Cin, dtype=torch.float64)
        for dy in range(3):
            for dx in range(3):
                sy, sx = yy + dy - 1, xx + dx - 1
                if 0 <= sy < H and 0 <= sx < W:
                    patch[dy, dx] = x[0, sy, sx].double().cpu()
        ref = torch.einsum("oiyx,yxi->o", w, patch) + b
        got = y[0, yy, xx].double().cpu()
        assert gate(got, ref, torch.bfloat16) <= 1.0, (yy, xx, gate(got, ref, torch.bfloat16))
    assert (1900 * W + 1500) * Cin * 2 > 2 ** 31  # the checked halos sit beyond 2 GiB
    del x, y


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_dgrad_wgrad(dt):
    ops = _ops()
    g = torch.Generator().manual_seed(2)
    N, H, W, Cin, Cout = 2, 16, 40, 48, 64
    x = torch.randn(N, H, W, Cin, generator=g, dtype=torch.float64).to(dt).double()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / 20).to(dt).double()
    gy = torch.randn(N, H, W, Cout, generator=g, dtype=torch.float64).to(dt).double()
    sc = torch.rand(Cin, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(Cin, generator=g, dtype=torch.float64) * 0.3
    xt = nchw(x).requires_grad_(True)
    xa = torch.relu(xt * sc[None, :, None, None] + sh[None, :, None, None])
    xa_q = tf(xt.detach(), sc[None, :, None, None], sh[None, :, None, None], dt) if dt == torch.bfloat16 else xa
    wt = w.clone().requires_grad_(True)
    y = F.conv2d(xa_q.detach() if dt == torch.bfloat16 else xa, wt, None, padding=1)
    y.backward(nchw(gy))
    # dgrad (w.r.t. the conv input, i.e. before the transform): kernel computes W^T gy
    gx_ref = nhwc(F.conv_transpose2d(nchw(gy), w, padding=1))
    gxd = torch.empty(N, H, W, Cin, dtype=dt, device=DEV)
    wpt = ops.conv3x3_pack(w.float().to(DEV), dt, flip=True)
    ops.conv3x3_fwd(ops.act(gy.to(DEV, dt)), wpt, ops.act(gxd))
    gxd2 = torch.empty_like(gxd)  # the dgrad entry point runs the same kernel (own symbol)
    ops.conv3x3_dgrad(ops.act(gy.to(DEV, dt)), wpt, ops.act(gxd2))
    # wgrad with fused transform
    dyd = gy.to(DEV, dt)
    ns = ops.conv3x3_wgrad_splits(ops.act(dyd), Cin, dt)
    dwp = torch.empty(ns * Cout * 9 * Cin, device=DEV)
    dbp = torch.empty(ns * Cout, device=DEV)
    ops.conv3x3_wgrad(ops.act(x.to(DEV, dt)), ops.act(dyd), dwp, dbp, ns, scale=sc.float().to(DEV),
                      shift=sh.float().to(DEV))
    dw = torch.empty(Cout, Cin, 3, 3, device=DEV)
    db = torch.empty(Cout, device=DEV)
    ops.wgrad_reduce(dwp, dbp, ns, Cout, Cin, 9, dw, db)
    torch.cuda.synchronize()
    assert torch.equal(gxd, gxd2)
    assert gate(gxd, gx_ref, dt) <= 1.0, gate(gxd, gx_ref, dt)
    assert gate(dw, wt.grad, dt) <= 1.0, gate(dw, wt.grad, dt)
    assert gate(db, gy.sum(dim=(0, 1, 2)), dt) <= 1.0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_wgrad_ragged_slots(dt):
    """The weight gradient over channel slots of concat buffers (x at channel 16, dY at 8), a partial
    input-channel chunk (40 of 64) and output-channel block (80 = 64 + 16), ragged tile rows and columns
    (13 x 40), a per-sample BN transform (nstride) and pixel splits whose tile ranges cross samples --
    against the fp64 weight gradient of the transformed operand (rounded to bf16 as the kernel stages it)."""
    ops = _ops()
    g = torch.Generator().manual_seed(43)
    N, H, W, Cin, Cout = 3, 13, 40, 40, 80
    xb = torch.randn(N, H, W, Cin + 24, generator=g).to(DEV, dt)
    dyb = torch.randn(N, H, W, Cout + 16, generator=g).to(DEV, dt)
    ns_stride = Cin + 8
    sc = (torch.rand(N, ns_stride, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(N, ns_stride, generator=g) * 0.3).to(DEV)
    x = xb[..., 16:16 + Cin].double().cpu()
    dy = dyb[..., 8:8 + Cout].double().cpu()
    xa = (x * sc[:, None, None, :Cin].double().cpu() + sh[:, None, None, :Cin].double().cpu()).clamp_min(0.0)
    if dt == torch.bfloat16:
        xa = xa.float().bfloat16().double()
    wt = torch.zeros(Cout, Cin, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv2d(nchw(xa), wt, None, padding=1).backward(nchw(dy))
    th, tw = (8, 16) if dt == torch.bfloat16 else (4, 32)  # the kernels' pixel tiles
    ntiles = N * -(-H // th) * -(-W // tw)
    tpi = ntiles // N
    crossing = [s for s in range(2, ntiles) if -(-ntiles // -(-ntiles // s)) == s and (-(-ntiles // s)) % tpi]
    assert crossing
    xv, dv = ops.act(xb, 16, Cin), ops.act(dyb, 8, Cout)
    for ns in (ops.conv3x3_wgrad_splits(dv, Cin, dt), crossing[0]):
        dwp = torch.empty(ns * Cout * 9 * Cin, device=DEV)
        dbp = torch.empty(ns * Cout, device=DEV)
        ops.conv3x3_wgrad(xv, dv, dwp, dbp, ns, scale=sc, shift=sh, nstride=ns_stride)
        dw = torch.empty(Cout, Cin, 3, 3, device=DEV)
        db = torch.empty(Cout, device=DEV)
        ops.wgrad_reduce(dwp, dbp, ns, Cout, Cin, 9, dw, db)
        torch.cuda.synchronize()
        assert rel(dw, wt.grad) < 1e-5, ns
        assert rel(db, dy.sum(dim=(0, 1, 2))) < 1e-5, ns


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin", [1, 3, 4, 6, 8])
def test_conv_small(dt, cin):
    ops = _ops()
    g = torch.Generator().manual_seed(3)
    N, H, W, Cout = 2, 24, 40, 64
    x = torch.rand(N, H, W, cin, generator=g, dtype=torch.float64).to(dt).double()
    w = torch.randn(Cout, cin, 3, 3, generator=g, dtype=torch.float64) / 3
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    ref = nhwc(F.conv2d(nchw(x), w.float().double(), b.float().double(), padding=1))
    y = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    tiles = ops.conv3x3_tiles(ops.act(y))
    st = torch.empty(tiles * (2 * Cout + 1), device=DEV)
    ops.conv_small_fwd(ops.act(x.to(DEV, dt)), w.float().to(DEV), b.float().to(DEV), ops.act(y), st)
    gy = torch.randn(N, H, W, Cout, generator=g, dtype=torch.float64).to(dt).double()
    ns = ops.conv_small_wgrad_splits(ops.act(gy.to(DEV, dt)))
    dwp = torch.empty(ns * Cout * 9 * cin, device=DEV)
    dbp = torch.empty(ns * Cout, device=DEV)
    ops.conv_small_wgrad(ops.act(x.to(DEV, dt)), ops.act(gy.to(DEV, dt)), dwp, dbp, ns)
    dw = torch.empty(Cout, cin, 3, 3, device=DEV)
    db = torch.empty(Cout, device=DEV)
    ops.wgrad_reduce(dwp, dbp, ns, Cout, cin, 9, dw, db)
    wt = w.clone().requires_grad_(True)
    F.conv2d(nchw(x), wt, None, padding=1).backward(nchw(gy))
    torch.cuda.synchronize()
    assert gate(y, ref, dt) <= 1.0, gate(y, ref, dt)
    assert rel(dw, wt.grad) < 1e-4
    assert rel(db, gy.sum(dim=(0, 1, 2))) < 1e-4
    gamma, beta = torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    mean, inv = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    ops.bn_finalize(st, tiles, Cout, gamma, beta, 1e-5, 0.1, None, None, mean, inv, None, None)
    torch.cuda.synchronize()
    # statistics come from the fp32 accumulators (before any bf16 rounding)
    yr = y.double().cpu() if dt == torch.float32 else ref
    assert rel(mean, yr.mean(dim=(0, 1, 2))) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bnrelu_pool_up_conv1x1(dt):
    ops = _ops()
    g = torch.Generator().manual_seed(4)
    N, H, W, C = 2, 12, 20, 32
    y = torch.randn(N, H, W, C, generator=g, dtype=torch.float64).to(dt).double()
    sc = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(C, generator=g, dtype=torch.float64) * 0.3
    a = torch.relu(y * sc + sh)
    yd = y.to(DEV, dt)
    scd, shd = sc.float().to(DEV), sh.float().to(DEV)
    # pool (+ act into a concat slot)
    cat = torch.zeros(N, H, W, C + 16, dtype=dt, device=DEV)
    pooled = torch.empty(N, H // 2, W // 2, C, dtype=dt, device=DEV)
    ops.bnrelu_pool(ops.act(yd), scd, shd, ops.act(cat, 16, C), ops.act(pooled))
    # upsample into a slot
    up = torch.zeros(N, 2 * H, 2 * W, C + 8, dtype=dt, device=DEV)
    ops.bnrelu_upsample(ops.act(yd), scd, shd, ops.act(up, 0, C))
    # dec1 1x1
    K = 3
    w = torch.randn(K, C, generator=g, dtype=torch.float64) / 5
    b = torch.randn(K, generator=g, dtype=torch.float64)
    z = torch.empty(N, H, W, K, device=DEV)
    ops.bnrelu_conv1x1(ops.act(yd), scd, shd, w.float().to(DEV), b.float().to(DEV), K, z)
    torch.cuda.synchronize()
    tol = TOL[dt]
    assert rel(cat[..., 16:], a) < tol
    assert float(cat[..., :16].abs().max()) == 0.0
    assert rel(pooled, nhwc(F.max_pool2d(nchw(a), 2))) < tol
    up_ref = nhwc(F.interpolate(nchw(a), scale_factor=2, mode="bilinear", align_corners=False))
    assert rel(up[..., :C], up_ref) < tol
    assert float(up[..., C:].abs().max()) == 0.0
    assert rel(z, a @ w.t() + b) < tol


@pytest.mark.parametrize("shape", [(1, 13, 21, 16), (2, 7, 9, 32), (4, 512, 512, 128)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bnrelu_upsample_row_sweep_shapes(shape, dt):
    """The row-sweep BN+ReLU -> x2 bilinear upsample (bnrelu_up_rows_kernel: 4 or 8 low-res rows per thread) on
    ragged row blocks, odd widths and the bench's largest launch (8 rows per thread), written into a concat slot,
    against F.interpolate of the BN+ReLU output on the GPU (models.py:229-236)."""
    ops = _ops()
    N, H, W, C = shape
    g = torch.Generator(device=DEV).manual_seed(7)
    y = torch.randn(N, H, W, C, generator=g, device=DEV).to(dt)
    sc = torch.rand(C, generator=g, device=DEV) + 0.5
    sh = torch.randn(C, generator=g, device=DEV) * 0.3
    up = torch.full((N, 2 * H, 2 * W, C + 8), 7.0, dtype=dt, device=DEV)
    ops.bnrelu_upsample(ops.act(y), sc, sh, ops.act(up, 0, C))
    a = torch.relu(y.float() * sc + sh)
    ref = nhwc(F.interpolate(nchw(a), scale_factor=2, mode="bilinear", align_corners=False))
    err = float((up[..., :C].float() - ref).abs().max() / ref.abs().max())
    assert err < TOL[dt], err
    assert bool((up[..., C:] == 7.0).all())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_backward_helpers(dt):
    ops = _ops()
    g = torch.Generator().manual_seed(5)
    N, H, W, C = 2, 8, 16, 32
    # --- BN + ReLU backward
    y = torch.randn(N, H, W, C, generator=g, dtype=torch.float64).to(dt).double()
    gamma = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(C, generator=g, dtype=torch.float64) * 0.2
    go = torch.randn(N, H, W, C, generator=g, dtype=torch.float64).to(dt).double()
    yt = nchw(y).requires_grad_(True)
    gt, bt = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    out = torch.relu(F.batch_norm(yt, None, None, gt, bt, True, 0.1, 1e-5))
    out.backward(nchw(go))
    mean = y.mean(dim=(0, 1, 2))
    inv = 1.0 / torch.sqrt(y.var(dim=(0, 1, 2), unbiased=False) + 1e-5)
    gd, yd = go.to(DEV, dt), y.to(DEV, dt)
    f = lambda t: t.float().to(DEV)
    tiles = ops.bn_bwd_tiles(ops.act(yd))
    part = torch.empty(tiles * 2 * C, device=DEV)
    sc, sh = f(gamma * inv), f(beta - mean * gamma * inv)  # the forward affine (defines the ReLU mask)
    ops.bn_bwd_reduce(ops.act(gd), ops.act(yd), f(mean), f(inv), sc, sh, part)
    red = torch.empty(2 * C, device=DEV)
    ops.colsum(part, tiles, 2 * C, red)
    gy = torch.empty_like(yd)
    ops.bn_bwd_apply(ops.act(gd), ops.act(yd), f(mean), f(inv), sc, sh, red[:C], red[C:], ops.act(gy))
    torch.cuda.synchronize()
    assert rel(red[:C], bt.grad) < 1e-4
    assert rel(red[C:], gt.grad) < 1e-4
    assert rel(gy, nhwc(yt.grad)) < TOL[dt]
    # --- max-pool backward + skip add (with ties)
    act = torch.relu(torch.randn(N, H, W, C, generator=g, dtype=torch.float64)).to(dt).double()
    act[0, 0, 0, :] = act[0, 0, 1, :]  # tie inside a window
    gp = torch.randn(N, H // 2, W // 2, C, generator=g, dtype=torch.float64).to(dt).double()
    gs = torch.randn(N, H, W, C, generator=g, dtype=torch.float64).to(dt).double()
    at = nchw(act).requires_grad_(True)
    F.max_pool2d(at, 2).backward(nchw(gp))
    out_ref = nhwc(at.grad) + gs
    cat = torch.zeros(N, H, W, C + 8, dtype=dt, device=DEV)
    cat[..., 8:] = act.to(DEV, dt)
    gcat = torch.zeros(N, H, W, C + 8, dtype=dt, device=DEV)
    gcat[..., 8:] = gs.to(DEV, dt)
    gout = torch.empty(N, H, W, C, dtype=dt, device=DEV)
    ops.pool_bwd_add(ops.act(cat, 8, C), ops.act(gp.to(DEV, dt)), ops.act(gcat, 8, C), ops.act(gout))
    # --- upsample backward from a channel slice
    gh = torch.randn(N, 2 * H, 2 * W, C + 16, generator=g, dtype=torch.float64).to(dt).double()
    lo = torch.zeros(N, H, W, C, dtype=torch.float64).requires_grad_(True)
    F.interpolate(nchw(lo), scale_factor=2, mode="bilinear", align_corners=False).backward(nchw(gh[..., :C]))
    glo = torch.empty(N, H, W, C, dtype=dt, device=DEV)
    ops.upsample_bwd(ops.act(gh.to(DEV, dt), 0, C), ops.act(glo))
    torch.cuda.synchronize()
    assert rel(gout, out_ref) < TOL[dt]
    assert rel(glo, lo.grad) < TOL[dt]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv1x1_bwd(dt):
    ops = _ops()
    g = torch.Generator().manual_seed(6)
    N, H, W, C, K = 2, 8, 24, 64, 2
    y = torch.randn(N, H, W, C, generator=g, dtype=torch.float64).to(dt).double()
    sc = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(C, generator=g, dtype=torch.float64) * 0.3
    w = torch.randn(K, C, generator=g, dtype=torch.float64) / 4
    gz = torch.randn(N, H, W, K, generator=g, dtype=torch.float64)
    a = torch.relu(y * sc + sh)
    yd = y.to(DEV, dt)
    gact = torch.empty_like(yd)
    tiles = ops.conv1x1_bwd_tiles(ops.act(yd))
    part = torch.empty(tiles * (K * C + K), device=DEV)
    ops.conv1x1_bwd(ops.act(yd), sc.float().to(DEV), sh.float().to(DEV), w.float().to(DEV), K, gz.float().to(DEV),
                    ops.act(gact), part)
    red = torch.empty(K * C + K, device=DEV)
    ops.colsum(part, tiles, K * C + K, red)
    torch.cuda.synchronize()
    assert rel(gact, gz @ w) < TOL[dt]
    gw_ref = torch.einsum("nhwk,nhwc->kc", gz, a)
    assert rel(red[:K * C].view(K, C), gw_ref) < TOL[dt]
    assert rel(red[K * C:], gz.sum(dim=(0, 1, 2))) < 1e-4


@pytest.mark.parametrize("dt,C,K", [(torch.bfloat16, 64, 2), (torch.bfloat16, 128, 2), (torch.bfloat16, 128, 3),
                                    (torch.float32, 64, 3)])
def test_conv1x1_bwd_fused_bn_reduce(dt, C, K):
    """conv1x1_bwd with y's BN-backward reduction fused in: gact and the (gW, gb) partials equal the
    plain kernel's bit for bit; the BN partial sums match bn_bwd_reduce on the stored gact."""
    ops = _ops()
    g = torch.Generator().manual_seed(23)
    N, H, W = 2, 12, 40
    yd = torch.randn(N, H, W, C, generator=g).to(DEV, dt)
    mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
    istd = (torch.rand(C, generator=g) + 0.5).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV)
    sc = gamma * istd
    sh = beta - mean * sc
    w = (torch.randn(K, C, generator=g) / 4).to(DEV)
    gz = torch.randn(N, H, W, K, generator=g).to(DEV)
    tiles = ops.conv1x1_bwd_tiles(ops.act(yd))
    ga1, ga2 = torch.empty_like(yd), torch.empty_like(yd)
    p1 = torch.empty(tiles * (K * C + K), device=DEV)
    p2 = torch.empty_like(p1)
    bp = torch.empty(tiles * 2 * C, device=DEV)
    ops.conv1x1_bwd(ops.act(yd), sc, sh, w, K, gz, ops.act(ga1), p1)
    ops.conv1x1_bwd_bnr(ops.act(yd), sc, sh, w, K, gz, ops.act(ga2), p2, mean, istd, bp)
    red = torch.empty(2 * C, device=DEV)
    ops.colsum(bp, tiles, 2 * C, red)
    bt = ops.bn_bwd_tiles(ops.act(yd))
    bp2 = torch.empty(bt * 2 * C, device=DEV)
    ops.bn_bwd_reduce(ops.act(ga1), ops.act(yd), mean, istd, sc, sh, bp2)
    red2 = torch.empty(2 * C, device=DEV)
    ops.colsum(bp2, bt, 2 * C, red2)
    torch.cuda.synchronize()
    assert torch.equal(ga1, ga2)
    assert torch.equal(p1, p2)
    assert rel(red, red2) < 1e-5


def _head_ref(z, w1, b1, gamma, beta, w2, b2):
    u = F.interpolate(z, scale_factor=2, mode="bilinear", align_corners=False)
    h = F.conv2d(u, w1, b1, padding=1)
    a = torch.relu(F.batch_norm(h, None, None, gamma, beta, True, 0.1, 1e-5))
    return u + F.conv2d(a, w2, b2)


@pytest.mark.parametrize("K,dt,N,H,W", [(2, torch.float32, 2, 12, 20), (3, torch.float32, 2, 12, 20),
                                        (1, torch.bfloat16, 2, 12, 20), (2, torch.bfloat16, 2, 12, 20),
                                        (3, torch.bfloat16, 2, 12, 20),
                                        # 2H tiles away from the image border (the bf16 kernels' interior
                                        # staging path) next to border tiles
                                        (2, torch.bfloat16, 1, 40, 28), (3, torch.bfloat16, 1, 24, 40)])
def test_head_fwd_bwd(K, dt, N, H, W):
    """fp32: FMA path, 1e-4 of the fp64 reference.  bf16: MFMA path (bf16 operands,
    fp32 accumulation = the reference's autocast precision): each quantity within
    max(1e-2, 1.5x) the error that CPU bf16 autocast of the same head makes vs fp64
    (g_z and g_W1 pass through sums of bf16 g_h that cancel: autocast itself is
    off by 2-9% there)."""
    ops = _ops()
    g = torch.Generator().manual_seed(7)
    z = torch.randn(N, K, H, W, generator=g, dtype=torch.float64)
    w1 = torch.randn(64, K, 3, 3, generator=g, dtype=torch.float64) / 4
    b1 = torch.randn(64, generator=g, dtype=torch.float64) * 0.1
    gamma = torch.rand(64, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(64, generator=g, dtype=torch.float64) * 0.1
    w2 = torch.randn(K, 64, 1, 1, generator=g, dtype=torch.float64) / 8
    b2 = torch.randn(K, generator=g, dtype=torch.float64) * 0.1
    leaves = [t.clone().requires_grad_(True) for t in (z, w1, b1, gamma, beta, w2, b2)]
    out = _head_ref(*leaves)
    logit_ref = F.avg_pool2d(out, 2)
    glog = torch.randn(N, K, H, W, generator=g, dtype=torch.float64)
    logit_ref.backward(glog)
    f = lambda t: t.float().contiguous().to(DEV)
    zd = f(nhwc(z))
    ws = torch.empty(ops.head_workspace_bytes(N, H, W, K, dt), dtype=torch.uint8, device=DEV)
    rm, rv = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    mean, inv = torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    out2h = torch.empty(N, K, 2 * H, 2 * W, device=DEV)
    logits = torch.empty(N, K, H, W, device=DEV)
    ops.head_fwd(zd, N, H, W, K, f(w1), f(b1), f(gamma), f(beta), f(w2.reshape(K, 64)), f(b2), True, 1e-5, 0.1,
                 rm, rv, mean, inv, out2h, logits, ws, dtype=dt)
    gz = torch.empty(N, H, W, K, device=DEV)
    gw1, gb1 = torch.empty(64, K, 3, 3, device=DEV), torch.empty(64, device=DEV)
    gg, gbt = torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    gw2, gb2 = torch.empty(K, 64, device=DEV), torch.empty(K, device=DEV)
    ops.head_bwd(zd, N, H, W, K, f(w1), f(b1), f(gamma), f(beta), f(w2.reshape(K, 64)), mean, inv, f(glog), None,
                 gz, gw1, gb1, gg, gbt, gw2, gb2, ws, dtype=dt)
    torch.cuda.synchronize()
    names = ["out2h", "logits", "gz", "gw1", "gg", "gbt", "gw2", "gb2"]
    ours = [out2h, logits, gz, gw1, gg, gbt, gw2, gb2]
    refs = [out, logit_ref, nhwc(leaves[0].grad), leaves[1].grad, leaves[3].grad, leaves[4].grad,
            leaves[5].grad.reshape(K, 64), leaves[6].grad]
    if dt == torch.float32:
        tols = [1e-4] * len(names)
    else:
        ac = [t.float().clone().requires_grad_(True) for t in (z, w1, b1, gamma, beta, w2, b2)]
        with torch.autocast("cpu", dtype=torch.bfloat16):
            ao = _head_ref(*ac)
            al = F.avg_pool2d(ao, 2)
        al.float().backward(glog.float())
        acv = [ao.detach(), al.detach(), nhwc(ac[0].grad), ac[1].grad, ac[3].grad, ac[4].grad,
               ac[5].grad.reshape(K, 64), ac[6].grad]
        tols = [max(1e-2, 1.5 * rel(a, r)) for a, r in zip(acv, refs)]
    for nm, o, r, t in zip(names, ours, refs, tols):
        assert rel(o, r) < t, (nm, rel(o, r), t)


def test_head_bf16_persistent_tile_loop():
    """bf16 head at a size where the persistent blocks loop over several 32 x 32 / 16 x 16 2H tiles (with
    the next tile's z / g_o prefetched across iterations) and tiles are ragged at the border: forward,
    logits and every gradient against an fp32 torch autograd reference of the same head on the GPU
    (bf16 operand rounding ~1e-2; an indexing fault shows as O(1))."""
    ops = _ops()
    K, N, H, W = 2, 2, 408, 392
    g = torch.Generator(device=DEV).manual_seed(11)
    r = lambda *sh, sc=1.0: torch.randn(*sh, device=DEV, generator=g) * sc  # noqa: E731
    z, w1, b1 = r(N, K, H, W), r(64, K, 3, 3, sc=0.25), r(64, sc=0.1)
    gamma, beta = torch.rand(64, device=DEV, generator=g) + 0.5, r(64, sc=0.1)
    w2, b2, glog = r(K, 64, 1, 1, sc=0.125), r(K, sc=0.1), r(N, K, H, W)
    leaves = [t.clone().requires_grad_(True) for t in (z, w1, b1, gamma, beta, w2, b2)]
    out = _head_ref(*leaves)
    logit_ref = F.avg_pool2d(out, 2)
    logit_ref.backward(glog)
    zd = nhwc(z).contiguous()
    ws = torch.empty(ops.head_workspace_bytes(N, H, W, K, torch.bfloat16), dtype=torch.uint8, device=DEV)
    rm, rv = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    mean, inv = torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    out2h = torch.empty(N, K, 2 * H, 2 * W, device=DEV)
    logits = torch.empty(N, K, H, W, device=DEV)
    w2f = w2.reshape(K, 64).contiguous()
    ops.head_fwd(zd, N, H, W, K, w1, b1, gamma, beta, w2f, b2, True, 1e-5, 0.1, rm, rv, mean, inv, out2h, logits,
                 ws, dtype=torch.bfloat16)
    gz = torch.empty(N, H, W, K, device=DEV)
    gw1, gb1 = torch.empty(64, K, 3, 3, device=DEV), torch.empty(64, device=DEV)
    gg, gbt = torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    gw2, gb2 = torch.empty(K, 64, device=DEV), torch.empty(K, device=DEV)
    ops.head_bwd(zd, N, H, W, K, w1, b1, gamma, beta, w2f, mean, inv, glog.contiguous(), None, gz, gw1, gb1, gg,
                 gbt, gw2, gb2, ws, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    checks = [("out2h", out2h, out, 2e-2), ("logits", logits, logit_ref, 2e-2),
              ("gz", gz, nhwc(leaves[0].grad), 0.1), ("gw1", gw1, leaves[1].grad, 0.1),
              ("gg", gg, leaves[3].grad, 3e-2), ("gbt", gbt, leaves[4].grad, 3e-2),
              ("gw2", gw2, leaves[5].grad.reshape(K, 64), 3e-2), ("gb2", gb2, leaves[6].grad, 1e-3)]
    errs = {nm: rel(o, ref) for nm, o, ref, _ in checks}
    print("head bf16 persistent-loop errors vs fp32:", errs)
    for nm, _, _, t in checks:
        assert errs[nm] < t, (nm, errs[nm], t)
    assert float(gb1.abs().max()) < 1e-3 * float(gw1.abs().max()) + 1e-5  # pre-BN bias: ~0


@pytest.mark.parametrize("K,N,H,W,shift", [(1, 2, 12, 20, 0.0), (2, 2, 12, 20, 0.0), (3, 1, 9, 13, 0.0),
                                            (2, 2, 32, 24, 6.0)])
def test_head_bf16_batch_stats(K, N, H, W, shift):
    """bf16 head statistics come from the im2col second moments (head_gram_mfma_kernel): mean and
    1/std of h = conv3x3(bf16(u), bf16(W1)) + b1 over the 2H image, against fp64 statistics of the
    same bf16-rounded operands.  Ragged tiles (2H, 2W not multiples of 16) and a z offset of 6
    (mean >> std: the centering's cancellation) included."""
    ops = _ops()
    g = torch.Generator().manual_seed(11)
    z = torch.randn(N, K, H, W, generator=g, dtype=torch.float64) + shift
    w1 = torch.randn(64, K, 3, 3, generator=g, dtype=torch.float64) / 4
    b1 = torch.randn(64, generator=g, dtype=torch.float64) * 0.1
    gamma = torch.rand(64, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(64, generator=g, dtype=torch.float64) * 0.1
    w2 = torch.randn(K, 64, generator=g, dtype=torch.float64) / 8
    b2 = torch.randn(K, generator=g, dtype=torch.float64) * 0.1
    u = F.interpolate(z.float(), scale_factor=2, mode="bilinear", align_corners=False)
    ub = u.bfloat16().double()
    wb = w1.float().bfloat16().double()
    h = F.conv2d(ub, wb, b1.float().double(), padding=1)
    m_ref = h.mean((0, 2, 3))
    v_ref = h.var((0, 2, 3), unbiased=False)
    f = lambda t: t.float().contiguous().to(DEV)
    ws = torch.empty(ops.head_workspace_bytes(N, H, W, K, torch.bfloat16), dtype=torch.uint8, device=DEV)
    rm, rv = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    mean, inv = torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    logits = torch.empty(N, K, H, W, device=DEV)
    ops.head_fwd(f(nhwc(z)), N, H, W, K, f(w1), f(b1), f(gamma), f(beta), f(w2), f(b2), True, 1e-5, 0.1,
                 rm, rv, mean, inv, None, logits, ws, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    inv_ref = 1.0 / torch.sqrt(v_ref + 1e-5)
    assert (mean.double().cpu() - m_ref).abs().max() < 1e-4 * (m_ref.abs().max() + v_ref.sqrt().max())
    assert rel(inv.double().cpu(), inv_ref) < 1e-4
    n = N * 4 * H * W
    assert rel(rv.double().cpu(), 0.9 + 0.1 * v_ref * n / (n - 1)) < 1e-4
    assert rel(rm.double().cpu(), 0.1 * m_ref) < 1e-4


@pytest.mark.parametrize("shift", [0.0, 30.0])
def test_head_bf16_batch_stats_bench_size(shift):
    """The Gram-statistics head BN (head_gram_mfma_kernel) at the bench's size (N 4, 1024^2, K 2: 16.8 M
    pixels at 2H) with logits offset by 30 (|mean| / std ~ 30: the one-pass covariance's cancellation,
    ADVICE r3): mean, 1/std and the running statistics within 1e-4 of fp64 statistics of the same bf16
    operands.  The reference statistics come from the exact im2col second moments in fp64 (torch on the
    GPU): mean_c = w_c . m + b1_c, var_c = w_c^T Cov w_c over the 19-entry column (9 taps x K, zero
    padded at the borders) -- the identity the kernel uses, evaluated without rounding."""
    ops = _ops()
    N, K, H, W = 4, 2, 1024, 1024
    g = torch.Generator(device=DEV).manual_seed(5)
    z = torch.randn(N, K, H, W, generator=g, device=DEV, dtype=torch.float64) * 2 + shift
    w1 = torch.randn(64, K, 3, 3, generator=g, device=DEV, dtype=torch.float64) / 4
    b1 = torch.randn(64, generator=g, device=DEV, dtype=torch.float64) * 0.1
    gamma = torch.rand(64, generator=g, device=DEV, dtype=torch.float64) + 0.5
    beta = torch.randn(64, generator=g, device=DEV, dtype=torch.float64) * 0.1
    w2 = torch.randn(K, 64, generator=g, device=DEV, dtype=torch.float64) / 8
    b2 = torch.randn(K, generator=g, device=DEV, dtype=torch.float64) * 0.1
    ub = F.interpolate(z.float(), scale_factor=2, mode="bilinear", align_corners=False).bfloat16().double()
    wb = w1.float().bfloat16().double().reshape(64, K * 9)
    b1f = b1.float().double()
    n = N * 4 * H * W
    s1 = torch.zeros(K * 9, dtype=torch.float64, device=DEV)
    s2 = torch.zeros(K * 9, K * 9, dtype=torch.float64, device=DEV)
    for i in range(N):  # per sample: the unfolded column is 18 x 4 M fp64
        col = F.unfold(ub[i:i + 1], 3, padding=1)[0]
        s1 += col.sum(1)
        s2 += col @ col.T
        del col
    m = s1 / n
    cov = s2 / n - torch.outer(m, m)
    m_ref = wb @ m + b1f
    v_ref = ((wb @ cov) * wb).sum(1)
    f = lambda t: t.float().contiguous()  # noqa: E731
    ws = torch.empty(ops.head_workspace_bytes(N, H, W, K, torch.bfloat16), dtype=torch.uint8, device=DEV)
    rm, rv = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    mean, inv = torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    logits = torch.empty(N, K, H, W, device=DEV)
    ops.head_fwd(f(z.permute(0, 2, 3, 1)), N, H, W, K, f(w1), f(b1), f(gamma), f(beta), f(w2), f(b2), True, 1e-5,
                 0.1, rm, rv, mean, inv, None, logits, ws, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    inv_ref = 1.0 / torch.sqrt(v_ref + 1e-5)
    em = float((mean.double() - m_ref).abs().max() / v_ref.sqrt().max())
    ei = rel(inv.double(), inv_ref)
    print(f"head Gram stats at 1024^2 x 4, z offset {shift}: mean err / std {em:.2e}, 1/std rel {ei:.2e}")
    assert em < 1e-4 and ei < 1e-4
    assert rel(rv.double(), 0.9 + 0.1 * v_ref * n / (n - 1)) < 1e-4
    assert float((rm.double() - 0.1 * m_ref).abs().max()) < 1e-5 * float(v_ref.sqrt().max())


@pytest.mark.parametrize("K", [2, 3])
def test_loss_fwd_bwd(K):
    from oracle import eunet_ref as R
    ops = _ops()
    g = torch.Generator().manual_seed(8)
    N, H, W = 3, 20, 28
    logits = torch.randn(N, K, H, W, generator=g, dtype=torch.float64) * 2
    target = torch.randint(0, K, (N, H, W), generator=g)
    lt = logits.clone().requires_grad_(True)
    ref = sum(R.combined_loss(lt[i], target[i]) for i in range(N)) / N
    ref.backward()
    from eunet.losses import combined_loss
    ld = logits.float().to(DEV).requires_grad_(True)
    loss, parts = combined_loss(ld, target.to(DEV), return_parts=True)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) < 1e-5 * abs(ref.item())
    assert rel(ld.grad, lt.grad) < 1e-4
    p0 = R.combined_loss(logits[0], target[0], parts=True)[1]
    assert abs(parts[0, 0].item() - p0["focal"].item()) < 1e-5 * abs(p0["focal"].item()) + 1e-7


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_dgrad_bnbwd_fused(dt):
    """dgrad with the BN-backward reduction fused into its epilogue: gx identical to the
    plain dgrad, partial sums equal to (sum g', sum g' xhat) of the stored gx."""
    ops = _ops()
    g = torch.Generator().manual_seed(11)
    N, H, W, Cin, Cout, YT, YO = 2, 20, 44, 64, 128, 144, 16  # gx has Cout channels, y a channel slice
    gy = torch.randn(N, H, W, Cin, generator=g).to(DEV, dt)
    w = (torch.randn(Cin, Cout, 3, 3, generator=g) / 20).to(DEV)  # conv weight [Cin_out][Cout_in]
    ybuf = torch.randn(N, H, W, YT, generator=g).to(DEV, dt)
    mean = torch.randn(Cout, generator=g).to(DEV) * 0.1
    istd = (torch.rand(Cout, generator=g) + 0.5).to(DEV)
    gamma = (torch.rand(Cout, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(Cout, generator=g) * 0.2).to(DEV)
    wpt = ops.conv3x3_pack(w, dt, flip=True)
    gx_ref = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    ops.conv3x3_fwd(ops.act(gy), wpt, ops.act(gx_ref))
    gx = torch.empty_like(gx_ref)
    tiles = ops.conv3x3_tiles(ops.act(gx))
    part = torch.empty(tiles * 2 * Cout, device=DEV)
    sc, sh = gamma * istd, beta - mean * gamma * istd  # the forward affine (defines the ReLU mask)
    ops.conv3x3_dgrad_bnbwd(ops.act(gy), wpt, ops.act(gx), ops.act(ybuf, YO, Cout), mean, istd, sc, sh, part)
    red = torch.empty(2 * Cout, device=DEV)
    ops.colsum(part, tiles, 2 * Cout, red)
    torch.cuda.synchronize()
    assert torch.equal(gx, gx_ref)
    y = ybuf[..., YO:YO + Cout].double()
    xh = (y - mean.double()) * istd.double()
    gp = torch.where(gamma.double() * xh + beta.double() > 0, gx.double(), torch.zeros_like(xh))
    s1 = gp.sum(dim=(0, 1, 2))
    s2 = (gp * xh).sum(dim=(0, 1, 2))
    assert rel(red[:Cout], s1) < 1e-5
    assert rel(red[Cout:], s2) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_per_sample_affine_and_gscale(dt):
    """Dropout2d folded into the operand transform (in_nstride: per-sample scale/shift) for
    the forward and the wgrad, and the per-sample output scale of the fused dgrad."""
    ops = _ops()
    g = torch.Generator().manual_seed(12)
    N, H, W, Cin, Cout = 3, 16, 36, 32, 64
    x = torch.randn(N, H, W, Cin, generator=g).to(dt).double()
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / 17
    sc = torch.rand(N, Cin, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(N, Cin, generator=g, dtype=torch.float64) * 0.3
    keep = (torch.rand(N, Cin, generator=g) > 0.3).double()
    scn, shn = sc * keep / 0.7, sh * keep / 0.7
    xt = tf(x, scn[:, None, None, :], shn[:, None, None, :], dt)
    ref = nhwc(F.conv2d(nchw(xt), w.to(dt).double(), None, padding=1))
    y = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    wp = ops.conv3x3_pack(w.float().to(DEV), dt, flip=False)
    ops.conv3x3_fwd(ops.act(x.to(DEV, dt)), wp, ops.act(y), scale=scn.float().to(DEV), shift=shn.float().to(DEV),
                    nstride=Cin)
    torch.cuda.synchronize()
    assert gate(y, ref, dt) <= 1.0, gate(y, ref, dt)
    gy = torch.randn(N, H, W, Cout, generator=g).to(dt).double()
    ns = ops.conv3x3_wgrad_splits(ops.act(gy.to(DEV, dt)), Cin, dt)
    dwp = torch.empty(ns * Cout * 9 * Cin, device=DEV)
    ops.conv3x3_wgrad(ops.act(x.to(DEV, dt)), ops.act(gy.to(DEV, dt)), dwp, None, ns, scale=scn.float().to(DEV),
                      shift=shn.float().to(DEV), nstride=Cin)
    dw = torch.empty(Cout, Cin, 3, 3, device=DEV)
    ops.wgrad_reduce(dwp, None, ns, Cout, Cin, 9, dw, None)
    wt = w.clone().requires_grad_(True)
    F.conv2d(nchw(xt), wt, None, padding=1).backward(nchw(gy))
    torch.cuda.synchronize()
    assert gate(dw, wt.grad, dt) <= 1.0, gate(dw, wt.grad, dt)
    # dgrad with gscale: gx = conv_transpose(gy) * gs[n][c]
    gs = (keep / 0.7).float().to(DEV)
    wpt = ops.conv3x3_pack(w.float().to(DEV), dt, flip=True)
    gx0 = torch.empty(N, H, W, Cin, dtype=dt, device=DEV)
    ops.conv3x3_fwd(ops.act(gy.to(DEV, dt)), wpt, ops.act(gx0))
    gx = torch.empty_like(gx0)
    yb = torch.randn(N, H, W, Cin, generator=g).to(DEV, dt)
    ones, zeros = torch.ones(Cin, device=DEV), torch.zeros(Cin, device=DEV)
    tiles = ops.conv3x3_tiles(ops.act(gx))
    part = torch.empty(tiles * 2 * Cin, device=DEV)
    ops.conv3x3_dgrad_bnbwd(ops.act(gy.to(DEV, dt)), wpt, ops.act(gx), ops.act(yb), zeros, ones, ones, zeros, part,
                            gscale=gs)
    torch.cuda.synchronize()
    exp = (gx0.double() * gs.double()[:, None, None, :]).to(dt).double()
    assert rel(gx, exp) < (1e-6 if dt == torch.float32 else 1e-2)
    gx_ref = nhwc(F.conv_transpose2d(nchw(gy), w.to(dt).double(), padding=1)) * gs.double().cpu()[:, None, None, :]
    assert gate(gx, gx_ref, dt) <= 1.0, gate(gx, gx_ref, dt)


def test_conv3x3_cin64_ragged_slice():
    """The Cin == 64 bf16 shape (two K-chunks per block, the enc1.3 / dec2.3 layers) through
    conv3x3_fwd_kernel: ragged 16 x 32 tiles at both image edges, a partial third co-block, a
    channel-slice input with the per-sample BN+ReLU transform, bias, BN partials, and the fused
    dgrad epilogue (BN-backward reduction + Dropout2d scale)."""
    ops = _ops()
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(14)
    N, H, W, Cin, Cout, CT, CO = 2, 100, 300, 64, 136, 80, 8
    buf = torch.randn(N, H, W, CT, generator=g).to(DEV, dt)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / 24
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    sc = torch.rand(N, Cin, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(N, Cin, generator=g, dtype=torch.float64) * 0.3
    x = buf.double().cpu()[..., CO:CO + Cin]
    xt = tf(x, sc[:, None, None, :], sh[:, None, None, :], dt)
    ref = nhwc(F.conv2d(nchw(xt), w.to(dt).double(), b.float().double(), padding=1))
    y = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    wp = ops.conv3x3_pack(w.float().to(DEV), dt, flip=False)
    tiles = ops.conv3x3_tiles(ops.act(y))
    st = torch.empty(tiles * (2 * Cout + 1), dtype=torch.float32, device=DEV)
    ops.conv3x3_fwd(ops.act(buf, CO, Cin), wp, ops.act(y), bias=b.float().to(DEV), scale=sc.float().to(DEV),
                    shift=sh.float().to(DEV), nstride=Cin, stats=st)
    gamma, beta = torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    mean, inv = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    s1, s2 = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    ops.bn_finalize(st, tiles, Cout, gamma, beta, 1e-5, 0.1, rm, rv, mean, inv, s1, s2)
    torch.cuda.synchronize()
    assert gate(y, ref, dt) <= 1.0, gate(y, ref, dt)
    assert rel(mean, ref.mean(dim=(0, 1, 2))) < 1e-2
    assert rel(1.0 / inv ** 2 - 1e-5, ref.var(dim=(0, 1, 2), unbiased=False)) < 1e-1
    # dgrad of a 136 -> 64 conv (Cin of the dgrad = 64): gx = conv_transpose(gy) * gs, fused BN-bwd sums
    w2 = torch.randn(Cin, Cout, 3, 3, generator=g, dtype=torch.float64) / 24  # conv weight [64 out][136 in]
    gy = torch.randn(N, H, W, Cin, generator=g).to(dt).double()
    gs = ((torch.rand(N, Cout, generator=g) > 0.3).double() / 0.7)
    yb = torch.randn(N, H, W, Cout, generator=g).to(DEV, dt)
    bm = (torch.randn(Cout, generator=g) * 0.1).to(DEV)
    bi = (torch.rand(Cout, generator=g) + 0.5).to(DEV)
    bgam = (torch.rand(Cout, generator=g) + 0.5).to(DEV)
    bbet = (torch.randn(Cout, generator=g) * 0.2).to(DEV)
    wpt = ops.conv3x3_pack(w2.float().to(DEV), dt, flip=True)
    gx = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    part = torch.empty(tiles * 2 * Cout, device=DEV)
    ops.conv3x3_dgrad_bnbwd(ops.act(gy.to(DEV, dt)), wpt, ops.act(gx), ops.act(yb), bm, bi, bgam * bi,
                            bbet - bm * bgam * bi, part, gscale=gs.float().to(DEV))
    red = torch.empty(2 * Cout, device=DEV)
    ops.colsum(part, tiles, 2 * Cout, red)
    torch.cuda.synchronize()
    gx_ref = nhwc(F.conv_transpose2d(nchw(gy), w2.to(dt).double(), padding=1)) * gs.float().double()[:, None, None, :]
    assert gate(gx, gx_ref, dt) <= 1.0, gate(gx, gx_ref, dt)
    xh = (yb.double() - bm.double()) * bi.double()
    gp = torch.where(bgam.double() * xh + bbet.double() > 0, gx.double(), torch.zeros_like(xh))
    assert rel(red[:Cout], gp.sum(dim=(0, 1, 2))) < 1e-5
    assert rel(red[Cout:], (gp * xh).sum(dim=(0, 1, 2))) < 1e-5


def test_conv3x3_deep_layer_shapes():
    """A deep-layer shape in bf16: Cin 272 (a partial last 32-channel K-chunk), Cout 256 (four
    co-blocks), ragged tiles, a channel-slice input with the per-sample BN+ReLU transform, bias
    and BN partials; then the fused dgrad epilogue (BN-backward reduction + Dropout2d scale) of
    a 288 -> 256 conv, against fp64 references."""
    ops = _ops()
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(15)
    N, H, W, Cin, Cout, CT, CO = 2, 20, 44, 272, 256, 304, 16
    buf = torch.randn(N, H, W, CT, generator=g).to(DEV, dt)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / 50
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    sc = torch.rand(N, Cin, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(N, Cin, generator=g, dtype=torch.float64) * 0.3
    x = buf.double().cpu()[..., CO:CO + Cin]
    xt = tf(x, sc[:, None, None, :], sh[:, None, None, :], dt)
    ref = nhwc(F.conv2d(nchw(xt), w.to(dt).double(), b.float().double(), padding=1))
    y = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    wp = ops.conv3x3_pack(w.float().to(DEV), dt, flip=False)
    tiles = ops.conv3x3_tiles(ops.act(y))
    st = torch.empty(tiles * (2 * Cout + 1), dtype=torch.float32, device=DEV)
    ops.conv3x3_fwd(ops.act(buf, CO, Cin), wp, ops.act(y), bias=b.float().to(DEV), scale=sc.float().to(DEV),
                    shift=sh.float().to(DEV), nstride=Cin, stats=st)
    gamma, beta = torch.ones(Cout, device=DEV), torch.zeros(Cout, device=DEV)
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    mean, inv = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    s1, s2 = torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
    ops.bn_finalize(st, tiles, Cout, gamma, beta, 1e-5, 0.1, rm, rv, mean, inv, s1, s2)
    torch.cuda.synchronize()
    assert gate(y, ref, dt) <= 1.0, gate(y, ref, dt)
    yr = y.double().cpu()  # the stored outputs (stats are taken from the fp32 accumulators)
    assert rel(mean, yr.mean(dim=(0, 1, 2))) < 1e-2
    assert rel(1.0 / inv ** 2 - 1e-5, yr.var(dim=(0, 1, 2), unbiased=False)) < 2e-2
    # dgrad of a 256 -> 288 conv: gx [.., 256] = conv_transpose(gy [.., 288]) * gs, fused BN-bwd sums
    Cd = 288
    w2 = torch.randn(Cd, Cout, 3, 3, generator=g, dtype=torch.float64) / 50  # conv weight [288 out][256 in]
    gy = torch.randn(N, H, W, Cd, generator=g).to(dt).double()
    gs = ((torch.rand(N, Cout, generator=g) > 0.3).double() / 0.7)
    yb = torch.randn(N, H, W, Cout, generator=g).to(DEV, dt)
    bm = (torch.randn(Cout, generator=g) * 0.1).to(DEV)
    bi = (torch.rand(Cout, generator=g) + 0.5).to(DEV)
    bgam = (torch.rand(Cout, generator=g) + 0.5).to(DEV)
    bbet = (torch.randn(Cout, generator=g) * 0.2).to(DEV)
    wpt = ops.conv3x3_pack(w2.float().to(DEV), dt, flip=True)
    gx = torch.empty(N, H, W, Cout, dtype=dt, device=DEV)
    part = torch.empty(tiles * 2 * Cout, device=DEV)
    ops.conv3x3_dgrad_bnbwd(ops.act(gy.to(DEV, dt)), wpt, ops.act(gx), ops.act(yb), bm, bi, bgam * bi,
                            bbet - bm * bgam * bi, part, gscale=gs.float().to(DEV))
    gx_plain = torch.empty_like(gx)
    ops.conv3x3_dgrad(ops.act(gy.to(DEV, dt)), wpt, ops.act(gx_plain))
    red = torch.empty(2 * Cout, device=DEV)
    ops.colsum(part, tiles, 2 * Cout, red)
    torch.cuda.synchronize()
    gx_ref = nhwc(F.conv_transpose2d(nchw(gy), w2.to(dt).double(), padding=1))
    assert gate(gx_plain, gx_ref, dt) <= 1.0, gate(gx_plain, gx_ref, dt)
    assert gate(gx, gx_ref * gs.float().double()[:, None, None, :], dt) <= 1.0
    xh = (yb.double() - bm.double()) * bi.double()
    gp = torch.where(bgam.double() * xh + bbet.double() > 0, gx.double(), torch.zeros_like(xh))
    assert rel(red[:Cout], gp.sum(dim=(0, 1, 2))) < 1e-5
    assert rel(red[Cout:], (gp * xh).sum(dim=(0, 1, 2))) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("h,w", [(7, 9), (8, 16), (1, 3)])
def test_upsample_bwd_odd_sizes(dt, h, w):
    """2x2-per-thread adjoint of the x2 bilinear upsample at odd / tiny low-res sizes."""
    ops = _ops()
    g = torch.Generator().manual_seed(13)
    N, C = 2, 16
    gh = torch.randn(N, 2 * h, 2 * w, C, generator=g, dtype=torch.float64).to(dt).double()
    lo = torch.zeros(N, h, w, C, dtype=torch.float64).requires_grad_(True)
    F.interpolate(nchw(lo), scale_factor=2, mode="bilinear", align_corners=False).backward(nchw(gh))
    glo = torch.empty(N, h, w, C, dtype=dt, device=DEV)
    ops.upsample_bwd(ops.act(gh.to(DEV, dt)), ops.act(glo))
    torch.cuda.synchronize()
    assert rel(glo, lo.grad) < TOL[dt]


@pytest.mark.parametrize("C", [1, 2, 3])
@pytest.mark.parametrize("h,w", [(7, 9), (16, 24), (1, 3)])
def test_upsample_bwd_small_channels(C, h, w):
    """fp32 K-channel adjoint used for the head's logits (K = 2 has its own kernel)."""
    ops = _ops()
    g = torch.Generator().manual_seed(15)
    N = 2
    gh = torch.randn(N, 2 * h, 2 * w, C, generator=g, dtype=torch.float64)
    lo = torch.zeros(N, h, w, C, dtype=torch.float64).requires_grad_(True)
    F.interpolate(nchw(lo), scale_factor=2, mode="bilinear", align_corners=False).backward(nchw(gh))
    glo = torch.empty(N, h, w, C, dtype=torch.float32, device=DEV)
    ops.upsample_bwd(ops.act(gh.to(DEV, torch.float32)), ops.act(glo))
    torch.cuda.synchronize()
    assert rel(glo, lo.grad) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bnrelu(dt):
    """Materialised DoubleConv activation relu(y * scale + shift) on a channel slice."""
    ops = _ops()
    g = torch.Generator().manual_seed(16)
    N, H, W, C, CT, CO = 2, 9, 13, 48, 64, 8
    ybuf = torch.randn(N, H, W, CT, generator=g).to(DEV, dt)
    sc = (torch.rand(C, generator=g) + 0.5).to(DEV)
    sh = (torch.randn(C, generator=g) * 0.3).to(DEV)
    out = torch.empty(N, H, W, C, dtype=dt, device=DEV)
    ops.bnrelu(ops.act(ybuf, CO, C), sc, sh, ops.act(out))
    torch.cuda.synchronize()
    ref = torch.relu(ybuf[..., CO:CO + C].double() * sc.double() + sh.double())
    assert rel(out, ref) < (1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kind", ["pool", "up"])
@pytest.mark.parametrize("C,big", [(64, False), (96, False), (192, False), (768, False), (96, True)])
def test_fused_bn_reduce_in_gradient_producers(dt, kind, C, big):
    """pool_bwd_add / upsample_bwd with the BN-backward reduction fused in: the gradient equals
    the plain kernel's bit for bit, the partial sums equal bn_bwd_reduce on that gradient.  The
    fused max-pool adjoint takes its argmax from relu(y scale + shift) recomputed from y, so the
    saved activation here is the one bnrelu_pool stores for that y (the engine's contract).
    C = 96 / 192 / 768 (base 96: 12 / 24 / 96 bf16 units) run in 192-thread blocks; big: the
    grid-stride loop wraps (more outputs than the capped grid has threads)."""
    ops = _ops()
    g = torch.Generator().manual_seed(17)
    N = 4 if big else 2
    if big:
        h, w = (260, 520) if kind == "pool" else (200, 400)
    else:
        h, w = (10, 14) if kind == "pool" else (7, 9)   # gradient (output) spatial size
    gout = torch.empty(N, h, w, C, dtype=dt, device=DEV)
    gref = torch.empty_like(gout)
    y = torch.randn(N, h, w, C, generator=g).to(DEV, dt)
    mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
    istd = (torch.rand(C, generator=g) + 0.5).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.2).to(DEV)
    sc, sh = gamma * istd, beta - mean * gamma * istd  # the forward affine (defines the ReLU mask)
    if kind == "pool":
        act = torch.empty(N, h, w, C, dtype=dt, device=DEV)
        ops.bnrelu_pool(ops.act(y), sc, sh, ops.act(act), ops.act(torch.empty(N, h // 2, w // 2, C, dtype=dt,
                                                                              device=DEV)))
        gp = torch.randn(N, h // 2, w // 2, C, generator=g).to(DEV, dt)
        gs = torch.randn(N, h, w, C, generator=g).to(DEV, dt)
        ops.pool_bwd_add(ops.act(act), ops.act(gp), ops.act(gs), ops.act(gref))
        rows = ops.pool_bwd_add_bnr_rows(ops.act(gout))
        part = torch.empty(rows * 2 * C, device=DEV)
        ops.pool_bwd_add_bnr(ops.act(act), ops.act(gp), ops.act(gs), ops.act(gout), ops.act(y), mean, istd, sc,
                             sh, part)
    else:
        gh = torch.randn(N, 2 * h, 2 * w, C, generator=g).to(DEV, dt)
        ops.upsample_bwd(ops.act(gh), ops.act(gref))
        rows = ops.upsample_bwd_bnr_rows(ops.act(gout))
        part = torch.empty(rows * 2 * C, device=DEV)
        ops.upsample_bwd_bnr(ops.act(gh), ops.act(gout), ops.act(y), mean, istd, sc, sh, part)
    assert rows > 0
    red = torch.empty(2 * C, device=DEV)
    ops.colsum(part, rows, 2 * C, red)
    tiles = ops.bn_bwd_tiles(ops.act(y))
    p2 = torch.empty(tiles * 2 * C, device=DEV)
    ops.bn_bwd_reduce(ops.act(gref), ops.act(y), mean, istd, sc, sh, p2)
    red2 = torch.empty(2 * C, device=DEV)
    ops.colsum(p2, tiles, 2 * C, red2)
    torch.cuda.synchronize()
    assert torch.equal(gout, gref)
    assert rel(red, red2) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,K", [(64, 2), (64, 1), (96, 3), (128, 2), (8, 3)])
def test_bnrelu_conv1x1_shapes(dt, C, K):
    """dec1 (BN+ReLU -> 1x1 conv): every K, one and two 64-channel groups, a channel slice of a
    wider buffer, and a pixel count that leaves a partial block step (4 x 32 pixels)."""
    ops = _ops()
    g = torch.Generator().manual_seed(40 + C + K)
    N, H, W, CT, CO = 3, 13, 27, C + 16, 8
    buf = torch.randn(N, H, W, CT, generator=g, dtype=torch.float64).to(dt)
    y = buf.double()[..., CO:CO + C]
    sc = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    sh = torch.randn(C, generator=g, dtype=torch.float64) * 0.3
    w = torch.randn(K, C, generator=g, dtype=torch.float64) / 5
    b = torch.randn(K, generator=g, dtype=torch.float64)
    ref = torch.einsum("nhwc,kc->nhwk", torch.relu(y * sc + sh), w) + b
    z = torch.empty(N, H, W, K, device=DEV)
    ops.bnrelu_conv1x1(ops.act(buf.to(DEV), CO, C), sc.float().to(DEV), sh.float().to(DEV), w.float().to(DEV),
                       b.float().to(DEV), K, z)
    torch.cuda.synchronize()
    assert rel(z, ref) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,H,W,C,Cx,nextbn,gs", [(2, 40, 70, 64, 192, False, False),  # 3 co-blocks, ragged
                                                  (1, 64, 96, 128, 64, True, False),   # 4 K-chunks, next BN
                                                  (2, 16, 32, 32, 96, True, True)])    # partial co-block, gscale
def test_conv3x3_dgrad_fused_bn_apply_bit_exact(dt, N, H, W, C, Cx, nextbn, gs):
    """eunet_conv3x3_dgrad_fused (the BN-backward apply in the dgrad's operand staging) against the
    unfused path it replaces, bn_bwd_apply + conv3x3_dgrad(_bnbwd): the stored gy, gx and the next
    BN's reduction rows agree bit for bit, and gy matches the fp64 formula."""
    ops = _ops()
    g0 = torch.Generator().manual_seed(31)
    G = torch.randn(N, H, W, C, generator=g0).to(DEV, dt)
    y = torch.randn(N, H, W, C, generator=g0).to(DEV, dt)
    mean = (torch.randn(C, generator=g0) * 0.1).to(DEV)
    invstd = (torch.rand(C, generator=g0) + 0.5).to(DEV)
    gamma = torch.randn(C, generator=g0).to(DEV)
    beta = torch.randn(C, generator=g0).to(DEV)
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    dbeta = torch.randn(C, generator=g0).to(DEV) * 100
    dgamma = torch.randn(C, generator=g0).to(DEV) * 100
    w = (torch.randn(C, Cx, 3, 3, generator=g0) / (3 * C ** 0.5)).to(DEV)  # conv Cx -> C (dgrad: C -> Cx)
    wpt = ops.conv3x3_pack(w, dt, flip=True)
    yn = torch.randn(N, H, W, Cx, generator=g0).to(DEV, dt) if nextbn else None
    nb = [torch.randn(Cx, generator=g0).to(DEV) * 0.2 + o for o in (0.0, 1.0, 1.0, 0.0)] if nextbn else [None] * 4
    gsc = (torch.rand(N, Cx, generator=g0) + 0.5).to(DEV) if gs else None
    # unfused reference path
    gy_ref = torch.empty_like(G)
    ops.bn_bwd_apply(ops.act(G), ops.act(y), mean, invstd, scale, shift, dbeta, dgamma, ops.act(gy_ref))
    gx_ref = torch.empty(N, H, W, Cx, dtype=dt, device=DEV)
    tiles = ops.conv3x3_tiles(ops.act(gx_ref))
    part_ref = torch.zeros(tiles * 2 * Cx, device=DEV) if nextbn else None
    if nextbn:
        ops.conv3x3_dgrad_bnbwd(ops.act(gy_ref), wpt, ops.act(gx_ref), ops.act(yn), *nb, part_ref, gscale=gsc)
    else:
        ops.conv3x3_dgrad(ops.act(gy_ref), wpt, ops.act(gx_ref), gscale=gsc)
    # fused
    coef = torch.empty(4 * C, device=DEV)
    ops.bn_bwd_coef(mean, invstd, scale, shift, dbeta, dgamma, N * H * W, coef)
    gy = torch.full_like(G, float("nan"))
    gx = torch.empty_like(gx_ref)
    part = torch.zeros_like(part_ref) if nextbn else None
    ops.conv3x3_dgrad_fused(ops.act(G), ops.act(y), coef, ops.act(gy), wpt, ops.act(gx),
                            ops.act(yn) if nextbn else None, *nb, part, gscale=gsc)
    torch.cuda.synchronize()
    assert torch.equal(gy, gy_ref), "gy stored by the fused staging must equal bn_bwd_apply's"
    assert torch.equal(gx, gx_ref)
    if nextbn:
        assert torch.equal(part, part_ref)
    # the formula itself (fp64): gy = scale (g' - dbeta/n - xhat dgamma/n)
    gd, yd = G.double().cpu(), y.double().cpu()
    n = N * H * W
    mask = (yd * scale.double().cpu() + shift.double().cpu()) > 0
    gp = torch.where(mask, gd, torch.zeros_like(gd))
    xh = (yd - mean.double().cpu()) * invstd.double().cpu()
    want = scale.double().cpu() * (gp - dbeta.double().cpu() / n - xh * dgamma.double().cpu() / n)
    assert rel(gy, want) < TOL[dt]
    # the apply with the coefficient table equals the standalone apply too
    gy2 = torch.empty_like(G)
    ops.bn_bwd_apply_coef(ops.act(G), ops.act(y), coef, ops.act(gy2))
    torch.cuda.synchronize()
    assert torch.equal(gy2, gy_ref)


def test_conv3x3_dgrad_bf16_fp32_output():
    """The bf16 data gradient with an fp32 output (the dual-branch gate's g_f2): the same fp32
    accumulators stored without the bf16 rounding -- rounding them gives the bf16-output launch bit
    for bit -- and within fp32 accuracy of the fp64 transposed convolution of the bf16 operands."""
    ops = _ops()
    g0 = torch.Generator().manual_seed(41)
    N, H, W, C, Cx = 2, 40, 72, 256, 8
    dy = torch.randn(N, H, W, C, generator=g0).to(DEV, torch.bfloat16)
    w = (torch.randn(C, Cx, 3, 3, generator=g0) / 48).to(DEV)
    wpt = ops.conv3x3_pack(w, torch.bfloat16, flip=True)
    gb = torch.empty(N, H, W, Cx, dtype=torch.bfloat16, device=DEV)
    gf = torch.empty(N, H, W, Cx, dtype=torch.float32, device=DEV)
    ops.conv3x3_dgrad(ops.act(dy), wpt, ops.act(gb))
    ops.conv3x3_dgrad(ops.act(dy), wpt, ops.act(gf))
    torch.cuda.synchronize()
    assert torch.equal(gf.to(torch.bfloat16), gb)
    ref = nhwc(F.conv_transpose2d(nchw(dy.double().cpu()), w.to(torch.bfloat16).double().cpu(), padding=1))
    assert rel(gf, ref) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv3x3_pack_many_matches_pack(dt):
    """eunet_conv3x3_pack_many (flat block map, 16-byte units) writes exactly what the one-tensor
    pack writes, padding included, for ragged channel counts and both operand roles, across more
    tensors than one launch holds."""
    ops = _ops()
    torch.manual_seed(5)
    shapes = [(64, 1), (64, 3), (5, 7), (96, 130), (512, 256), (33, 64), (2, 17), (128, 192)]
    items = [(torch.randn(co, ci, 3, 3, device=DEV), flip) for co, ci in shapes for flip in (False, True)]
    items = items * 3  # 48 > EUNET_PACK_MAX: two launches
    many = ops.conv3x3_pack_many(items, dt)
    for (w, flip), got in zip(items, many):
        ref = ops.conv3x3_pack(w, dt, flip=flip)
        assert got.shape == ref.shape
        assert torch.equal(got.view(torch.int16 if dt == torch.bfloat16 else torch.int32),
                           ref.view(torch.int16 if dt == torch.bfloat16 else torch.int32)), (w.shape, flip)

