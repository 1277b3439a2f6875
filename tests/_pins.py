"""Branch configuration of a GPU training forward, for the branch-pinned oracle (test infrastructure).

The kernels decide each ReLU from the BatchNorm affine of the stored pre-BN conv output,
fmaf(y, scale, shift) > 0 (conv3x3 operand staging, bnrelu_pool / bnrelu_upsample / bnrelu_conv1x1,
and every BN-backward site), and each 2x2 max-pool from round(relu(fmaf(y, scale, shift))) in the
compute dtype with the first maximum in row-major order winning (bnrelu_pool_kernel; the adjoint
recomputes the same argmax).  The same rules evaluated here on the engine's own saved tensors
(UNetEngine.keep_state) give the oracle (oracle/eunet_ref.py _relu / _pool) the branches the GPU
took.  In fp64, y * scale is exact for fp32 / bf16 operands, so the sign of y * scale + shift is the
sign of the fused multiply-add's exact result -- the mask is the kernel's.  The pooled values are
rounded fp64 -> fp32 (-> bf16): a double rounding that can differ from the kernel's single rounding
only for results exactly between two representable values, which does not occur in these tests'
inputs in practice (a wrong pin would show as a single-element gradient outlier).

Not pinned: the 2H head's ReLU (enhance.1; its pre-BN input is recomputed inside the head kernels and
never stored) -- the oracle keeps its own branches there.  With K <= 3 input channels the head conv's
fp32 error is ~1e-7 relative, so a branch can differ only for activations within ~1e-7 of the kink.
"""
import torch

POOLED = ("enc1", "enc2", "enc3")


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def relu_mask(y, scale, shift):
    """fmaf(y, scale, shift) > 0 per element, y NHWC (any float dtype), scale / shift [C] or [N, C];
    returns a bool NCHW tensor on the CPU."""
    y = y.detach().double().cpu()
    sc, sh = scale.detach().double().cpu(), shift.detach().double().cpu()
    if sc.dim() == 2:
        sc, sh = sc[:, None, None, :], sh[:, None, None, :]
    return _nchw((y * sc + sh) > 0).contiguous()


def pool_argmax(y, scale, shift, dtype):
    """2x2 argmax (0..3, row-major, first maximum wins) of round_dtype(relu(fmaf(y, scale, shift)))."""
    y = y.detach().double().cpu()
    v = (y * scale.detach().double().cpu() + shift.detach().double().cpu()).float()
    if dtype == torch.bfloat16:
        v = v.bfloat16().float()
    v = _nchw(v.clamp_min(0.0))
    B, C, H, W = v.shape
    w = v.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
    idx = torch.zeros(B, C, H // 2, W // 2, dtype=torch.long)
    best = w[..., 0].clone()
    for j in (1, 2, 3):
        gt = w[..., j] > best  # strictly greater: the first maximum stays
        idx[gt] = j
        best = torch.where(gt, w[..., j], best)
    return idx


def trunk_pins(S, dtype):
    """UNetEngine.forward_trunk state -> eunet_ref.trunk pins."""
    pins = {}
    for nm in ("enc1", "enc2", "enc3", "enc4", "dec4", "dec3", "dec2"):
        s = S[nm]
        pins[nm + ".1"] = relu_mask(s["ya"], s["bna"]["scale"], s["bna"]["shift"])
        pins[nm + ".4"] = relu_mask(s["yb"], s["bnb"]["scale"], s["bnb"]["shift"])
    for i, nm in enumerate(POOLED, 1):
        s = S[nm]
        pins[f"pool{i}"] = pool_argmax(s["yb"], s["bnb"]["scale"], s["bnb"]["shift"], dtype)
    return pins


def model_pins(model):
    """Pins of the last training forward of an EnhancedUNet whose engine had keep_state set."""
    eng = model._engine
    S = eng.last_state
    if not getattr(model, "dual_branch", False):
        return trunk_pins(S, eng.dtype)
    pins = {"unetpp": trunk_pins(S["SA"], eng.dtype), "deeplab": trunk_pins(S["SB"], eng.dtype)}
    # fusion head: the ReLU after each BN is applied by the next kernel with the BN affine
    # (Dropout2d folded in: relu(x) * m = relu(x * m) for m >= 0; a dropped channel passes nothing
    # either way, so the mask of the un-dropped affine is used)
    for key, y, h in (("fusion_head.1", "y1", "h1"), ("fusion_head.5", "y2", "h2"), ("fusion_head.9", "y3", "h3")):
        pins[key] = relu_mask(S[y], S[h]["scale"], S[h]["shift"])
    return pins


def keep(model, on=True):
    model._engine.keep_state = on
    return model


# ---- audit: the pins must be the oracle's own branches up to rounding ---------------------------------
# A pin is adopted by the oracle without question, so a kernel bug that flipped masks far from the kink
# (a wrong shift channel, a tile-seam indexing error in the stored ya / yb) would be copied into the
# oracle's forward and backward.  audit() compares every pin with the oracle's OWN branch at the same
# element (the ReLU input / pool window the pinned oracle computed, record= of eunet_ref.forward /
# dual_ref.dual_forward) and requires each disagreement to sit within `tol` x max|h| of the kink (ReLU)
# or of a tie (pool: the oracle's top value minus its value at the pinned index).
TOL_FP32 = 1e-5
TOL_BF16 = 2e-2  # ~5 bf16 units of roundoff (2^-8) of the largest activation: the floor of the bf16 bound
# bf16: rounding accumulates over the 15 layers, so a deep layer's activations sit a few % of their
# scale from fp64 for ANY bf16 implementation.  The bf16 bound is therefore relative to the reference
# itself: per site 2 x the worst disputed |h| of the oracle run under CPU bf16 autocast (audit(...,
# ref=) with the autocast run's own pins, pins_from_record), floored at TOL_BF16.


def _audit_trunk(pins, rec, tol, out, prefix=""):
    for key, pin in pins.items():
        if key.startswith("pool"):
            continue
        h = rec[key].double()
        pin = pin.to(torch.bool)
        dis = (h > 0) != pin
        n = int(dis.sum())
        worst = float(h[dis].abs().max() / h.abs().max()) if n else 0.0
        out[prefix + key] = (n, worst)
    for i in (1, 2, 3):
        key = f"pool{i}"
        if key not in pins:
            continue
        v = rec[f"enc{i}.4"].double().clamp_min(0.0)
        B, C, H, W = v.shape
        w = v.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
        top, own = w.max(-1)  # first maximum, as the kernels' rule
        at_pin = w.gather(-1, pins[key].long().unsqueeze(-1)).squeeze(-1)
        dis = own != pins[key].long()
        n = int(dis.sum())
        worst = float((top - at_pin)[dis].max() / v.max().clamp_min(1e-300)) if n else 0.0
        out[prefix + key] = (n, worst)


def pins_from_record(rec):
    """Pins of an oracle run's own branches from its record (ReLU inputs, NCHW): mask = h > 0; pool argmax
    (first maximum) of relu(h) of the pooled blocks' second ReLU.  Trunk or dual layout."""
    if "unetpp" in rec:
        out = {"unetpp": pins_from_record(rec["unetpp"]), "deeplab": pins_from_record(rec["deeplab"])}
        out.update({k: (v > 0) for k, v in rec.items() if k.startswith("fusion_head")})
        return out
    pins = {k: (v > 0) for k, v in rec.items()}
    for i, nm in enumerate(POOLED, 1):
        v = rec[nm + ".4"].double().clamp_min(0.0)
        B, C, H, W = v.shape
        w = v.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
        idx = torch.zeros(B, C, H // 2, W // 2, dtype=torch.long)
        best = w[..., 0].clone()
        for j in (1, 2, 3):
            gt = w[..., j] > best
            idx[gt] = j
            best = torch.where(gt, w[..., j], best)
        pins[f"pool{i}"] = idx
    return pins


def audit(pins, rec, dtype, tol=None, label="", ref=None):
    """Assert that every pin disagreeing with the oracle's own branch is within tol (relative to the
    site's largest activation) of the kink / tie; return {site: (disputed count, worst ratio)} and print
    the totals.  pins / rec: trunk dicts, or the dual layout ({'unetpp': .., 'deeplab': .., 'fusion_head.k'})."""
    tol = tol if tol is not None else (TOL_BF16 if dtype in (torch.bfloat16, "bf16") else TOL_FP32)
    out = {}
    if "unetpp" in pins:
        _audit_trunk(pins["unetpp"], rec["unetpp"], tol, out, "unetpp.")
        _audit_trunk(pins["deeplab"], rec["deeplab"], tol, out, "deeplab.")
        _audit_trunk({k: v for k, v in pins.items() if k.startswith("fusion_head")}, rec, tol, out)
    else:
        _audit_trunk(pins, rec, tol, out)
    total = sum(n for n, _ in out.values())
    worst = max((w, k) for k, (_, w) in out.items())
    site_tol = {k: max(tol, 2.0 * ref[k][1]) if ref else tol for k in out}
    ratio = max((out[k][1] / site_tol[k], k) for k in out)
    print(f"pin audit {label}: {total} disputed branch(es) over {len(out)} sites, worst {worst[0]:.2e} of max|h| "
          f"at {worst[1]}; worst / bound {ratio[0]:.2f} at {ratio[1]} (floor {tol:.0e}"
          + (", 2 x the bf16-autocast oracle's own)" if ref else ")"))
    bad = {k: (v, site_tol[k]) for k, v in out.items() if v[1] > site_tol[k]}
    assert not bad, f"pins far from the oracle's own kink / tie (a kernel branch bug?): {bad}"
    return out


def autocast_reference(run_autocast, run_fp64):
    """The bf16 audit's reference: run_autocast(record) runs the oracle forward under CPU bf16 autocast
    filling record; its own branches (pins_from_record) are audited against run_fp64(pins, record), the
    fp64 oracle pinned to them.  Returns that audit's {site: (count, worst)} for audit(..., ref=)."""
    rac = {}
    with torch.no_grad():
        run_autocast(rac)
    pac = pins_from_record(rac)
    del rac
    r64 = {}
    with torch.no_grad():
        run_fp64(pac, r64)
    return audit(pac, r64, "bf16", tol=float("inf"), label="bf16-autocast oracle (the bound's reference)")
