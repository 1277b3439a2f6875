"""Explicit forward/backward schedule of the Enhanced-UNet hot path over libeunet_hip.

Reference structure (models.py:199-240, 304-339):
    e1 = enc1(x); e2 = enc2(pool(e1)); e3 = enc3(pool(e2)); e4 = enc4(pool(e3))
    d4 = dec4(cat[up(e4), e3]); d3 = dec3(cat[up(d4), e2]); d2 = dec2(cat[up(d3), e1])
    out = u + enhance(u),  u = dec1(up(d2))  (== up(dec1(d2)), computed that way)

Data layout in HBM (NHWC, dtype = fp32 or bf16):
  * each DoubleConv keeps only its two PRE-BatchNorm conv outputs y_a, y_b;
    BN+ReLU of y_a is applied inside the operand load of conv b (and of the
    wgrad that needs it); BN+ReLU of y_b is applied by its single consumer
    (pool / upsample / dec1 kernel), so no post-ReLU tensor of a block is
    written except the skip activations;
  * the skip activations e1..e3 and the upsampled decoder inputs are written
    straight into their concat buffers cat2/cat3/cat4 (torch.cat never runs);
  * the 2H tail is fused in the head kernels (never materialised).
Backward mirrors it; every parameter gradient is written into a slot handed
out by a GradSink (the data-parallel sink launches bucketed all-reduces as
soon as a bucket is complete, overlapping RCCL with the rest of backward).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import kprof, ops
from ._lib import EunetError

ENCODER_SCOPE = "conv3x3.encoder_train"  # kprof family of every encoder conv3x3 launch (fwd, dgrad, wgrad)

BLOCKS = ("enc1", "enc2", "enc3", "enc4", "dec4", "dec3", "dec2")
BN_EPS = 1e-5
BN_MOMENTUM = 0.1
class Grad1x1:
    """A gradient w.r.t. relu(bn(y)) held as dec1's W^T g_z instead of a tensor (UNetEngine.dec1_recompute)."""

    def __init__(self, w, k, gz):
        self.w, self.k, self.gz = w, k, gz


class GradPool:
    """A gradient w.r.t. relu(bn(y)) held as gskip + maxpool-adjoint(gpool) (UNetEngine.pool_recompute)."""

    def __init__(self, gpool, gskip):
        self.gpool, self.gskip = gpool, gskip


class GradSink:
    """Default sink: a fresh fp32 tensor per parameter gradient."""

    def __init__(self, device):
        self.device = device
        self.grads: Dict[str, torch.Tensor] = {}

    def slot(self, name: str, shape) -> torch.Tensor:
        t = torch.empty(shape, dtype=torch.float32, device=self.device)
        self.grads[name] = t
        return t

    def ready(self, names):  # hook point for data-parallel overlap
        pass

    def finish(self):
        return self.grads


def _e(shape, dtype, device):
    return torch.empty(shape, dtype=dtype, device=device)


_SIDE = {}


def side_stream(device) -> torch.cuda.Stream:
    """The per-device side stream the weight gradients run on (see UNetEngine.overlap_wgrad)."""
    key = torch.device(device).index
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


def _per_block(flag, nm) -> bool:
    """An engine knob that is a collection of block names, or any other value taken as a bool (every
    block or none: True / False / 0 / 1)."""
    if isinstance(flag, (set, frozenset, list, tuple)):
        return nm in flag
    return bool(flag)


class UNetEngine:
    """One BasicUNet trunk (+ the enhance head for the single-branch model).  prefix names the
    trunk's parameters in the owning module ('model.' for EnhancedUNet, 'unetpp.' / 'deeplab.'
    for the branches of the dual-branch model).

    overlap_wgrad: the weight gradients of each DoubleConv (wgrad + split reduction) run on a
    side stream, concurrently with the data-gradient chain (dgrad, BN backward) on the launch
    stream; the two meet again before the gradients are handed out.  Same kernels and operands,
    so the results are bit-identical either way."""

    overlap_wgrad = True
    # Schedule choices, with their measured defaults (instance or class attributes; the library and
    # this module read nothing from the process environment):
    # materialize_za -- DoubleConv's first BN+ReLU, za = relu(bn1(ya)), for the second conv:
    #   False (default since round 2): applied inside both operand stagings (nothing stored); the
    #     forward's halo staging loads the BN constants once per K-chunk with the halo, so the
    #     transform is free there, and the weight gradient pays it on the side stream; A/B +0.9 /
    #     +2.1 % img/s (profiles/r02_ab_za.txt; round 1's opposite result: profiles/r01_ab_za.txt)
    #   True: one elementwise pass on the main stream; conv .3's forward and wgrad read za as is
    materialize_za = False
    # fuse_bn_reduce -- a block's BN-b backward reduction fused into the kernel producing its output
    # gradient (upsample / max-pool / 1x1 adjoints) instead of a separate bn_bwd_reduce pass
    fuse_bn_reduce = True
    # wg3_late -- conv .3's weight gradient joins the side stream after the block's BN-a backward
    # rather than before conv .3's data gradient: the side stream's wgrad blocks hold whole CUs
    # (256 VGPRs x 8 waves), and bn_bwd_apply on the critical launch stream waited for CU slots;
    # this way the wgrad overlaps conv .0's data gradient instead.  A/B +0.6 % img/s, 6 of 7
    # alternating pairs on one box (profiles/r02_ab_conv.txt)
    wg3_late = True
    # wg3_early_last -- in the trunk's last block (no input gradient, so no conv .0 data gradient follows
    # to overlap), conv .3's weight gradient joins the side stream as soon as its dY is ready instead of
    # running at the step's tail (profiles/r04_step_timeline.txt).  Measured neutral (173.0-174.7 vs
    # 173.6-174.2 img/s, three alternating pairs, profiles/r04_ab.txt): off
    wg3_early_last = False
    # fuse_bn_apply -- the apply half of the DoubleConv's second BatchNorm backward (gy = k1 g' + k2
    # y + k3) inside conv .3's data-gradient operand staging (eunet_conv3x3_dgrad_fused), which also
    # stores gy for conv .3's weight gradient.  Same values, bit for bit, but measured slower: the
    # dgrad's staging carries two loads per halo unit, the transform and the gy stores while the
    # standalone apply streams at ~4.9 TB/s beside the side stream's weight gradients -- 26.0-26.1 vs
    # 25.3-25.5 ms/step in three alternating same-box rounds (profiles/r03_ab.txt).  Off by default.
    # A set of block names ({"enc4", "dec4"}) fuses those blocks only.
    fuse_bn_apply = False
    # fuse_bn_apply_a -- the same for the first BatchNorm (conv .0's data gradient; needs
    # fuse_bn_apply).  Off: conv .0's weight gradient then has to wait for that dgrad and overlaps the
    # next level's HBM-bound upsample / max-pool adjoints instead of the dgrad (they ran 2.7x longer:
    # +0.85 ms/step in a same-box A/B, profiles/r03_ab.txt)
    fuse_bn_apply_a = False
    # dec1_recompute -- dec1's input gradient W^T g_z (64 channels at H) is not stored: conv1x1_bwd only
    # reduces it for dec2's second BatchNorm, and that BatchNorm's apply recomputes it per pixel from g_z
    # (eunet_bn_bwd_apply_1x1: the same gy bit for bit, 2 x 537 MB less HBM traffic at the bench shape).
    # Needs fuse_bn_reduce and dec2 outside fuse_bn_apply (whose fused dgrad reads the stored gradient).
    dec1_recompute = True
    # pool_recompute -- the same for the encoders' output gradients gskip + maxpool-adjoint(gpool):
    # pool_bwd_add_bnr only reduces them, the block's apply recomputes them per 2x2 window
    # (eunet_bn_bwd_apply_pool: the same gy bit for bit, 0.75 C per pixel less traffic).  Needs
    # fuse_bn_reduce, the block outside fuse_bn_apply, and even H and W at the level.  Round 5 measured it
    # equal (182.4 vs 182.7 img/s, profiles/r05_ab.txt r5pr); with round 6's weight gradient it is +0.3 / +1.0 %
    # in two same-box runs of three alternating rounds each (profiles/r06_ab.txt r6pr): on
    pool_recompute = True
    # dgrad_first -- after a DoubleConv's BN-a backward, conv .0's data gradient is issued on the launch
    # stream before the side-stream weight gradients (which wait on an event recorded right after the
    # apply, not on the launch stream's tail).  Closes half of the ~24 us apply -> dgrad launch-stream gap
    # per block, but the dgrads then take the CUs first and the squeezed weight gradients spread over the
    # HBM-bound kernels: step time unchanged in a same-box A/B (+0.1 %), the conv family's wall-time
    # fraction 0.369 -> 0.341 (profiles/r03_ab.txt).  Off by default.
    dgrad_first = False
    # fork_once -- after a DoubleConv's BN-a backward, the side stream's three waits on the launch stream
    # (conv .3's and conv .0's weight gradients, the bucket hook) share one event recorded there, instead of
    # one wait_stream each (each record is a marker packet the launch stream's next kernel, conv .0's data
    # gradient, queues behind: ~21 us per block).  Measured slower: 173.6-174.1 vs 175.5-176.6 img/s in four
    # alternating pairs (profiles/r04_ab.txt) -- like dgrad_first, a data gradient that reaches the CUs
    # before the side stream's weight gradients costs the step more than the gap.  Off.
    fork_once = False
    # device_fence_forks -- the side stream's forks and joins wait through eunet_stream_wait (events with a
    # device-scope release) instead of torch's Stream.wait_stream (a system-scope release: an L2 writeback
    # and invalidate on the launch stream at every fork)
    device_fence_forks = True
    # keep_state -- tests: the last training forward's saved tensors (pre-BN conv outputs, BN affines)
    # stay reachable as self.last_state, so a checker can read the branch configuration (ReLU masks,
    # max-pool argmax) the kernels took (tests/_pins.py)
    keep_state = False

    def _wait(self, to, frm):
        """stream `to` waits for the work enqueued on `frm` so far"""
        if self.device_fence_forks:
            ops.stream_wait(frm, to)
        else:
            to.wait_stream(frm)

    def __init__(self, model, prefix: str = "model."):
        self.m = model
        self.prefix = prefix
        self.base = model.base_ch
        self.K = model.num_classes
        self.cin = model.in_channels
        self.dtype = model.compute_dtype

    # ------------------------------------------------------------------ utils
    def _P(self):
        return dict(self.m.named_parameters())

    def _B(self):
        return dict(self.m.named_buffers())

    def _bn(self, prefix, stats, tiles, C, training, P, B):
        dev = P[prefix + ".weight"].device
        scale, shift = _e(C, torch.float32, dev), _e(C, torch.float32, dev)
        if training:
            mean, invstd = _e(C, torch.float32, dev), _e(C, torch.float32, dev)
            ops.bn_finalize(stats, tiles, C, P[prefix + ".weight"], P[prefix + ".bias"], BN_EPS, BN_MOMENTUM,
                            B[prefix + ".running_mean"], B[prefix + ".running_var"], mean, invstd, scale, shift,
                            B[prefix + ".num_batches_tracked"])
            return dict(mean=mean, invstd=invstd, scale=scale, shift=shift)
        ops.bn_eval_affine(P[prefix + ".weight"], P[prefix + ".bias"], B[prefix + ".running_mean"],
                           B[prefix + ".running_var"], BN_EPS, scale, shift)
        return dict(mean=None, invstd=None, scale=scale, shift=shift)

    def _stats_buf(self, y):
        tiles = ops.conv3x3_tiles(ops.act(y))
        C = y.shape[3]
        return _e(tiles * (2 * C + 1), torch.float32, y.device), tiles

    def _pack_all(self, P, training: bool):
        """Every 3x3 weight of the trunk packed in one launch: the forward operands and, when
        training, the dgrad (transposed + flipped) operands -- the weights do not change between
        this forward and its backward.  name -> packed tensor; flipped ones under name + "^T"."""
        items, names = [], []
        for nm in BLOCKS:
            p = f"{self.prefix}{nm}"
            for i in ((3,) if nm == "enc1" else (0, 3)):  # enc1.0 runs on the direct small-Cin kernel
                items.append((P[f"{p}.{i}.weight"], False))
                names.append(f"{p}.{i}.weight")
            if training:
                for i in ((3,) if nm == "enc1" else (3, 0)):
                    items.append((P[f"{p}.{i}.weight"], True))
                    names.append(f"{p}.{i}.weight^T")
        return dict(zip(names, ops.conv3x3_pack_many(items, self.dtype)))

    def _block_fwd(self, nm, X: ops.Act, training, P, B, small: bool, wps=None):
        with kprof.scope(ENCODER_SCOPE if nm.startswith("enc") else None):
            return self._block_fwd_impl(nm, X, training, P, B, small, wps)

    def _block_fwd_impl(self, nm, X: ops.Act, training, P, B, small: bool, wps=None):
        p = f"{self.prefix}{nm}"
        N, H, W = X.n, X.h, X.w
        C = P[p + ".0.weight"].shape[0]
        dev = P[p + ".0.weight"].device
        ya = _e((N, H, W, C), self.dtype, dev)
        yb = _e((N, H, W, C), self.dtype, dev)
        st, tiles = self._stats_buf(ya) if training else (None, 0)
        enc = "conv3x3_fwd.encoder" if nm.startswith("enc") else None  # bench: the encoder's MFMA convs
        if small:
            ops.conv_small_fwd(X, P[p + ".0.weight"], P[p + ".0.bias"], ops.act(ya), st)
        else:
            wp = wps[p + ".0.weight"] if wps else ops.conv3x3_pack(P[p + ".0.weight"], self.dtype, flip=False)
            ops.conv3x3_fwd(X, wp, ops.act(ya), bias=P[p + ".0.bias"], stats=st, sub=enc)
        bna = self._bn(p + ".1", st, tiles, C, training, P, B)
        wp = wps[p + ".3.weight"] if wps else ops.conv3x3_pack(P[p + ".3.weight"], self.dtype, flip=False)
        za = None
        if self.materialize_za:  # one BN+ReLU pass; conv .3 forward and weight gradient read za as is
            za = _e((N, H, W, C), self.dtype, dev)
            ops.bnrelu(ops.act(ya), bna["scale"], bna["shift"], ops.act(za))
            ops.conv3x3_fwd(ops.act(za), wp, ops.act(yb), bias=P[p + ".3.bias"], stats=st, sub=enc)
        else:  # BN+ReLU applied while staging conv .3's operand tiles (forward and wgrad)
            ops.conv3x3_fwd(ops.act(ya), wp, ops.act(yb), bias=P[p + ".3.bias"], scale=bna["scale"],
                            shift=bna["shift"], stats=st, sub=enc)
        bnb = self._bn(p + ".4", st, tiles, C, training, P, B)
        return dict(ya=ya, za=za, yb=yb, bna=bna, bnb=bnb, X=X)

    # ---------------------------------------------------------------- forward
    def forward(self, x: torch.Tensor, training: bool, want: str = "logits"):
        """x [N,Cin,H,W] fp32 -> logits [N,K,H,W] ('logits', the 2x2 mean of the
        2H output) or out2h [N,K,2H,2W] ('out2h', the reference forward)."""
        S = self.forward_trunk(x, training)
        P, B = self._P(), self._B()
        N, H, W, K, dev = S["N"], S["H"], S["W"], self.K, x.device
        z = S["z"]
        hws = _e(ops.head_workspace_bytes(N, H, W, K, self.dtype), torch.uint8, dev)
        hmean = _e(64, torch.float32, dev) if training else None
        hinv = _e(64, torch.float32, dev) if training else None
        out2h = _e((N, K, 2 * H, 2 * W), torch.float32, dev) if want == "out2h" else None
        logits = _e((N, K, H, W), torch.float32, dev) if want == "logits" else None
        ops.head_fwd(z, N, H, W, K, P["enhance.0.weight"], P["enhance.0.bias"], P["enhance.1.weight"],
                     P["enhance.1.bias"], P["enhance.3.weight"].reshape(K, 64).contiguous(), P["enhance.3.bias"],
                     training, BN_EPS, BN_MOMENTUM, B["enhance.1.running_mean"], B["enhance.1.running_var"],
                     hmean, hinv, out2h, logits, hws, dtype=self.dtype)
        if training:
            guard = ops.update_guard(dev)  # eunet_bn_finalize counts the other BNs' batches under it
            if guard is None:
                B["enhance.1.num_batches_tracked"].add_(1)
            else:
                B["enhance.1.num_batches_tracked"].add_(guard.eq(0).long().reshape(()))
        S.update(hmean=hmean, hinv=hinv, want=want)
        return (logits if want == "logits" else out2h), S

    def forward_trunk(self, x: torch.Tensor, training: bool):
        """BasicUNet trunk up to z = dec1(d2) at input resolution, NHWC fp32 [N,H,W,K]
        (models.py:227-237 with dec1 commuted before the final upsample)."""
        if not x.is_cuda:
            raise EunetError("EnhancedUNet (eunet) runs on the GPU only; no CPU fallback")
        N, Cin, H, W = x.shape
        if Cin != self.cin:
            raise ValueError(f"expected {self.cin} input channels, got {Cin}")
        if H % 8 or W % 8:
            raise ValueError("H and W must be multiples of 8 (the reference pads to /32)")
        P, B = self._P(), self._B()
        dt, dev, b, K = self.dtype, x.device, self.base, self.K
        ch = [b, 2 * b, 4 * b, 8 * b]
        lv = [(H >> i, W >> i) for i in range(4)]
        S = {}
        wps = self._pack_all(P, training)
        S["wp"] = wps
        xin = _e((N, H, W, Cin), dt, dev)
        ops.nchw_to_nhwc(x.contiguous().float(), xin)
        cat4 = _e((N, *lv[2], ch[3] + ch[2]), dt, dev)
        cat3 = _e((N, *lv[1], ch[2] + ch[1]), dt, dev)
        cat2 = _e((N, *lv[0], ch[1] + ch[0]), dt, dev)
        p1 = _e((N, *lv[1], ch[0]), dt, dev)
        p2 = _e((N, *lv[2], ch[1]), dt, dev)
        p3 = _e((N, *lv[3], ch[2]), dt, dev)
        S.update(xin=xin, cat4=cat4, cat3=cat3, cat2=cat2, p1=p1, p2=p2, p3=p3)

        def consume_pool(nm, cat, coff, pooled):
            s = S[nm]
            ops.bnrelu_pool(ops.act(s["yb"]), s["bnb"]["scale"], s["bnb"]["shift"],
                            ops.act(cat, coff, s["yb"].shape[3]), ops.act(pooled))

        def consume_up(nm, cat):
            s = S[nm]
            ops.bnrelu_upsample(ops.act(s["yb"]), s["bnb"]["scale"], s["bnb"]["shift"],
                                ops.act(cat, 0, s["yb"].shape[3]))

        S["enc1"] = self._block_fwd("enc1", ops.act(xin), training, P, B, small=True, wps=wps)
        consume_pool("enc1", cat2, ch[1], p1)
        S["enc2"] = self._block_fwd("enc2", ops.act(p1), training, P, B, small=False, wps=wps)
        consume_pool("enc2", cat3, ch[2], p2)
        S["enc3"] = self._block_fwd("enc3", ops.act(p2), training, P, B, small=False, wps=wps)
        consume_pool("enc3", cat4, ch[3], p3)
        S["enc4"] = self._block_fwd("enc4", ops.act(p3), training, P, B, small=False, wps=wps)
        consume_up("enc4", cat4)
        S["dec4"] = self._block_fwd("dec4", ops.act(cat4), training, P, B, small=False, wps=wps)
        consume_up("dec4", cat3)
        S["dec3"] = self._block_fwd("dec3", ops.act(cat3), training, P, B, small=False, wps=wps)
        consume_up("dec3", cat2)
        S["dec2"] = self._block_fwd("dec2", ops.act(cat2), training, P, B, small=False, wps=wps)
        s = S["dec2"]
        z = _e((N, H, W, K), torch.float32, dev)
        ops.bnrelu_conv1x1(ops.act(s["yb"]), s["bnb"]["scale"], s["bnb"]["shift"],
                           P[self.prefix + "dec1.weight"].reshape(K, b).contiguous(), P[self.prefix + "dec1.bias"], K, z)
        S.update(z=z, N=N, H=H, W=W)
        return S

    # --------------------------------------------------------------- backward
    def _block_bwd(self, nm, G, S, P, sink, need_gx: bool, small: bool, gred=(None, 0)):
        with kprof.scope(ENCODER_SCOPE if nm.startswith("enc") else None):
            return self._block_bwd_impl(nm, G, S, P, sink, need_gx, small, gred)

    def _block_bwd_impl(self, nm, G: "torch.Tensor | Grad1x1 | GradPool", S, P, sink: GradSink, need_gx: bool,
                        small: bool, gred=(None, 0)):
        """gred: (part, rows) of the block's BN-b backward reduction when G's producer fused it."""
        p = f"{self.prefix}{nm}"
        s = S[nm]
        ya, yb, bna, bnb, X = s["ya"], s["yb"], s["bna"], s["bnb"], s["X"]
        N, H, W, C = yb.shape
        dev, dt = yb.device, self.dtype

        def bn_back(prefix, g, y, bn, part=None, tiles=0):
            if isinstance(g, (Grad1x1, GradPool)):  # reduced by its producer, recomputed by the apply
                dbeta, dgamma = sink.slot(prefix + ".bias", (C,)), sink.slot(prefix + ".weight", (C,))
                ops.colsum(part, tiles, 2 * C, dbeta, split=C, out_hi=dgamma)
                gy = torch.empty_like(y)
                if isinstance(g, Grad1x1):
                    ops.bn_bwd_apply_1x1(ops.act(y), g.w, g.k, g.gz, bn["mean"], bn["invstd"], bn["scale"],
                                         bn["shift"], dbeta, dgamma, ops.act(gy))
                else:
                    ops.bn_bwd_apply_pool(g.gpool, g.gskip, ops.act(y), bn["mean"], bn["invstd"], bn["scale"],
                                          bn["shift"], dbeta, dgamma, ops.act(gy))
                return gy
            if part is None:  # reduction not fused into the producer of g
                tiles = ops.bn_bwd_tiles(ops.act(y))
                part = _e(tiles * 2 * C, torch.float32, dev)
                ops.bn_bwd_reduce(ops.act(g), ops.act(y), bn["mean"], bn["invstd"], bn["scale"],
                                  bn["shift"], part)
            dbeta, dgamma = sink.slot(prefix + ".bias", (C,)), sink.slot(prefix + ".weight", (C,))
            ops.colsum(part, tiles, 2 * C, dbeta, split=C, out_hi=dgamma)
            gy = torch.empty_like(y)
            ops.bn_bwd_apply(ops.act(g), ops.act(y), bn["mean"], bn["invstd"], bn["scale"],
                             bn["shift"], dbeta, dgamma, ops.act(gy))
            return gy

        def dgrad0(gya):  # conv .0's data gradient (the block's input gradient)
            wpt = S["wp"].get(p + ".0.weight^T") if S.get("wp") else None
            if wpt is None:
                wpt = ops.conv3x3_pack(P[p + ".0.weight"], dt, flip=True)
            gx = _e((N, H, W, X.c), dt, dev)
            ops.conv3x3_dgrad(ops.act(gya), wpt, ops.act(gx))
            return gx

        main = torch.cuda.current_stream(dev)
        side = side_stream(dev) if self.overlap_wgrad else None

        def wgrad(conv, xa: ops.Act, gy, scale=None, shift=None, small_conv=False, on_main=False, ready=None):
            # the gradient slots are allocated on the launch stream (their consumers run there)
            dw = sink.slot(conv + ".weight", (C, xa.c, 3, 3))
            db = sink.slot(conv + ".bias", (C,))
            if side is None or on_main:
                return wgrad_on_stream(xa, gy, dw, db, scale, shift, small_conv)
            if ready is not None:
                side.wait_event(ready)  # recorded on the launch stream once gy was complete
            else:
                self._wait(side, main)  # gy (and everything before it) is ready
            with torch.cuda.stream(side):
                wgrad_on_stream(xa, gy, dw, db, scale, shift, small_conv)
            for t in (gy, xa._keep, dw, db):  # the caching allocator must not hand these out early
                t.record_stream(side)

        def wgrad_on_stream(xa: ops.Act, gy, dw, db, scale=None, shift=None, small_conv=False):
            cin = xa.c
            gya = ops.act(gy)
            if small_conv:
                ns = ops.conv_small_wgrad_splits(gya)
            else:
                ns = ops.conv3x3_wgrad_splits(gya, cin, dt)
            dwp = _e(ns * C * 9 * cin, torch.float32, dev)
            dbp = _e(ns * C, torch.float32, dev)
            if small_conv:
                ops.conv_small_wgrad(xa, gya, dwp, dbp, ns)
            else:
                ops.conv3x3_wgrad(xa, gya, dwp, dbp, ns, scale=scale, shift=shift)
            ops.wgrad_reduce(dwp, dbp, ns, C, cin, 9, dw, db)

        if _per_block(self.fuse_bn_apply, nm):
            return self._block_bwd_fused(nm, G, S, P, sink, need_gx, small, gred, wgrad, side, main)
        gyb = bn_back(p + ".4", G, yb, bnb, part=gred[0], tiles=gred[1])

        def wgrad3():
            if s.get("za") is not None:
                wgrad(p + ".3", ops.act(s["za"]), gyb)
            else:
                wgrad(p + ".3", ops.act(ya), gyb, bna["scale"], bna["shift"])
        early3 = not self.wg3_late or (self.wg3_early_last and not need_gx)
        if early3:
            wgrad3()
        wpt = S["wp"].get(p + ".3.weight^T") if S.get("wp") else None
        if wpt is None:
            wpt = ops.conv3x3_pack(P[p + ".3.weight"], dt, flip=True)
        gaa = torch.empty_like(ya)
        ctiles = ops.conv3x3_tiles(ops.act(gaa))
        cpart = _e(ctiles * 2 * C, torch.float32, dev)
        ops.conv3x3_dgrad_bnbwd(ops.act(gyb), wpt, ops.act(gaa), ops.act(ya), bna["mean"], bna["invstd"],
                                bna["scale"], bna["shift"], cpart)
        gya = bn_back(p + ".1", gaa, ya, bna, part=cpart, tiles=ctiles)
        ev = None
        gx = None
        if side is not None and (self.fork_once or (self.dgrad_first and need_gx)):
            ev = torch.cuda.Event()
            ev.record(main)  # gyb, gya and the BN-parameter gradients are complete
            if self.dgrad_first and need_gx:
                gx = dgrad0(gya)
        if not early3:
            if s.get("za") is not None:
                wgrad(p + ".3", ops.act(s["za"]), gyb, ready=ev)
            else:
                wgrad(p + ".3", ops.act(ya), gyb, bna["scale"], bna["shift"], ready=ev)
        del gyb
        # the trunk's last weight gradient (no data gradient follows it): on the main stream, which is
        # otherwise idle here, instead of queueing behind the side stream's conv .3 wgrad
        wgrad(p + ".0", X, gya, small_conv=small, on_main=not need_gx, ready=ev)
        del gaa
        names = [f"{p}.{i}.{w}" for i in (0, 1, 3, 4) for w in ("weight", "bias")]
        if side is None:
            sink.ready(names)
        else:  # a bucket all-reduce launched here orders after both streams' work, without stalling main
            if ev is not None:
                side.wait_event(ev)
            else:
                self._wait(side, main)
            with torch.cuda.stream(side):
                sink.ready(names)
        if not need_gx:
            return None
        return gx if gx is not None else dgrad0(gya)

    def _block_bwd_fused(self, nm, G, S, P, sink, need_gx, small, gred, wgrad, side, main):
        """_block_bwd with each BN backward's apply fused into the data gradient that consumes it:
        colsum -> (dbeta, dgamma) -> coefficient table; the dgrad stages gy = k1 g' + k2 y + k3 from
        (g, y) and stores it for the weight gradient, which therefore follows its dgrad."""
        p = f"{self.prefix}{nm}"
        s = S[nm]
        ya, yb, bna, bnb, X = s["ya"], s["yb"], s["bna"], s["bnb"], s["X"]
        N, H, W, C = yb.shape
        dev, dt = yb.device, self.dtype

        def bn_coef(prefix, g, y, bn, part=None, tiles=0):
            if part is None:  # reduction not fused into the producer of g
                tiles = ops.bn_bwd_tiles(ops.act(y))
                part = _e(tiles * 2 * C, torch.float32, dev)
                ops.bn_bwd_reduce(ops.act(g), ops.act(y), bn["mean"], bn["invstd"], bn["scale"],
                                  bn["shift"], part)
            dbeta, dgamma = sink.slot(prefix + ".bias", (C,)), sink.slot(prefix + ".weight", (C,))
            ops.colsum(part, tiles, 2 * C, dbeta, split=C, out_hi=dgamma)
            coef = _e(4 * C, torch.float32, dev)
            ops.bn_bwd_coef(bn["mean"], bn["invstd"], bn["scale"], bn["shift"], dbeta, dgamma, N * H * W, coef)
            return coef

        def packed(conv):
            wpt = S["wp"].get(conv + ".weight^T") if S.get("wp") else None
            return wpt if wpt is not None else ops.conv3x3_pack(P[conv + ".weight"], dt, flip=True)

        coefb = bn_coef(p + ".4", G, yb, bnb, part=gred[0], tiles=gred[1])
        gyb = torch.empty_like(yb)
        gaa = torch.empty_like(ya)
        ctiles = ops.conv3x3_tiles(ops.act(gaa))
        cpart = _e(ctiles * 2 * C, torch.float32, dev)
        ops.conv3x3_dgrad_fused(ops.act(G), ops.act(yb), coefb, ops.act(gyb), packed(p + ".3"), ops.act(gaa),
                                ops.act(ya), bna["mean"], bna["invstd"], bna["scale"], bna["shift"], cpart)

        def wgrad3():
            if s.get("za") is not None:
                wgrad(p + ".3", ops.act(s["za"]), gyb)
            else:
                wgrad(p + ".3", ops.act(ya), gyb, bna["scale"], bna["shift"])
        early3 = not self.wg3_late or (self.wg3_early_last and not need_gx)
        if early3:
            wgrad3()
        coefa = bn_coef(p + ".1", gaa, ya, bna, part=cpart, tiles=ctiles)
        if self.wg3_late:
            wgrad3()
        del gyb
        gya = torch.empty_like(ya)
        gx = None
        if need_gx and _per_block(self.fuse_bn_apply_a, nm):
            gx = _e((N, H, W, X.c), dt, dev)
            ops.conv3x3_dgrad_fused(ops.act(gaa), ops.act(ya), coefa, ops.act(gya), packed(p + ".0"), ops.act(gx))
            wgrad(p + ".0", X, gya, small_conv=small)
        else:  # gy materialised; conv .0's weight gradient overlaps its data gradient (round 2's order)
            ops.bn_bwd_apply_coef(ops.act(gaa), ops.act(ya), coefa, ops.act(gya))
            # the trunk's last weight gradient (no data gradient follows it): on the then idle main stream
            wgrad(p + ".0", X, gya, small_conv=small, on_main=not need_gx)
            if need_gx:
                gx = _e((N, H, W, X.c), dt, dev)
                ops.conv3x3_dgrad(ops.act(gya), packed(p + ".0"), ops.act(gx))
        del gaa, gya
        names = [f"{p}.{i}.{w}" for i in (0, 1, 3, 4) for w in ("weight", "bias")]
        if side is None:
            sink.ready(names)
        else:  # a bucket all-reduce launched here orders after both streams' work, without stalling main
            self._wait(side, main)
            with torch.cuda.stream(side):
                sink.ready(names)
        return gx

    def backward(self, S, g_out: torch.Tensor, sink: Optional[GradSink] = None):
        P = self._P()
        N, H, W, K, b = S["N"], S["H"], S["W"], self.K, self.base
        dev, dt = g_out.device, self.dtype
        ch = [b, 2 * b, 4 * b, 8 * b]
        sink = sink or GradSink(dev)
        g_out = g_out.contiguous().float()
        # ---- 2H head -> gz
        gz = _e((N, H, W, K), torch.float32, dev)
        hws = _e(ops.head_workspace_bytes(N, H, W, K, dt), torch.uint8, dev)
        gw1 = sink.slot("enhance.0.weight", (64, K, 3, 3))
        gb1 = sink.slot("enhance.0.bias", (64,))
        gg = sink.slot("enhance.1.weight", (64,))
        gbt = sink.slot("enhance.1.bias", (64,))
        gw2 = sink.slot("enhance.3.weight", (K, 64, 1, 1))
        gb2 = sink.slot("enhance.3.bias", (K,))
        glog = g_out if S["want"] == "logits" else None
        gout2h = g_out if S["want"] == "out2h" else None
        ops.head_bwd(S["z"], N, H, W, K, P["enhance.0.weight"], P["enhance.0.bias"], P["enhance.1.weight"],
                     P["enhance.1.bias"], P["enhance.3.weight"].reshape(K, 64).contiguous(), S["hmean"], S["hinv"],
                     glog, gout2h, gz, gw1, gb1, gg, gbt, gw2, gb2, hws, dtype=dt)
        sink.ready(["enhance.0.weight", "enhance.0.bias", "enhance.1.weight", "enhance.1.bias",
                    "enhance.3.weight", "enhance.3.bias"])
        self.backward_trunk(S, gz, sink)
        return sink.finish()

    def backward_trunk(self, S, gz: torch.Tensor, sink: GradSink):
        """Backward of forward_trunk from gz = d loss / d z (NHWC fp32 [N,H,W,K]): every trunk gradient
        is written into (and reported ready to) the sink; the caller calls sink.finish()."""
        P = self._P()
        N, H, W, K, b = S["N"], S["H"], S["W"], self.K, self.base
        dev, dt = gz.device, self.dtype
        ch = [b, 2 * b, 4 * b, 8 * b]
        pre = self.prefix

        def bnr_args(nm):
            s = S[nm]
            return (ops.act(s["yb"]), s["bnb"]["mean"], s["bnb"]["invstd"], s["bnb"]["scale"], s["bnb"]["shift"])

        def up_bwd(ghi: ops.Act, glo: torch.Tensor, nm):
            """g w.r.t. block nm's output from the upsample adjoint, its BN-b reduction fused."""
            rows = ops.upsample_bwd_bnr_rows(ops.act(glo)) if self.fuse_bn_reduce else 0
            if not rows:
                ops.upsample_bwd(ghi, ops.act(glo))
                return None, 0
            part = _e(rows * 2 * glo.shape[3], torch.float32, dev)
            ops.upsample_bwd_bnr(ghi, ops.act(glo), *bnr_args(nm), part)
            return part, rows

        def pool_bwd(act_saved: ops.Act, gpool: ops.Act, gskip: ops.Act, shape, nm):
            """block nm's output gradient (a tensor, or GradPool when the apply recomputes it) and the
            (part, rows) of its fused BN-b reduction."""
            rows = ops.pool_bwd_add_bnr_rows(act_saved) if self.fuse_bn_reduce else 0  # (gout's shape)
            if not rows:
                gout = _e(shape, dt, dev)
                ops.pool_bwd_add(act_saved, gpool, gskip, ops.act(gout))
                return gout, (None, 0)
            part = _e(rows * 2 * shape[3], torch.float32, dev)
            if (self.pool_recompute and not _per_block(self.fuse_bn_apply, nm) and shape[1] % 2 == 0
                    and shape[2] % 2 == 0):
                ops.pool_bwd_add_bnr(act_saved, gpool, gskip, None, *bnr_args(nm), part)
                return GradPool(gpool, gskip), (part, rows)
            gout = _e(shape, dt, dev)
            ops.pool_bwd_add_bnr(act_saved, gpool, gskip, ops.act(gout), *bnr_args(nm), part)
            return gout, (part, rows)

        # ---- dec1 (1x1) -> gradient w.r.t. d2 = relu(bn(y_b of dec2))
        s2 = S["dec2"]
        yb_act = ops.act(s2["yb"])
        tiles = ops.conv1x1_bwd_tiles(yb_act)
        part = _e(tiles * (K * b + K), torch.float32, dev)
        w1 = P[pre + "dec1.weight"].reshape(K, b).contiguous()
        bnb2 = s2["bnb"]
        red2 = (None, 0)
        if self.fuse_bn_reduce:
            bpart = _e(tiles * 2 * b, torch.float32, dev)
            if self.dec1_recompute and not _per_block(self.fuse_bn_apply, "dec2"):
                gd2 = Grad1x1(w1, K, gz)
                ops.conv1x1_bwd_bnr(yb_act, bnb2["scale"], bnb2["shift"], w1, K, gz, None, part,
                                    bnb2["mean"], bnb2["invstd"], bpart)
            else:
                gd2 = torch.empty_like(s2["yb"])
                ops.conv1x1_bwd_bnr(yb_act, bnb2["scale"], bnb2["shift"], w1, K, gz, ops.act(gd2), part,
                                    bnb2["mean"], bnb2["invstd"], bpart)
            red2 = (bpart, tiles)
        else:
            gd2 = torch.empty_like(s2["yb"])
            ops.conv1x1_bwd(yb_act, bnb2["scale"], bnb2["shift"], w1, K, gz, ops.act(gd2), part)
        # the column sums go straight into the two gradient slots (colsum's split output)
        ops.colsum(part, tiles, K * b + K, sink.slot(pre + "dec1.weight", (K, b, 1, 1)), split=K * b,
                   out_hi=sink.slot(pre + "dec1.bias", (K,)))
        sink.ready([pre + "dec1.weight", pre + "dec1.bias"])
        # ---- decoder
        g_cat2 = self._block_bwd("dec2", gd2, S, P, sink, need_gx=True, small=False, gred=red2)
        del gd2
        g_d3 = _e((N, H >> 1, W >> 1, ch[1]), dt, dev)
        red = up_bwd(ops.act(g_cat2, 0, ch[1]), g_d3, "dec3")
        g_cat3 = self._block_bwd("dec3", g_d3, S, P, sink, need_gx=True, small=False, gred=red)
        del g_d3
        g_d4 = _e((N, H >> 2, W >> 2, ch[2]), dt, dev)
        red = up_bwd(ops.act(g_cat3, 0, ch[2]), g_d4, "dec4")
        g_cat4 = self._block_bwd("dec4", g_d4, S, P, sink, need_gx=True, small=False, gred=red)
        del g_d4
        g_e4 = _e((N, H >> 3, W >> 3, ch[3]), dt, dev)
        red = up_bwd(ops.act(g_cat4, 0, ch[3]), g_e4, "enc4")
        # ---- encoder (skip gradients + max-pool backward)
        g_p3 = self._block_bwd("enc4", g_e4, S, P, sink, need_gx=True, small=False, gred=red)
        del g_e4
        g_e3, red = pool_bwd(ops.act(S["cat4"], ch[3], ch[2]), ops.act(g_p3), ops.act(g_cat4, ch[3], ch[2]),
                             (N, H >> 2, W >> 2, ch[2]), "enc3")
        del g_p3, g_cat4
        g_p2 = self._block_bwd("enc3", g_e3, S, P, sink, need_gx=True, small=False, gred=red)
        del g_e3
        g_e2, red = pool_bwd(ops.act(S["cat3"], ch[2], ch[1]), ops.act(g_p2), ops.act(g_cat3, ch[2], ch[1]),
                             (N, H >> 1, W >> 1, ch[1]), "enc2")
        del g_p2, g_cat3
        g_p1 = self._block_bwd("enc2", g_e2, S, P, sink, need_gx=True, small=False, gred=red)
        del g_e2
        g_e1, red = pool_bwd(ops.act(S["cat2"], ch[1], ch[0]), ops.act(g_p1), ops.act(g_cat2, ch[1], ch[0]),
                             (N, H, W, ch[0]), "enc1")
        del g_p1, g_cat2
        self._block_bwd("enc1", g_e1, S, P, sink, need_gx=False, small=True, gred=red)
        if self.overlap_wgrad:
            self._wait(torch.cuda.current_stream(dev), side_stream(dev))
        # the caller finishes the sink: the dual-branch model runs two trunks into one sink (finishing it
        # here made a DataParallel BucketSink wait for buckets the second trunk had not filled yet)


class UNetFunction(torch.autograd.Function):
    """autograd boundary: forward/backward of the whole network in one node."""

    @staticmethod
    def forward(ctx, x, want, engine, sink_factory, *params):
        out, S = engine.forward(x, training=True, want=want)
        if engine.keep_state:
            engine.last_state = S
        ctx.S = S
        ctx.engine = engine
        ctx.sink_factory = sink_factory
        ctx.names = [n for n, _ in engine.m.named_parameters()]
        return out

    @staticmethod
    def backward(ctx, g):
        sink = ctx.sink_factory() if ctx.sink_factory is not None else None
        grads = ctx.engine.backward(ctx.S, g, sink)
        ctx.S = None
        return (None, None, None, None) + tuple(grads.get(n) for n in ctx.names)
