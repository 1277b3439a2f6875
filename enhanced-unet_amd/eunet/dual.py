"""Dual-branch Enhanced-UNet (the reference's SMP path) on the HIP kernels.

Reference (models.py:253-302 construction, 316-333 forward):
    out_main = unetpp(x); out_aux = deeplab(x); ff = cat(out_main, out_aux)
    ff = ff * attention_gate(ff)       # Conv3x3(2K->K) BN GELU Conv1x1(K->2K) BN Sigmoid
    fused = fusion_head(ff) + fusion_residual(ff)
    _aux_outputs = {'unetpp': out_main, 'deeplab': out_aux}
The SMP backbones are third-party and need pretrained weights (absent here); the
branches are BasicUNet trunks ending at input resolution (oracle/dual_ref.py
documents the definition and its pinning).

Schedule (all network arithmetic in libeunet_hip):
  trunks      UNetEngine.forward_trunk x2 -> za, zb [N,H,W,K] fp32 NHWC
  gate        gate_fwd / gate_mid_fwd / gate_out_fwd (fusion.hip), BN finalize between
  head        conv_small_fwd (2K->256), conv3x3_fwd (256->128, 128->64) on MFMA with
              BN+ReLU(+Dropout2d as a per-sample affine) fused into each operand load
  output      fusion_out_fwd: 1x1 head + residual -> fused [N,K,H,W] NCHW
Backward mirrors it (fusion_out_bwd, conv1x1_bwd, BN backward, wgrad / dgrad with the
Dropout2d scale in the dgrad epilogue, gate_bwd1-3) and ends in the two trunks.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from . import engine, ops
from .engine import BN_EPS, BN_MOMENTUM, GradSink, UNetEngine, _e

DROP_P = (0.2, 0.15)   # models.py:287, 291
HEAD_CH = (256, 128, 64)  # models.py:285-293
BRANCHES = ("unetpp", "deeplab")


class DualEngine:
    # narrow_mfma -- fusion_head.0 (2K -> 256 channels, 3x3) on the MFMA forward over f2's 8 zero-padded
    # channels instead of conv_small_fwd's per-pixel FMAs (3.7 ms per launch at configs[4]): HBM-bound on its
    # output (profiles/r05_ab.txt r5d)
    narrow_mfma = True

    def __init__(self, model):
        self.m = model
        self.K = model.num_classes
        self.ea = UNetEngine(model, prefix="unetpp.")
        self.eb = UNetEngine(model, prefix="deeplab.")
        self.drop_keep = None  # tests: fixed ([N,256], [N,128]) keep masks instead of bernoulli draws
        self.keep_state = False  # tests: keep the last training forward's state as last_state (engine.py)

    @property
    def dtype(self):
        return self.ea.dtype

    @dtype.setter
    def dtype(self, dt):
        self.ea.dtype = dt
        self.eb.dtype = dt

    def _P(self):
        return dict(self.m.named_parameters())

    def _B(self):
        return dict(self.m.named_buffers())

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, training: bool):
        SA = self.ea.forward_trunk(x, training)
        SB = self.eb.forward_trunk(x, training)
        P, B = self._P(), self._B()
        K, dt, dev = self.K, self.dtype, x.device
        N, H, W = SA["N"], SA["H"], SA["W"]
        za, zb = SA["z"], SB["z"]
        bn = self.ea._bn
        tiles, _ = ops.fusion_tiles(N, H, W)
        S = dict(SA=SA, SB=SB, N=N, H=H, W=W, training=training)
        # ---- attention gate (models.py:278-284, 322-323)
        a = _e((N, H, W, K), torch.float32, dev)
        st1 = _e(tiles * (2 * K + 1), torch.float32, dev)
        aux_a = _e((N, K, H, W), torch.float32, dev)
        aux_b = _e((N, K, H, W), torch.float32, dev)
        ops.gate_fwd(za, zb, K, P["attention_gate.0.weight"].contiguous(), a, st1, aux_a, aux_b)
        g1 = bn("attention_gate.1", st1, tiles, K, training, P, B)
        b = _e((N, H, W, 2 * K), torch.float32, dev)
        st2 = _e(tiles * (4 * K + 1), torch.float32, dev)
        ops.gate_mid_fwd(za, zb, K, a, g1["scale"], g1["shift"], P["attention_gate.3.weight"].reshape(2 * K, K)
                         .contiguous(), b, st2)
        g2 = bn("attention_gate.4", st2, tiles, 2 * K, training, P, B)
        f2 = torch.zeros((N, H, W, 8), dtype=dt, device=dev)
        ops.gate_out_fwd(za, zb, K, b, g2["scale"], g2["shift"], ops.act(f2, 0, 2 * K))
        S.update(a=a, b=b, g1=g1, g2=g2, f2=f2)
        # ---- fusion head (models.py:285-294)
        y1 = _e((N, H, W, HEAD_CH[0]), dt, dev)
        st, ct = self.ea._stats_buf(y1) if training else (None, 0)
        if self.narrow_mfma:
            ops.conv3x3_fwd_narrow(ops.act(f2), 2 * K, ops.conv3x3_pack(P["fusion_head.0.weight"], dt, flip=False),
                                   ops.act(y1), stats=st)
        else:
            ops.conv_small_fwd(ops.act(f2, 0, 2 * K), P["fusion_head.0.weight"].contiguous(), None, ops.act(y1), st)
        h1 = bn("fusion_head.1", st, ct, HEAD_CH[0], training, P, B)
        d1 = self._dropout(h1, 0, N, training, dev)
        y2 = _e((N, H, W, HEAD_CH[1]), dt, dev)
        st, ct = self.ea._stats_buf(y2) if training else (None, 0)
        ops.conv3x3_fwd(ops.act(y1), ops.conv3x3_pack(P["fusion_head.4.weight"], dt, flip=False), ops.act(y2),
                        scale=d1["scale"], shift=d1["shift"], stats=st, nstride=d1["nstride"])
        h2 = bn("fusion_head.5", st, ct, HEAD_CH[1], training, P, B)
        d2 = self._dropout(h2, 1, N, training, dev)
        y3 = _e((N, H, W, HEAD_CH[2]), dt, dev)
        st, ct = self.ea._stats_buf(y3) if training else (None, 0)
        ops.conv3x3_fwd(ops.act(y2), ops.conv3x3_pack(P["fusion_head.8.weight"], dt, flip=False), ops.act(y3),
                        scale=d2["scale"], shift=d2["shift"], stats=st, nstride=d2["nstride"])
        h3 = bn("fusion_head.9", st, ct, HEAD_CH[2], training, P, B)
        out = _e((N, K, H, W), torch.float32, dev)
        ops.fusion_out_fwd(za, zb, K, ops.act(y3), h3["scale"], h3["shift"],
                           P["fusion_head.11.weight"].reshape(K, HEAD_CH[2]).contiguous(), P["fusion_head.11.bias"],
                           b, g2["scale"], g2["shift"], P["fusion_residual.weight"].reshape(K, 2 * K).contiguous(),
                           P["fusion_residual.bias"], out)
        S.update(y1=y1, y2=y2, y3=y3, h1=h1, h2=h2, h3=h3, d1=d1, d2=d2)
        return out, aux_a, aux_b, S

    def _dropout(self, h, i, N, training, dev):
        """Dropout2d(p) after BN+ReLU folded into per-sample affines (eunet_dropout_affine)."""
        if not training:
            return dict(scale=h["scale"], shift=h["shift"], nstride=0, gscale=None)
        C = h["scale"].numel()
        if self.drop_keep is not None:
            keep = self.drop_keep[i].to(dev, torch.float32).contiguous()
        else:
            keep = torch.empty((N, C), dtype=torch.float32, device=dev).bernoulli_(1.0 - DROP_P[i])
        sc, sh, gs = (_e((N, C), torch.float32, dev) for _ in range(3))
        ops.dropout_affine(h["scale"], h["shift"], keep, DROP_P[i], sc, sh, gs)
        return dict(scale=sc, shift=sh, nstride=C, gscale=gs)

    # ----------------------------------------------------------------- backward
    def _bn_back(self, prefix, g, y, bn, P, sink, part=None, tiles=0):
        C = y.shape[3]
        dev = y.device
        if part is None:
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

    def _wgrad(self, name, xa: ops.Act, gy, sink, d=None):
        C = gy.shape[3]
        dev = gy.device
        gya = ops.act(gy)
        ns = ops.conv3x3_wgrad_splits(gya, xa.c, self.dtype)
        dwp = _e(ns * C * 9 * xa.c, torch.float32, dev)
        ops.conv3x3_wgrad(xa, gya, dwp, None, ns, scale=d["scale"], shift=d["shift"], nstride=d["nstride"])
        ops.wgrad_reduce(dwp, None, ns, C, xa.c, 9, sink.slot(name, (C, xa.c, 3, 3)), None)

    def backward(self, S, g_out, g_aux_a, g_aux_b, sink: Optional[GradSink] = None):
        P = self._P()
        K, dt = self.K, self.dtype
        N, H, W = S["N"], S["H"], S["W"]
        dev = g_out.device
        sink = sink or GradSink(dev)
        za, zb = S["SA"]["z"], S["SB"]["z"]
        tiles, gtiles = ops.fusion_tiles(N, H, W)
        g1, g2, h1, h2, h3, d1, d2 = (S[k] for k in ("g1", "g2", "h1", "h2", "h3", "d1", "d2"))
        y1, y2, y3, a, b, f2 = (S[k] for k in ("y1", "y2", "y3", "a", "b", "f2"))
        g_out = g_out.contiguous().float()
        # ---- output 1x1 + residual (models.py:294, 296, 325-328)
        gz = _e((N, H, W, K), torch.float32, dev)
        gf2res = _e((N, H, W, 2 * K), torch.float32, dev)
        nv = K * 2 * K + K
        part = _e(tiles * nv, torch.float32, dev)
        ops.fusion_out_bwd(za, zb, K, g_out, b, g2["scale"], g2["shift"],
                           P["fusion_residual.weight"].reshape(K, 2 * K).contiguous(), gz, gf2res, part)
        red = _e(nv, torch.float32, dev)
        ops.colsum(part, tiles, nv, red)
        sink.slot("fusion_residual.weight", (K, 2 * K, 1, 1)).copy_(red[:2 * K * K].view(K, 2 * K, 1, 1))
        sink.slot("fusion_residual.bias", (K,)).copy_(red[2 * K * K:])
        C3 = HEAD_CH[2]
        g3 = torch.empty_like(y3)
        ct = ops.conv1x1_bwd_tiles(ops.act(y3))
        part = _e(ct * (K * C3 + K), torch.float32, dev)
        w11 = P["fusion_head.11.weight"].reshape(K, C3).contiguous()
        red3 = (None, 0)
        if engine.UNetEngine.fuse_bn_reduce:
            bpart = _e(ct * 2 * C3, torch.float32, dev)
            ops.conv1x1_bwd_bnr(ops.act(y3), h3["scale"], h3["shift"], w11, K, gz, ops.act(g3), part,
                                h3["mean"], h3["invstd"], bpart)
            red3 = (bpart, ct)
        else:
            ops.conv1x1_bwd(ops.act(y3), h3["scale"], h3["shift"], w11, K, gz, ops.act(g3), part)
        red = _e(K * C3 + K, torch.float32, dev)
        ops.colsum(part, ct, K * C3 + K, red)
        sink.slot("fusion_head.11.weight", (K, C3, 1, 1)).copy_(red[:K * C3].view(K, C3, 1, 1))
        sink.slot("fusion_head.11.bias", (K,)).copy_(red[K * C3:])
        sink.ready(["fusion_residual.weight", "fusion_residual.bias", "fusion_head.11.weight", "fusion_head.11.bias"])
        # ---- conv 128->64 (fusion_head.8/.9)
        gy3 = self._bn_back("fusion_head.9", g3, y3, h3, P, sink, part=red3[0], tiles=red3[1])
        del g3
        self._wgrad("fusion_head.8.weight", ops.act(y2), gy3, sink, d2)
        gg2 = torch.empty_like(y2)
        ct = ops.conv3x3_tiles(ops.act(gg2))
        cpart = _e(ct * 2 * HEAD_CH[1], torch.float32, dev)
        ops.conv3x3_dgrad_bnbwd(ops.act(gy3), ops.conv3x3_pack(P["fusion_head.8.weight"], dt, flip=True),
                                ops.act(gg2), ops.act(y2), h2["mean"], h2["invstd"], h2["scale"],
                                h2["shift"], cpart, gscale=d2["gscale"])
        del gy3
        sink.ready(["fusion_head.9.weight", "fusion_head.9.bias", "fusion_head.8.weight"])
        # ---- conv 256->128 (fusion_head.4/.5)
        gy2 = self._bn_back("fusion_head.5", gg2, y2, h2, P, sink, part=cpart, tiles=ct)
        del gg2
        self._wgrad("fusion_head.4.weight", ops.act(y1), gy2, sink, d1)
        gg1 = torch.empty_like(y1)
        ct = ops.conv3x3_tiles(ops.act(gg1))
        cpart = _e(ct * 2 * HEAD_CH[0], torch.float32, dev)
        ops.conv3x3_dgrad_bnbwd(ops.act(gy2), ops.conv3x3_pack(P["fusion_head.4.weight"], dt, flip=True),
                                ops.act(gg1), ops.act(y1), h1["mean"], h1["invstd"], h1["scale"],
                                h1["shift"], cpart, gscale=d1["gscale"])
        del gy2
        sink.ready(["fusion_head.5.weight", "fusion_head.5.bias", "fusion_head.4.weight"])
        # ---- conv 2K->256 (fusion_head.0/.1)
        gy1 = self._bn_back("fusion_head.1", gg1, y1, h1, P, sink, part=cpart, tiles=ct)
        del gg1
        f2a = ops.act(f2, 0, 2 * K)
        ns = ops.conv_small_wgrad_splits(ops.act(gy1))
        dwp = _e(ns * HEAD_CH[0] * 9 * 2 * K, torch.float32, dev)
        ops.conv_small_wgrad(f2a, ops.act(gy1), dwp, None, ns)
        ops.wgrad_reduce(dwp, None, ns, HEAD_CH[0], 2 * K, 9, sink.slot("fusion_head.0.weight", (HEAD_CH[0], 2 * K, 3, 3)),
                         None)
        # g_f2 leaves the bf16 dgrad in fp32: the gate backward's BN sums cancel strongly, and a
        # bf16-rounded g_f2 left attention_gate.1's gradient at 1.1 relative L2 vs the fp64 oracle
        # (bf16 autocast of the reference: 0.24; tests/test_gpu_dual.py bf16 gradient parity)
        gf2c = _e((N, H, W, 8), torch.float32, dev)
        ops.conv3x3_dgrad(ops.act(gy1), ops.conv3x3_pack(P["fusion_head.0.weight"], dt, flip=True), ops.act(gf2c))
        del gy1
        sink.ready(["fusion_head.1.weight", "fusion_head.1.bias", "fusion_head.0.weight"])
        # ---- attention gate backward
        gffd = _e((N, H, W, 2 * K), torch.float32, dev)
        gbhat = _e((N, H, W, 2 * K), torch.float32, dev)
        part = _e(tiles * 4 * K, torch.float32, dev)
        ops.gate_bwd1(za, zb, K, ops.act(gf2c), gf2res, b, g2["mean"], g2["invstd"], P["attention_gate.4.weight"],
                      P["attention_gate.4.bias"], gffd, gbhat, part)
        red2 = _e(4 * K, torch.float32, dev)
        ops.colsum(part, tiles, 4 * K, red2)
        sink.slot("attention_gate.4.bias", (2 * K,)).copy_(red2[:2 * K])
        sink.slot("attention_gate.4.weight", (2 * K,)).copy_(red2[2 * K:])
        nv = 2 * K * K + 2 * K
        gabn = _e((N, H, W, K), torch.float32, dev)
        part = _e(tiles * nv, torch.float32, dev)
        ops.gate_bwd2(N, H, W, K, gbhat, b, g2["mean"], g2["invstd"], P["attention_gate.4.weight"], red2[:2 * K],
                      red2[2 * K:], a, g1["mean"], g1["invstd"], P["attention_gate.1.weight"],
                      P["attention_gate.1.bias"], P["attention_gate.3.weight"].reshape(2 * K, K).contiguous(), gabn,
                      part)
        red1 = _e(nv, torch.float32, dev)
        ops.colsum(part, tiles, nv, red1)
        sink.slot("attention_gate.3.weight", (2 * K, K, 1, 1)).copy_(red1[:2 * K * K].view(2 * K, K, 1, 1))
        db1, dg1 = red1[2 * K * K:2 * K * K + K], red1[2 * K * K + K:]
        sink.slot("attention_gate.1.bias", (K,)).copy_(db1)
        sink.slot("attention_gate.1.weight", (K,)).copy_(dg1)
        gz_a = _e((N, H, W, K), torch.float32, dev)
        gz_b = _e((N, H, W, K), torch.float32, dev)
        nw = K * 2 * K * 9
        part = _e(gtiles * nw, torch.float32, dev)
        ops.gate_bwd3(za, zb, K, gabn, a, g1["mean"], g1["invstd"], P["attention_gate.1.weight"], db1, dg1,
                      P["attention_gate.0.weight"].contiguous(), gffd,
                      None if g_aux_a is None else g_aux_a.contiguous().float(),
                      None if g_aux_b is None else g_aux_b.contiguous().float(), gz_a, gz_b, part)
        ops.colsum(part, gtiles, nw, sink.slot("attention_gate.0.weight", (K, 2 * K, 3, 3)).view(-1))
        sink.ready(["attention_gate.4.weight", "attention_gate.4.bias", "attention_gate.3.weight",
                    "attention_gate.1.weight", "attention_gate.1.bias", "attention_gate.0.weight"])
        # ---- the two branch trunks
        self.ea.backward_trunk(S["SA"], gz_a, sink)
        self.eb.backward_trunk(S["SB"], gz_b, sink)
        return sink.finish()


def dual_backward_order(model) -> List[str]:
    """Parameter names in the order DualEngine.backward produces their gradients."""
    names = [n for n, _ in model.named_parameters()]
    head = ["fusion_residual.weight", "fusion_residual.bias", "fusion_head.11.weight", "fusion_head.11.bias",
            "fusion_head.9.weight", "fusion_head.9.bias", "fusion_head.8.weight",
            "fusion_head.5.weight", "fusion_head.5.bias", "fusion_head.4.weight",
            "fusion_head.1.weight", "fusion_head.1.bias", "fusion_head.0.weight",
            "attention_gate.4.weight", "attention_gate.4.bias", "attention_gate.3.weight",
            "attention_gate.1.weight", "attention_gate.1.bias", "attention_gate.0.weight"]
    order = list(head)
    for br in BRANCHES:
        order += [n for n in names if n.startswith(f"{br}.dec1.")]
        for blk in ("dec2", "dec3", "dec4", "enc4", "enc3", "enc2", "enc1"):
            pre = f"{br}.{blk}."
            blk_names = [n for n in names if n.startswith(pre)]
            blk_names.sort(key=lambda n: {"4": 0, "3": 1, "1": 2, "0": 3}[n[len(pre)]])
            order += blk_names
    assert sorted(order) == sorted(names), "backward order must cover every parameter"
    return order


class DualFunction(torch.autograd.Function):
    """autograd boundary of the dual-branch network: outputs (fused, aux unetpp, aux deeplab)."""

    @staticmethod
    def forward(ctx, x, engine, sink_factory, *params):
        out, aux_a, aux_b, S = engine.forward(x, training=True)
        if engine.keep_state:
            engine.last_state = S
        ctx.S, ctx.engine, ctx.sink_factory = S, engine, sink_factory
        ctx.names = [n for n, _ in engine.m.named_parameters()]
        return out, aux_a, aux_b

    @staticmethod
    def backward(ctx, g_out, g_a, g_b):
        sink = ctx.sink_factory() if ctx.sink_factory is not None else None
        if g_out is None:
            N, H, W, K = ctx.S["N"], ctx.S["H"], ctx.S["W"], ctx.engine.K
            g_out = torch.zeros((N, K, H, W), dtype=torch.float32, device=ctx.S["f2"].device)
        grads = ctx.engine.backward(ctx.S, g_out, g_a, g_b, sink)
        ctx.S = None
        return (None, None, None) + tuple(grads.get(n) for n in ctx.names)
