"""Phase shares of conv3x3_fwd_kernel blocks from a stamp-instrumented diagnostic build (-DCONV_STAMP=1,
tools/build_stamp.sh -> abl/libstamp.so): wave 0 of each block records s_memtime around its staging
(+ barriers), MFMA chunks (issue) and epilogue.  Read the SHARES, not the lengths: the stamps' waits
forbid some overlap the product kernel has.  The epilogue is split into its pre-pass (bias, BN
statistics), the two LDS-staged store passes (staging + barrier, stores + fused reduction) and the
final cross-wave reduction.

    EUNET_LIB=abl/libstamp.so python tools/conv_stamps.py [--only enc1.3]

Per layer and pass (fwd with the BN+ReLU operand transform as the bench runs the .3 convs, plain
forward for .0, dgrad with the fused BN-backward reduction): mean cycles per block and the shares of
staging / MFMA / epilogue, blocks per CU in flight (sum of block lifetimes / launch span / 256 CUs).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd"), os.path.dirname(os.path.abspath(__file__))]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from conv_bench import layers  # noqa: E402
from eunet import _lib, ops  # noqa: E402


NST = 11  # conv3x3.hip STAMP_N
EPI = ("pre", "p0_stage", "p0_store", "p1_stage", "p1_store", "reduce")


def read_stamps(nblocks):
    buf = np.zeros(nblocks * NST, dtype=np.uint64)
    lib = _lib.load()
    rc = lib.eunet_conv_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes))
    if rc:
        raise SystemExit(f"eunet_conv_stamps rc={rc}: is EUNET_LIB a -DCONV_STAMP=1 build?")
    st = buf.reshape(nblocks, NST).astype(np.float64)
    return st[st[:, 1] > 0]  # blocks that wrote their row


def report(name, kind, nblocks, fn):
    fn()
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    st = read_stamps(nblocks)
    t0, tot, stage, mfma, epi = st[:, :5].T
    span = (t0 + tot).max() - t0.min()
    row = {"layer": name, "pass": kind, "blocks": int(len(st)), "cyc_per_block": round(float(tot.mean())),
           "stage": round(float(stage.sum() / tot.sum()), 3), "mfma": round(float(mfma.sum() / tot.sum()), 3),
           "epilogue": round(float(epi.sum() / tot.sum()), 3),
           "blocks_in_flight_per_cu": round(float(tot.sum() / span / 256), 2)}
    for i, k in enumerate(EPI):  # the epilogue's parts, as shares of the whole block
        row["epi_" + k] = round(float(st[:, 5 + i].sum() / tot.sum()), 3)
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--base", type=int, default=64)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    lib = _lib.load()
    lib.eunet_conv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    dt, dev = torch.bfloat16, "cuda"
    for name, lvl, cin, cout in layers(a.base):
        if a.only and a.only not in name:
            continue
        H = a.size >> lvl
        x = torch.randn(a.batch, H, H, cin, device=dev).to(dt)
        y = torch.empty(a.batch, H, H, cout, device=dev, dtype=dt)
        gy = torch.randn(a.batch, H, H, cout, device=dev).to(dt)
        gx = torch.empty(a.batch, H, H, cin, device=dev, dtype=dt)
        w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
        bias = torch.zeros(cout, device=dev)
        sc, sh = torch.ones(cin, device=dev), torch.zeros(cin, device=dev)
        wp = ops.conv3x3_pack(w, dt, flip=False)
        wpt = ops.conv3x3_pack(w, dt, flip=True)
        tiles = ops.conv3x3_tiles(ops.act(y))
        st = torch.empty(tiles * (2 * cout + 1), device=dev)
        xa, ya, gya, gxa = ops.act(x), ops.act(y), ops.act(gy), ops.act(gx)
        tr = name.endswith(".3")  # the .3 convs stage their input through BN+ReLU
        nb_f = tiles * ((cout + 63) // 64)
        report(name, "fwd", nb_f, lambda: ops.conv3x3_fwd(xa, wp, ya, bias=bias, scale=sc if tr else None,
                                                           shift=sh if tr else None, stats=st))
        yb = torch.randn(a.batch, H, H, cin, device=dev).to(dt)
        one, zero = torch.ones(cin, device=dev), torch.zeros(cin, device=dev)
        gtiles = ops.conv3x3_tiles(gxa)
        cpart = torch.empty(gtiles * 2 * cin, device=dev)
        nb_d = gtiles * ((cin + 63) // 64)
        report(name, "dgrad", nb_d,
               lambda: ops.conv3x3_dgrad_bnbwd(gya, wpt, gxa, ops.act(yb), zero, one, one, zero, cpart))


if __name__ == "__main__":
    main()
