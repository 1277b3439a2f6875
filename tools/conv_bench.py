"""Per-layer conv3x3 timing for the cfg3 step shapes (fwd, dgrad, wgrad), HIP events.

    python tools/conv_bench.py [--batch 4] [--size 1024] [--dtype bf16] [--reps 5]
Prints one JSON line per (layer, pass) and a summary; used to steer kernel work.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402

from eunet import ops  # noqa: E402


def layers(b):
    return [("enc1.3", 0, b, b), ("enc2.0", 1, b, 2 * b), ("enc2.3", 1, 2 * b, 2 * b),
            ("enc3.0", 2, 2 * b, 4 * b), ("enc3.3", 2, 4 * b, 4 * b), ("enc4.0", 3, 4 * b, 8 * b),
            ("enc4.3", 3, 8 * b, 8 * b), ("dec4.0", 2, 12 * b, 4 * b), ("dec4.3", 2, 4 * b, 4 * b),
            ("dec3.0", 1, 6 * b, 2 * b), ("dec3.3", 1, 2 * b, 2 * b), ("dec2.0", 0, 3 * b, b),
            ("dec2.3", 0, b, b)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--base", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--transform", action="store_true",
                    help="forward / wgrad with the BN+ReLU operand transform (the bench path materialises it)")
    ap.add_argument("--no-stats", action="store_true", help="forward without BN partials")
    ap.add_argument("--plain-dgrad", action="store_true", help="dgrad without the fused BN-backward reduction")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    dev = "cuda"
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "wred": 0.0}
    flops_tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
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
        sc = torch.ones(cin, device=dev)
        sh = torch.zeros(cin, device=dev)
        wp = ops.conv3x3_pack(w, dt, flip=False)
        wpt = ops.conv3x3_pack(w, dt, flip=True)
        tiles = ops.conv3x3_tiles(ops.act(y))
        st = torch.empty(tiles * (2 * cout + 1), device=dev)
        flops = 2.0 * 9 * cin * cout * a.batch * H * H
        xa, ya, gya, gxa = ops.act(x), ops.act(y), ops.act(gy), ops.act(gx)
        tsc, tsh = (sc, sh) if a.transform else (None, None)
        tst = None if a.no_stats else st
        t_f = timeit(lambda: ops.conv3x3_fwd(xa, wp, ya, bias=bias, scale=tsc, shift=tsh, stats=tst), a.reps)
        # dgrad as the engine runs it: fused with the BN-backward reduction of the layer it feeds
        yb = torch.randn(a.batch, H, H, cin, device=dev).to(dt)
        one, zero = torch.ones(cin, device=dev), torch.zeros(cin, device=dev)
        cpart = torch.empty(ops.conv3x3_tiles(gxa) * 2 * cin, device=dev)
        if a.plain_dgrad:
            t_d = timeit(lambda: ops.conv3x3_dgrad(gya, wpt, gxa), a.reps)
        else:
            t_d = timeit(lambda: ops.conv3x3_dgrad_bnbwd(gya, wpt, gxa, ops.act(yb), zero, one, one, zero, cpart),
                         a.reps)
        ns = ops.conv3x3_wgrad_splits(gya, cin, dt)
        dwp = torch.empty(ns * cout * 9 * cin, device=dev)
        dbp = torch.empty(ns * cout, device=dev)
        dw = torch.empty(cout, cin, 3, 3, device=dev)
        db = torch.empty(cout, device=dev)
        t_w = timeit(lambda: ops.conv3x3_wgrad(xa, gya, dwp, dbp, ns, scale=tsc, shift=tsh), a.reps)
        t_r = timeit(lambda: ops.wgrad_reduce(dwp, dbp, ns, cout, cin, 9, dw, db), a.reps)
        for k, t in (("fwd", t_f), ("dgrad", t_d), ("wgrad", t_w)):
            tot[k] += t
            flops_tot[k] += flops
        tot["wred"] += t_r
        print(json.dumps({"layer": name, "H": H, "cin": cin, "cout": cout, "fwd_ms": round(t_f, 4),
                          "fwd_tf": round(flops / t_f / 1e9, 1), "dgrad_ms": round(t_d, 4),
                          "dgrad_tf": round(flops / t_d / 1e9, 1), "wgrad_ms": round(t_w, 4),
                          "wgrad_tf": round(flops / t_w / 1e9, 1), "wred_ms": round(t_r, 4), "splits": ns}),
              flush=True)
    print(json.dumps({"summary": {k: round(v, 3) for k, v in tot.items()},
                      "tflops": {k: round(flops_tot[k] / tot[k] / 1e9, 1) for k in flops_tot if tot[k]}}))


if __name__ == "__main__":
    main()
