"""Phase shares of head_gh_mfma_kernel blocks from a stamp-instrumented diagnostic build (-DHEAD_STAMP=1,
tools/build_stamp.sh -> abl/libstamp.so): per block, wave 0's s_memtime sums over its tiles of staging
(z / u / g_o with the barriers), the row phase and the tail (g_u, upsample adjoint, patch store), and the
final partial-row reduction.  Shares, not lengths (the stamps' waits forbid some overlap).

    EUNET_LIB=abl/libstamp.so python tools/head_stamps.py
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--k", type=int, default=2)
    a = ap.parse_args()
    from eunet import _lib, ops
    dev, N, H, W, K = "cuda", a.batch, a.size, a.size, a.k
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=1.0: torch.randn(*s, device=dev, generator=g) * sc  # noqa: E731
    z = r(N, H, W, K)
    w1, b1 = r(64, K, 3, 3, sc=0.3), r(64, sc=0.1)
    gamma, beta = 1 + r(64, sc=0.1), r(64, sc=0.1)
    w2, b2 = r(K, 64, sc=0.2), r(K, sc=0.1)
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    mean, inv = torch.empty(64, device=dev), torch.empty(64, device=dev)
    logits = torch.empty(N, K, H, W, device=dev)
    ws = torch.empty(ops.head_workspace_bytes(N, H, W, K, torch.bfloat16), dtype=torch.uint8, device=dev)
    glog = r(N, K, H, W, sc=1e-3)
    gz = torch.empty(N, H, W, K, device=dev)
    gw1, gb1, gg, gbt = (torch.empty_like(t) for t in (w1, b1, gamma, beta))
    gw2, gb2 = torch.empty_like(w2), torch.empty_like(b2)
    lib = _lib.load()
    lib.eunet_head_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    for _ in range(2):
        ops.head_fwd(z, N, H, W, K, w1, b1, gamma, beta, w2, b2, True, 1e-5, 0.1, rm, rv, mean, inv, None, logits, ws,
                     dtype=torch.bfloat16)
        ops.head_bwd(z, N, H, W, K, w1, b1, gamma, beta, w2, mean, inv, glog, None, gz, gw1, gb1, gg, gbt, gw2, gb2,
                     ws, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    buf = np.zeros(1024 * 5, dtype=np.uint64)
    if lib.eunet_head_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes)):
        raise SystemExit("eunet_head_stamps failed: is EUNET_LIB a -DHEAD_STAMP=1 build?")
    st = buf.reshape(1024, 5).astype(np.float64)
    st = st[st[:, 0] > 0]
    tot = st[:, 0].sum()
    print(json.dumps({"kernel": "head_gh_mfma", "blocks": len(st), "cyc_per_block": round(float(st[:, 0].mean())),
                      "staging": round(float(st[:, 1].sum() / tot), 3), "rows": round(float(st[:, 2].sum() / tot), 3),
                      "tail": round(float(st[:, 3].sum() / tot), 3), "final": round(float(st[:, 4].sum() / tot), 3)}))


if __name__ == "__main__":
    main()
