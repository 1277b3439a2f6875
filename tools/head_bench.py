"""The 2H head alone (eunet_head_fwd training + eunet_head_bwd, bf16) on the bench shape
(N 4, 1024^2, K 2), for rocprofv3 per-kernel times of library variants:

    EUNET_LIB=abl/libX.so rocprofv3 --kernel-trace --stats -- python tools/head_bench.py [--reps 10]

Diagnostic only (random weights; the timing does not depend on the values)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--k", type=int, default=2)
    a = ap.parse_args()
    from eunet import ops
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
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(a.reps + 2):
        if i == 2:
            ev[0].record()
        ops.head_fwd(z, N, H, W, K, w1, b1, gamma, beta, w2, b2, True, 1e-5, 0.1, rm, rv, mean, inv, None, logits, ws,
                     dtype=torch.bfloat16)
        ops.head_bwd(z, N, H, W, K, w1, b1, gamma, beta, w2, mean, inv, glog, None, gz, gw1, gb1, gg, gbt, gw2, gb2,
                     ws, dtype=torch.bfloat16)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"head fwd+bwd {ev[0].elapsed_time(ev[1]) / a.reps:.3f} ms  lib={os.environ.get('EUNET_LIB', 'in-tree')}",
          flush=True)


if __name__ == "__main__":
    main()
