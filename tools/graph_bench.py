"""Trainer.step eager vs StepGraph replay: images/s and the host issue time per eager step.

    python tools/graph_bench.py [--steps 30]

Two workloads: the reference's training tile (3-ch 640x480, batch 2, base 64, 3 classes, bf16)
and the bench's (1-ch 1024^2, batch 4, 2 classes).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402


def run(graph, B, H, W, steps, cin, K):
    from eunet.models import get_model
    from eunet.train_eval import Trainer
    torch.manual_seed(0)
    model = get_model("enhanced_unet", num_classes=K, in_channels=cin, dtype="bf16").to("cuda")
    tr = Trainer(model, "cuda", "enhanced_unet", total_epochs=50)
    tr.step_graph = graph
    x = torch.rand(B, cin, H, W, device="cuda")
    m = torch.randint(0, K, (B, H, W), device="cuda")
    for _ in range(4):
        tr.step(x, m, sync_loss=False)
    torch.cuda.synchronize()
    host = []
    for _ in range(5):  # issue time of one step with an idle device
        t0 = time.perf_counter()
        tr.step(x, m, sync_loss=False)
        host.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(x, m, sync_loss=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"ms_per_step": round(dt * 1e3, 3), "img_s": round(B / dt, 1),
            "host_issue_ms": round(sorted(host)[2] * 1e3, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    out = {}
    for name, (B, H, W, cin, K) in (("tile_640x480_b2", (2, 480, 640, 3, 3)), ("bench_1024_b4", (4, 1024, 1024, 1, 2))):
        for graph in (False, True):
            out[f"{name}_{'graph' if graph else 'eager'}"] = run(graph, B, H, W, a.steps, cin, K)
            print(name, graph, out[f"{name}_{'graph' if graph else 'eager'}"], flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
