"""Throughput of the device data path (eunet.data) against the trainer's consumption.

    python tools/loader_bench.py [--images 48] [--epochs 3] [--workers 4] [--prefetch 2]

Writes a synthetic LabelMe directory (800x600 JPEGs of bright-field-like cells + polygon JSONs,
so max_size=640 gives the reference's 640x480 training tiles, dataset.py:141-157), then measures
  loader   -- CellDataset('train', max_size=640) through eunet.data.DataLoader(batch 2, shuffled,
              every augmentation of dataset.py:204-300 live), images/s with the GPU work included;
  trainer  -- Trainer.step on device-resident 2 x 640x480 batches (base 64, 3-ch -> 3-cls as
              train_model builds it, bf16), images/s;
  epoch    -- Trainer.train_epoch(loader): the two together, images/s (eager steps, and with
              Trainer.step_graph: the step replayed from a captured HIP graph).
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def make_dataset(d, n, h=600, w=800, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    for i in range(n):
        img = np.full((h, w, 3), 170.0) + (20 * np.sin(xx / 97.0 + i) * np.cos(yy / 131.0))[..., None]
        shapes = []
        for c in range(int(rng.integers(25, 60))):
            cy, cx = rng.uniform(20, h - 20), rng.uniform(20, w - 20)
            ry, rx = rng.uniform(6, 18), rng.uniform(6, 18)
            dead = rng.random() < 0.3
            m = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
            img[m] -= 60 if dead else 35
            ang = np.linspace(0, 2 * np.pi, int(rng.integers(10, 24)), endpoint=False)
            pts = [[float(cx + rx * np.cos(a)), float(cy + ry * np.sin(a))] for a in ang]
            shapes.append({"label": "dead" if dead else "live", "points": pts})
        img += rng.normal(0, 6, img.shape)
        Image.fromarray(np.clip(img, 0, 255).astype(np.uint8)).save(os.path.join(d, f"cells{i:03d}.jpg"), quality=92)
        with open(os.path.join(d, f"cells{i:03d}.json"), "w") as f:
            json.dump({"shapes": shapes}, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=48)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--workers", type=int, default=4, help="host decode threads (0: in the loop)")
    ap.add_argument("--prefetch", type=int, default=2, help="batches prepared ahead on a side stream (0: none)")
    ap.add_argument("--host-noise", action="store_true", help="numpy noise (the reference's exact values)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--loader-only", action="store_true", help="only the workers+prefetch loader (for rocprofv3)")
    args = ap.parse_args()
    from eunet.data import CellDataset, DataLoader, collate_fn
    from eunet.models import get_model
    from eunet.train_eval import Trainer
    dev = "cuda"
    tmp = tempfile.mkdtemp(prefix="eunet_loader_")
    t0 = time.perf_counter()
    make_dataset(tmp, args.images)
    t_make = time.perf_counter() - t0
    configs = [("round2_path", dict(host_noise=True, host_ratio=True), 0, 0),
               ("sync_free_in_loop", dict(host_noise=args.host_noise), 0, 0),
               ("sync_free_prefetch", dict(host_noise=args.host_noise), 0, args.prefetch),
               ("sync_free_workers_prefetch", dict(host_noise=args.host_noise), args.workers, args.prefetch),
               ("sync_free_workers_thread", dict(host_noise=args.host_noise), args.workers, -args.prefetch)]
    loaders = {}
    rates = {}
    shape = None
    if args.loader_only:
        configs = configs[-2:-1]
    for label, kw, workers, prefetch in configs:
        ds = CellDataset(tmp, split="train", max_size=640, device=dev, **kw)
        loader = DataLoader(ds, batch_size=2, shuffle=True, collate_fn=collate_fn, workers=workers,
                            prefetch=abs(prefetch), thread=prefetch < 0)
        random.seed(0)
        np.random.seed(0)
        torch.manual_seed(0)
        for b in loader:  # warm-up epoch (allocator, kernels, thread pool)
            shape = tuple(b["images"].shape)
        torch.cuda.synchronize()
        n = 0
        t0 = time.perf_counter()
        for _ in range(args.epochs):
            for b in loader:
                n += b["images"].shape[0]
        torch.cuda.synchronize()
        rates[label] = round(n / (time.perf_counter() - t0), 1)
        print(f"loader {label}: {rates[label]} img/s", file=sys.stderr, flush=True)
        loaders[label] = (ds, loader)
    loader_ips = rates["sync_free_workers_prefetch"]
    if args.loader_only:
        print(json.dumps({"loader_img_s": loader_ips, "epochs": args.epochs + 1, "train_images": len(ds)}), flush=True)
        return

    model = get_model("enhanced_unet", num_classes=3, dtype="bf16").to(dev)
    tr = Trainer(model, dev, "enhanced_unet", total_epochs=50)
    x = torch.rand(2, 3, shape[2], shape[3], device=dev)
    m = torch.randint(0, 3, (2, shape[2], shape[3]), device=dev)
    for _ in range(3):
        tr.step(x, m, sync_loss=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step(x, m, sync_loss=False)
    torch.cuda.synchronize()
    trainer_ips = 2 * args.steps / (time.perf_counter() - t0)

    epoch_rates = {}
    for label in ("sync_free_in_loop", "sync_free_workers_prefetch", "sync_free_workers_prefetch+step_graph",
                  "sync_free_workers_thread", "sync_free_workers_thread+step_graph"):
        ds, loader = loaders[label.split("+")[0]]
        tr.step_graph = label.endswith("+step_graph")
        tr.train_epoch(loader)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for _ in range(args.epochs):
            tr.train_epoch(loader)
            n += len(ds)
        torch.cuda.synchronize()
        epoch_rates[label] = round(n / (time.perf_counter() - t0), 1)
        print(f"train_epoch {label}: {epoch_rates[label]} img/s", file=sys.stderr, flush=True)
    epoch_ips = max(epoch_rates.values())
    # where an epoch's host time goes: the loader's next() (decode hand-off + the next batch's device
    # work enqueued) vs Trainer.step, per batch, eager and graphed
    breakdown = {}
    for lname, graph in (("sync_free_workers_prefetch", False), ("sync_free_workers_prefetch", True),
                         ("sync_free_workers_thread", True)):
        ds, loader = loaders[lname]
        tr.step_graph = graph
        tr.train_epoch(loader)
        torch.cuda.synchronize()
        t_next = t_step = 0.0
        nb = 0
        t0 = time.perf_counter()
        for _ in range(args.epochs):
            it = iter(loader)
            while True:
                ta = time.perf_counter()
                b = next(it, None)
                tb = time.perf_counter()
                t_next += tb - ta
                if b is None:
                    break
                m = tr._masks(b, dev, 0, 0)
                tc = time.perf_counter()
                tr.step(b["images"], m, sync_loss=False)
                t_step += time.perf_counter() - tc
                nb += 1
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        breakdown[lname + ("+step_graph" if graph else "")] = {"ms_per_batch": round(wall / nb * 1e3, 3),
                                                    "next_ms": round(t_next / nb * 1e3, 3),
                                                    "step_ms": round(t_step / nb * 1e3, 3)}
    for _, ld in loaders.values():
        ld.close()
    print(json.dumps({"loader_img_s": loader_ips, "loader_img_s_by_config": rates,
                      "trainer_img_s": round(trainer_ips, 1),
                      "train_epoch_img_s": round(epoch_ips, 1), "train_epoch_img_s_by_loader": epoch_rates,
                      "epoch_host_breakdown": breakdown,
                      "tile": list(shape[2:]), "batch": 2,
                      "train_images": len(ds), "workers": args.workers, "prefetch": args.prefetch,
                      "host_noise": args.host_noise, "dataset_write_s": round(t_make, 1),
                      "host_cpus": os.cpu_count(), "omp_threads": os.environ.get("OMP_NUM_THREADS")}), flush=True)


if __name__ == "__main__":
    main()
