"""Benchmark of the MI355X Enhanced-UNet training step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json configs[2], the metric's config): base_ch=64,
1x1024x1024 synthetic bright-field tiles, 1-ch -> 2-class, batch 4 per GPU,
bf16 activations / MFMA (fp32 params, BN stats, loss, AdamW).  A "step" is one
full Trainer step (forward, fused loss, backward, bucketed RCCL all-reduce when
N>1, clip_grad_norm_, AdamW, loss.item()).  Inputs are resident in HBM before
the timed region.  value = images processed by all ranks / max-over-ranks time.

Also reported on the same JSON line:
  roofline     -- the dominant kernel family (conv3x3 implicit-GEMM fwd/dgrad),
                  algorithmic FLOPs / its summed launch time, measured with HIP
                  events on the launch stream over the timed region, vs the
                  gfx950 dense MFMA peak of the dtype;
  cpu_baseline -- the oracle (PyTorch CPU restatement of the reference step)
                  on the host cores, bounded sample, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "enhanced-unet_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training images/sec at 1024×1024 1-ch→2-cls, 1/2/4/8 MI355X; Dice vs CPU ref"
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}  # MI355X_MICROARCH.md dense MFMA peaks
HBM_PEAK_GBS = 8000.0


# The loss stays on the device (Trainer.train_epoch accumulates it there and reads it once per
# epoch), so the host queues step k+1 while step k runs.  EUNET_BENCH_SYNC_LOSS=1 reads
# loss.item() every step as the reference's loop does: ~0.7 ms/step of idle GPU (profiles/r01_ab_sync.txt).
SYNC_LOSS = os.environ.get("EUNET_BENCH_SYNC_LOSS", "0") == "1"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4, help="images per GPU")
    ap.add_argument("--base", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-size", type=int, default=1024, help="CPU baseline sample: one B=1 step at this size")
    ap.add_argument("--dice-size", type=int, default=1024, help="Dice-vs-CPU-reference image side (0 = skip)")
    ap.add_argument("--dual", action="store_true",
                    help="dual-branch model + deep supervision (BASELINE configs[4]: --dual --base 96 --size 2048)")
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle train step on the host CPU: one image, B=1 (bounded ~10-30 s)."""
    from oracle import eunet_ref as R
    from eunet import synth
    # the box exports OMP_NUM_THREADS = this job's CPU share; os.cpu_count() is the whole host
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    torch.set_num_threads(threads)
    S = R.formula_weights(args.base, 1, 2, dtype=torch.float32)
    tr = R.OracleTrainer(S, total_epochs=50)
    xw, mw = synth.batch(1, 64, 64, start_index=0)
    tr.step(xw, mw)  # warm-up (allocator / oneDNN init), not timed
    x, m = synth.batch(1, args.cpu_size, args.cpu_size, start_index=0)
    t0 = time.perf_counter()
    tr.step(x, m)
    dt = time.perf_counter() - t0
    scale = (args.cpu_size / args.size) ** 2  # images of the benchmark size per sample
    model = "?"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "?")
    except OSError:
        pass
    return {"value": round(scale / dt, 5), "unit": "img/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"1 oracle train step (PyTorch CPU fp32 restatement of Trainer.train_epoch), B=1, "
                      f"{args.cpu_size}x{args.cpu_size} 1-ch base {args.base} K 2; {dt:.2f} s on "
                      f"{torch.get_num_threads()} threads of {os.cpu_count()} ({model})"}


def dice_vs_cpu_ref(model, args, dev):
    """The metric's "Dice vs CPU ref": the trained model (its compute dtype) predicts a held-out
    synthetic tile on the GPU (eval mode, Evaluator._run_model_single + the reference's
    probability->mask rules, all HIP); the oracle runs the same weights in fp32 on the CPU
    (reference path: full 2H forward, bilinear resize, softmax, mask rules).  Reported:
    calculate_semantic_metrics(gpu_mask, cpu_mask) (GPU-counted), pixel agreement, max |dprob|."""
    from eunet import metrics, ops, synth
    from eunet.evaluator import Evaluator
    from oracle import evalpath_ref as E
    n = args.dice_size
    x, gt = synth.batch(1, n, n, start_index=100000, num_classes=2, in_channels=1)
    ev = Evaluator(model, dev, "enhanced_unet")
    model.eval()
    with torch.no_grad():
        probs = ev._run_model_single(x[0].to(dev))
        gpu_mask = ops.probs_to_mask(probs)
    model.train()
    S = {k: (v.detach().float().cpu() if v.is_floating_point() else v.cpu()) for k, v in model.state_dict().items()}
    t0 = time.perf_counter()
    with torch.no_grad():
        ref_probs = E.run_model_single(S, x[0])
    cpu_mask = E.convert_probs_to_mask(ref_probs.numpy())
    dt = time.perf_counter() - t0
    m = metrics.calculate_semantic_metrics(gpu_mask, cpu_mask)
    m_gt = metrics.calculate_semantic_metrics(gpu_mask, gt[0])
    agree = float((gpu_mask.cpu().numpy() == cpu_mask).mean())
    pg, pc = probs[1].double().cpu(), ref_probs[1].double()  # live-class probabilities
    soft = float(2 * (pg * pc).sum() / ((pg * pg).sum() + (pc * pc).sum()))
    return {"sem_mean_dice": round(m["sem_mean_dice"], 6), "sem_live_dice": round(m["sem_live_dice"], 6),
            "sem_background_dice": round(m["sem_background_dice"], 6), "pixel_agreement": round(agree, 7),
            "max_abs_prob_diff": round(float((probs.cpu() - ref_probs).abs().max()), 6),
            "live_soft_dice": round(soft, 7),
            "live_pixels_gpu": int((gpu_mask == 1).sum()), "live_pixels_cpu": int((cpu_mask == 1).sum()),
            "gpu_vs_synthetic_gt_live_dice": round(m_gt["sem_live_dice"], 6),
            "sample": f"1 held-out {n}x{n} synthetic tile after the timed steps; GPU {args.dtype} vs CPU fp32 "
                      f"oracle ({dt:.1f} s)"}


PMC_SUMMARY = os.path.join(ROOT, "profiles", "r01_pmc_summary.json")


def pmc_traffic(args, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary
    (tools/gpu_pmc.sh: FETCH_SIZE x2 + WRITE_SIZE, separate passes) of this same
    bench command; None when no summary for this workload exists."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("workload") != [args.base, args.size, args.batch, args.dtype]:
        return None
    k = d["kernels"].get(kernel)
    if not k:
        return None
    return round(k["hbm_bytes_per_launch"]), f"profiles/{os.path.basename(PMC_SUMMARY)} ({d['correction']})"


MFMA_SUMMARY = os.path.join(ROOT, "profiles", "r01_pmc_mfma_summary.json")


def pmc_mfma(kernel):
    """MFMA-pipe busy fraction and effective clock of `kernel` from the committed
    SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass of the default bench command
    (tools/gpu_pmc_mfma.sh); None when absent."""
    try:
        with open(MFMA_SUMMARY) as f:
            k = json.load(f)["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    if not k:
        return None
    return {"mfma_busy_frac": round(k["mfma_busy_frac"], 4), "clock_ghz": round(k["clock_ghz"], 3),
            "source": f"profiles/{os.path.basename(MFMA_SUMMARY)}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # nccl == RCCL over xGMI; EUNET_DIST_BACKEND=gloo only to rehearse N ranks on one GPU
        dist.init_process_group(os.environ.get("EUNET_DIST_BACKEND", "nccl"), init_method="env://")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from eunet import synth, kprof
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer

    torch.manual_seed(0)
    model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=args.base, dtype=args.dtype,
                         dual_branch=args.dual).to(dev)
    tr = Trainer(model, dev, "enhanced_unet", total_epochs=50)
    tr.epoch_lr_step(0)
    if world > 1:
        from eunet.dp import DataParallel
        tr.dp = DataParallel(model)
    x, m = synth.batch(args.batch, args.size, args.size, start_index=rank * args.batch, num_classes=2,
                       in_channels=1, device=dev)
    for _ in range(args.warmup):
        tr.step(x, m)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    with kprof.KernelTimer() as timer:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            tr.step(x, m, sync_loss=SYNC_LOSS)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    ks = timer.summary()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    imgs = world * args.batch * args.steps
    fam = ks.get("conv3x3_fwd", {"ms": 0.0, "flops": 0.0, "launches": 0, "bytes": 0.0})
    achieved = fam["flops"] / (fam["ms"] * 1e-3) / 1e12 if fam["ms"] else None
    peak = PEAK_TFLOPS[args.dtype]
    roof = {"kernel": "conv3x3_fwd_kernel (implicit-GEMM MFMA, fwd + dgrad launches)", "bound": "mfma",
            "achieved": round(achieved, 2) if achieved else None, "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4) if achieved else None, "traffic": None,
            "launches_per_step": fam["launches"] // max(1, args.steps),
            "kernel_ms_per_step": round(fam["ms"] / args.steps, 3),
            "algorithmic_bytes_per_launch": round(fam["bytes"] / max(1, fam["launches"]))}
    pmc = pmc_traffic(args, "conv3x3_fwd_kernel")
    if pmc is not None:
        roof["traffic"], roof["traffic_source"] = pmc
    mf = pmc_mfma("conv3x3_fwd_kernel") if (args.base, args.size, args.batch, args.dtype) == (64, 1024, 4, "bf16") \
        and not args.dual else None
    if mf is not None:
        roof["pmc_mfma"] = mf
    if "conv3x3_wgrad" in ks:
        wg = ks["conv3x3_wgrad"]
        roof["wgrad_tflops"] = round(wg["flops"] / (wg["ms"] * 1e-3) / 1e12, 2)
        roof["wgrad_ms_per_step"] = round(wg["ms"] / args.steps, 3)
    if "conv3x3_fwd.encoder" in ks:  # BASELINE north_star's target is stated on the 3x3 encoder convs
        en = ks["conv3x3_fwd.encoder"]
        en_tf = en["flops"] / (en["ms"] * 1e-3) / 1e12
        roof["encoder_fwd"] = {"achieved": round(en_tf, 2), "frac": round(en_tf / peak, 4),
                               "ms_per_step": round(en["ms"] / args.steps, 3),
                               "launches_per_step": en["launches"] // max(1, args.steps),
                               "covers": "forward launches of enc1.3 and enc2-4 .0/.3 (subset of the family "
                                         "above; enc1.0, Cin=1, runs on the HBM-bound conv_small kernel)"}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    dice = dice_vs_cpu_ref(model, args, dev) if args.dice_size > 0 and not args.dual else None
    from oracle.eunet_ref import flops_per_pixel
    from oracle.dual_ref import dual_flops_per_pixel
    fpp = dual_flops_per_pixel(args.base, 1, 2) if args.dual else flops_per_pixel(args.base, 1, 2)
    step_flops = fpp * args.size * args.size * args.batch
    line = {
        "metric": METRIC,
        "value": round(imgs / elapsed, 3),
        "unit": "img/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic bright-field tiles (eunet.synth, seeded), random-init weights",
        "config": {"workload": (f"dual-branch + deep supervision, " if args.dual else "") +
                               f"base_ch={args.base}, 1x{args.size}x{args.size} 1-ch->2-cls, batch "
                               f"{args.batch}/GPU, {args.dtype} " +
                               ("(BASELINE configs[4])" if args.dual else "(BASELINE configs[2]; configs[3] at N=8)"),
                   "global_batch": world * args.batch, "image_size": args.size, "parallelism": f"dp{world}"},
        "model_tflops_per_gpu": round(step_flops / (elapsed / args.steps) / 1e12, 2),
        "roofline": roof,
        "cpu_baseline": cpu,
        "dice_vs_cpu_ref": dice,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
