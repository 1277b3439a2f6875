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
                  on the host cores, bounded sample (1 warm-up + 3 timed steps), rank 0 at
                  N=1 only;
  parity       -- after the timed region, untimed: a fresh model of the same configuration
                  is trained for --dice-steps seeded steps on distinct synthetic batches
                  (so it segments the cells instead of sitting in a degenerate state), then
                  on held-out tiles its GPU logits (the bench dtype and fp32) are compared
                  with the fp64 CPU oracle on the same weights (logits_rel_err_vs_cpu), and
                  its GPU masks with the fp32 CPU oracle's masks (dice_vs_cpu_ref).

    python bench.py --dtype fp32 --size 512 --batch 8     # BASELINE configs[1] (fp32 MFMA path)
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
    ap.add_argument("--cpu-size", type=int, default=512,
                    help="CPU baseline sample: 1 warm-up + 3 timed B=1 steps at this size")
    ap.add_argument("--dice-size", type=int, default=1024, help="Dice-vs-CPU-reference image side (0 = skip)")
    ap.add_argument("--dice-steps", type=int, default=200, help="training steps of the parity model")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run the weight gradients on the launch stream (no side-stream overlap; A/B)")
    ap.add_argument("--dual", action="store_true",
                    help="dual-branch model + deep supervision (BASELINE configs[4]: --dual --base 96 --size 2048)")
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle train step on the host CPU (BASELINE.md 'CPU-baseline plan'): B=1 at --cpu-size,
    1 warm-up step + 3 timed steps on distinct seeded tiles (bounded ~10-30 s)."""
    from oracle import eunet_ref as R
    from eunet import synth
    # the box exports OMP_NUM_THREADS = this job's CPU share; os.cpu_count() is the whole host
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    torch.set_num_threads(threads)
    S = R.formula_weights(args.base, 1, 2, dtype=torch.float32)
    tr = R.OracleTrainer(S, total_epochs=50)
    xw, mw = synth.batch(1, args.cpu_size, args.cpu_size, start_index=0)
    tr.step(xw, mw)  # warm-up (allocator / oneDNN init), not timed
    steps = 3
    batches = [synth.batch(1, args.cpu_size, args.cpu_size, start_index=1 + i) for i in range(steps)]
    t0 = time.perf_counter()
    for x, m in batches:
        tr.step(x, m)
    dt = (time.perf_counter() - t0) / steps
    scale = (args.cpu_size / args.size) ** 2  # images of the benchmark size per sample
    model = "?"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "?")
    except OSError:
        pass
    return {"value": round(scale / dt, 5), "unit": "img/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle train steps (PyTorch CPU fp32 restatement of Trainer.train_epoch, fixture-"
                      f"pinned), B=1, {args.cpu_size}x{args.cpu_size} 1-ch base {args.base} K 2: 1 warm-up + "
                      f"3 timed, {dt:.2f} s/step on {torch.get_num_threads()} threads of {os.cpu_count()} "
                      f"({model}); value scaled to {args.size}x{args.size} images by pixel count"}


def train_parity_model(args, dev):
    """A model of the bench configuration trained for args.dice_steps seeded steps on distinct
    synthetic 256^2 batches of 4 (untimed): AdamW at the reference's base LR 4e-3 after a linear
    per-step warmup over the first fifth of the steps (the reference warms up per epoch,
    train_eval.py:122-132), so the parity legs compare a network that segments the cells rather
    than one sitting in a degenerate all-background / all-cell state."""
    from eunet import synth
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    torch.manual_seed(1)
    model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=args.base, dtype=args.dtype).to(dev)
    tr = Trainer(model, dev, "enhanced_unet", total_epochs=50)
    warm = max(1, args.dice_steps // 5)
    for s in range(args.dice_steps):
        for g in tr.optimizer.param_groups:
            g["lr"] = 4e-3 * min(1.0, (s + 1) / warm)
        x, m = synth.batch(4, 256, 256, start_index=10000 + 4 * s, num_classes=2, in_channels=1, device=dev)
        tr.step(x, m, sync_loss=False)
    torch.cuda.synchronize()
    return model


def _cpu_state(model):
    return {k: (v.detach().double().cpu() if v.is_floating_point() else v.cpu()) for k, v in model.state_dict().items()}


def logits_rel_err_vs_cpu(model, args, dev):
    """logits rel-err vs the CPU path.  Held-out 256^2 tile, eval mode, the trained
    parity model's weights: GPU forward_lowres (bench dtype and fp32) vs the fp64 oracle forward
    + the reference's bilinear 2H->H resize.  Per pixel |a-b| / max(|b|, 1e-3 max|b|) and the
    max-normalised max|a-b| / max|b|."""
    from eunet import synth
    from oracle import eunet_ref as R
    x, _ = synth.batch(1, 256, 256, start_index=200000, num_classes=2, in_channels=1)
    S = _cpu_state(model)
    with torch.no_grad():
        ref = torch.nn.functional.interpolate(R.forward(S, x.double(), training=False), size=(256, 256),
                                              mode="bilinear", align_corners=False)
    out = {}
    dtype0 = args.dtype
    model.eval()
    for dt in dict.fromkeys((dtype0, "fp32")):
        model.set_dtype(dt)
        with torch.no_grad():
            lg = model.forward_lowres(x.to(dev)).double().cpu()
        d = (lg - ref).abs()
        out[dt] = {"per_pixel": float((d / ref.abs().clamp_min(1e-3 * float(ref.abs().max()))).max()),
                   "max_normalised": float(d.max() / ref.abs().max())}
    model.set_dtype(dtype0)
    model.train()
    out["sample"] = "held-out 256x256 tile, eval mode, trained parity model; vs fp64 CPU oracle (gate: fp32 <= 1e-3)"
    return out


def dice_vs_cpu_ref(model, args, dev):
    """The metric's "Dice vs CPU ref": the trained parity model predicts a held-out synthetic tile
    on the GPU (eval mode, Evaluator._run_model_single + the reference's probability->mask rules,
    all HIP), in the bench dtype and in fp32; the oracle runs the same weights in fp32 on the CPU
    (reference path: full 2H forward, bilinear resize, softmax, mask rules).  Reported per GPU
    dtype: calculate_semantic_metrics(gpu_mask, cpu_mask) (GPU-counted), pixel agreement,
    max |dprob|, live-class soft Dice; and how well each predicts the synthetic ground truth."""
    from eunet import metrics, ops, synth
    from eunet.evaluator import Evaluator
    from oracle import evalpath_ref as E
    n = args.dice_size
    x, gt = synth.batch(1, n, n, start_index=100000, num_classes=2, in_channels=1)
    S = {k: (v.float() if v.is_floating_point() else v) for k, v in _cpu_state(model).items()}
    t0 = time.perf_counter()
    with torch.no_grad():
        ref_probs = E.run_model_single(S, x[0])
    cpu_mask = E.convert_probs_to_mask(ref_probs.numpy())
    dt_cpu = time.perf_counter() - t0
    ev = Evaluator(model, dev, "enhanced_unet")
    out = {}
    dtype0 = args.dtype
    model.eval()
    for dt in dict.fromkeys((dtype0, "fp32")):
        model.set_dtype(dt)
        with torch.no_grad():
            probs = ev._run_model_single(x[0].to(dev))
            gpu_mask = ops.probs_to_mask(probs)
        m = metrics.calculate_semantic_metrics(gpu_mask, cpu_mask)
        m_gt = metrics.calculate_semantic_metrics(gpu_mask, gt[0])
        pg, pc = probs[1].double().cpu(), ref_probs[1].double()  # live-class probabilities
        out[dt] = {"sem_mean_dice": round(m["sem_mean_dice"], 6), "sem_live_dice": round(m["sem_live_dice"], 6),
                   "sem_background_dice": round(m["sem_background_dice"], 6),
                   "pixel_agreement": round(float((gpu_mask.cpu().numpy() == cpu_mask).mean()), 7),
                   "max_abs_prob_diff": round(float((probs.cpu() - ref_probs).abs().max()), 6),
                   "live_soft_dice": round(float(2 * (pg * pc).sum() / ((pg * pg).sum() + (pc * pc).sum())), 7),
                   "live_pixels_gpu": int((gpu_mask == 1).sum()),
                   "gpu_vs_synthetic_gt_live_dice": round(m_gt["sem_live_dice"], 6)}
    model.set_dtype(dtype0)
    model.train()
    m_ref = metrics.calculate_semantic_metrics(cpu_mask, gt[0])
    out.update({"live_pixels_cpu": int((cpu_mask == 1).sum()),
                "cpu_vs_synthetic_gt_live_dice": round(m_ref["sem_live_dice"], 6),
                "sample": f"1 held-out {n}x{n} synthetic tile; model trained {args.dice_steps} steps (untimed); "
                          f"GPU vs CPU fp32 oracle ({dt_cpu:.1f} s)"})
    return out


PMC_SUMMARY = os.path.join(ROOT, "profiles", "r02_pmc_summary.json")


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


MFMA_SUMMARY = os.path.join(ROOT, "profiles", "r02_pmc_mfma_summary.json")


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


def _config_tag(args):
    if args.dual:
        return "(BASELINE configs[4])"
    if (args.base, args.size, args.batch, args.dtype) == (64, 512, 8, "fp32"):
        return "(BASELINE configs[1])"
    if (args.base, args.size, args.batch, args.dtype) == (64, 1024, 4, "bf16"):
        return "(BASELINE configs[2]; configs[3] at N=8)"
    return "(custom)"


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
    from eunet.engine import UNetEngine
    from eunet.models import EnhancedUNet
    UNetEngine.overlap_wgrad = not args.no_overlap
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
    roof = {"kernel": "conv3x3_fwd_kernel<T, false> (implicit-GEMM MFMA, forward launches)", "bound": "mfma",
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
    if "conv3x3_fwd.encoder" in ks:  # BASELINE north_star's target is stated on the 3x3 encoder convs
        en = ks["conv3x3_fwd.encoder"]
        en_tf = en["flops"] / (en["ms"] * 1e-3) / 1e12
        roof["encoder_fwd"] = {"achieved": round(en_tf, 2), "frac": round(en_tf / peak, 4),
                               "ms_per_step": round(en["ms"] / args.steps, 3),
                               "launches_per_step": en["launches"] // max(1, args.steps),
                               "covers": "forward launches of enc1.3 and enc2-4 .0/.3 (subset of the family "
                                         "above; enc1.0, Cin=1, runs on the HBM-bound conv_small kernel)"}
    # backward MFMA kernels: the weight gradients run on a side stream concurrently with the data
    # gradients (UNetEngine.overlap_wgrad), so these per-launch spans include time shared with the
    # other stream -- lower bounds of each kernel's own rate
    for key, nm in (("conv3x3_dgrad", "dgrad"), ("conv3x3_wgrad", "wgrad")):
        if key in ks and ks[key]["ms"]:
            k = ks[key]
            roof[f"{nm}_tflops_overlapped_spans"] = round(k["flops"] / (k["ms"] * 1e-3) / 1e12, 2)
            roof[f"{nm}_ms_per_step_spans"] = round(k["ms"] / args.steps, 3)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    dice = logits_err = None
    if args.dice_size > 0 and not args.dual:
        pmodel = train_parity_model(args, dev)
        logits_err = logits_rel_err_vs_cpu(pmodel, args, dev)
        dice = dice_vs_cpu_ref(pmodel, args, dev)
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
                               f"{args.batch}/GPU, {args.dtype} " + _config_tag(args),
                   "global_batch": world * args.batch, "image_size": args.size, "parallelism": f"dp{world}"},
        "model_tflops_per_gpu": round(step_flops / (elapsed / args.steps) / 1e12, 2),
        "roofline": roof,
        "cpu_baseline": cpu,
        "logits_rel_err_vs_cpu": logits_err,
        "dice_vs_cpu_ref": dice,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
