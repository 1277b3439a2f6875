"""Benchmark of the MI355X Enhanced-UNet training step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json configs[2], the metric's config): base_ch=64,
1x1024x1024 synthetic bright-field tiles, 1-ch -> 2-class, batch 4 per GPU,
bf16 activations / MFMA (fp32 params, BN stats, loss, AdamW).  A "step" is one
full Trainer step (forward, fused loss, backward, bucketed RCCL all-reduce when
N>1, clip_grad_norm_, AdamW; the loss stays on the device, as Trainer.train_epoch keeps
it).  Inputs are resident in HBM before the timed region.  value = images processed by all ranks / max-over-ranks time.

Also reported on the same JSON line:
  roofline      -- the dominant kernel family, the conv3x3 implicit-GEMM MFMA kernels (forward,
                   data gradient, weight gradient): algorithmic FLOPs / the wall time any of them
                   ran (union of HIP-event intervals on both streams of the timed region) vs the
                   gfx950 dense MFMA peak of the dtype; per kernel the overlapped-span rate and,
                   from the committed rocprofv3 --pmc pass, the serialised rate, MFMA-busy
                   fraction and HBM traffic; step_frac = whole-step model FLOPs / time / peak;
                   encoder_fwd = the north-star's "3x3 encoder convs" subset;
  dp_world1     -- the same per-rank workload through eunet.dp.DataParallel on RCCL at world
                   size 1 (BASELINE configs[3] per rank): ms/step and overhead vs the plain step;
  fp32_configs1 -- BASELINE configs[1] (base 64, 512^2, batch 8, fp32) timed in this same run;
  dual_configs4 -- BASELINE configs[4] per GPU (dual-branch base 96 + deep supervision, 2048^2,
                   batch 2, bf16) timed in this same run;
  steps_diag    -- per leg: min / median / max GPU time per step of the timed region (an event per
                   step boundary) and, from an extra untimed pass, the whole-step kernel-busy time
                   (union of every library launch's interval on both streams) and the idle rest;
  cpu_baseline  -- the oracle (PyTorch CPU restatement of the reference step) on the host
                   cores, bounded sample (1 warm-up + 3 timed steps), rank 0 at N=1 only;
  parity        -- after the timed region, untimed: a fresh model of the same configuration
                   is trained for --dice-steps seeded steps on distinct synthetic batches
                   (so it segments the cells instead of sitting in a degenerate state), then
                   on held-out tiles its GPU logits (the bench dtype and fp32) are compared
                   with the fp64 CPU oracle on the same weights (logits_rel_err_vs_cpu), and
                   its GPU masks with the fp32 CPU oracle's masks (dice_vs_cpu_ref).

    python bench.py --dtype fp32 --size 512 --batch 8     # BASELINE configs[1] alone
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
    ap.add_argument("--cpu-size", type=int, default=0,
                    help="CPU baseline sample: 1 warm-up + 3 timed B=1 steps at this size (0: the bench size)")
    ap.add_argument("--dice-size", type=int, default=1024, help="Dice-vs-CPU-reference image side (0 = skip)")
    ap.add_argument("--dice-steps", type=int, default=200, help="training steps of the parity model")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run the weight gradients on the launch stream (no side-stream overlap; A/B)")
    ap.add_argument("--no-dp-world1", action="store_true",
                    help="skip the DataParallel-on-RCCL world-1 leg (N=1 only)")
    ap.add_argument("--no-fp32-leg", action="store_true", help="skip the fp32 BASELINE configs[1] leg (N=1 only)")
    ap.add_argument("--no-dual-leg", action="store_true",
                    help="skip the dual-branch BASELINE configs[4] leg (N=1 only)")
    ap.add_argument("--step-graph", type=int, default=0,
                    help="1: Trainer.step_graph (each step's forward + loss + backward replayed from a HIP graph)")
    ap.add_argument("--dual", action="store_true",
                    help="dual-branch model + deep supervision (BASELINE configs[4]: --dual --base 96 --size 2048)")
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle train step on the host CPU (BASELINE.md 'CPU-baseline plan'): B=1 at the bench size
    (--cpu-size overrides), 1 warm-up step + 3 timed steps on distinct seeded tiles (~40 s at 1024^2)."""
    from oracle import eunet_ref as R
    from eunet import synth
    # the box exports OMP_NUM_THREADS = this job's CPU share; os.cpu_count() is the whole host
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    if not args.cpu_size:
        args.cpu_size = args.size
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
                      f"({model})" + ("" if args.cpu_size == args.size else
                                    f"; value scaled to {args.size}x{args.size} images by pixel count")}


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


# rocprofv3 --pmc summaries of the default bench command (tools/gpu_pmc.sh, tools/gpu_pmc_mfma.sh);
# the newest round's file that exists is used
def _profile(name):
    for r in ("r06", "r05", "r04", "r03", "r02"):
        f = os.path.join(ROOT, "profiles", f"{r}_{name}")
        if os.path.exists(f):
            return f
    return None


def _load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError, TypeError):
        return None


def pmc_traffic(args, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary (FETCH_SIZE x2 +
    WRITE_SIZE, separate passes) of this same bench command; None for another workload."""
    path = _profile("pmc_summary.json")
    d = _load_json(path)
    if not d or d.get("workload") != [args.base, args.size, args.batch, args.dtype]:
        return None
    k = d["kernels"].get(kernel)
    if not k:
        return None
    return k["hbm_bytes_per_launch"], f"profiles/{os.path.basename(path)} ({d['correction']})"


def pmc_mfma(args, kernel):
    """MFMA-pipe busy fraction, effective clock and serialised launch time of `kernel` from the
    committed SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass of the default bench command (the
    counter pass serialises the streams); None for another workload."""
    path = _profile("pmc_mfma_summary.json")
    d = _load_json(path)
    if not d or d.get("workload", [64, 1024, 4, "bf16"]) != [args.base, args.size, args.batch, args.dtype] \
            or args.dual:
        return None
    k = d["kernels"].get(kernel)
    if not k:
        return None
    return dict(k, source=f"profiles/{os.path.basename(path)}")


def _config_tag(args):
    if args.dual:
        return "(BASELINE configs[4])"
    if (args.base, args.size, args.batch, args.dtype) == (64, 512, 8, "fp32"):
        return "(BASELINE configs[1])"
    if (args.base, args.size, args.batch, args.dtype) == (64, 1024, 4, "bf16"):
        return "(BASELINE configs[2]; configs[3] at N=8)"
    return "(custom)"


def build_trainer(args, dev, dtype=None, base=None, dual=None):
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    torch.manual_seed(0)
    model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=base or args.base, dtype=dtype or args.dtype,
                         dual_branch=args.dual if dual is None else dual).to(dev)
    tr = Trainer(model, dev, "enhanced_unet", total_epochs=50)
    tr.epoch_lr_step(0)
    tr.step_graph = bool(args.step_graph)
    return tr


def timed_steps(tr, x, m, steps, warmup, world, dev):
    """W untimed warmup steps, then exactly K steps bracketed by barrier + synchronize; returns the
    max-over-ranks elapsed seconds and the kernel timer of the timed region."""
    from eunet import kprof
    graph = getattr(tr, "step_graph", False)
    for _ in range(max(warmup, tr.graph_warmup + 2) if graph else warmup):
        # (graph steps: deferred-loss warm-up steps, so the graph is captured before the timed region)
        tr.step(x, m, sync_loss=not graph)
    torch.cuda.synchronize()
    dp = getattr(tr, "dp", None)
    if dp is not None:
        dp.start_timing()
    if world > 1:
        dist.barrier()
    # one event per step boundary on the launch stream (K+1 markers, no per-kernel cost): the
    # per-step GPU spans expose a one-off stall that the mean alone would hide
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    ms0 = torch.cuda.memory_stats(dev)
    with kprof.KernelTimer() as timer:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        marks[0].record()
        host = [time.perf_counter()]
        for i in range(steps):
            tr.step(x, m, sync_loss=SYNC_LOSS)
            marks[i + 1].record()
            host.append(time.perf_counter())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    timer.dp = dp.stop_timing() if dp is not None else None
    timer.local_s = t1 - t0
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    timer.step_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(steps)]
    timer.host_ms = [1e3 * (host[i + 1] - host[i]) for i in range(steps)]
    ms1 = torch.cuda.memory_stats(dev)
    # device allocations / frees / OOM retries of the caching allocator inside the timed region (each
    # hipMalloc / hipFree can block the host; a retry frees the whole cache after a device sync)
    timer.alloc = {k: ms1.get(k, 0) - ms0.get(k, 0) for k in ("num_device_alloc", "num_device_free", "num_alloc_retries")}
    timer.alloc["reserved_gb"] = round(ms1.get("reserved_bytes.all.current", 0) / 2 ** 30, 2)
    return float(elapsed.item()), timer


def step_spread(timer):
    """min / median / max of the per-step GPU spans of the timed region (ms), the step index of the max
    and the host time of that step's issue (Trainer.step call to return: a host-side stall shows there,
    a GPU-side one only in the span)."""
    s = sorted(timer.step_ms)
    if not s:
        return None
    i = max(range(len(s)), key=lambda j: timer.step_ms[j])
    return {"min": round(s[0], 3), "median": round(s[len(s) // 2], 3), "max": round(s[-1], 3), "max_at": i,
            "host_ms_at_max": round(timer.host_ms[i], 3), "host_ms_max": round(max(timer.host_ms), 3),
            "allocator": timer.alloc}


def busy_pass(tr, x, m, steps=3):
    """Whole-step kernel-busy figure from an extra, untimed pass of `steps` steps after the timed region:
    every launching C-ABI call bracketed by events (kprof.BusyTimer), busy = the union of those intervals
    over both streams.  idle = instrumented span - busy: host gaps, synchronising calls and PyTorch's own
    kernels; the events themselves add a little to both."""
    from eunet import kprof
    tr.step(x, m, sync_loss=False)
    torch.cuda.synchronize()
    with kprof.BusyTimer() as bt:
        for _ in range(steps):
            tr.step(x, m, sync_loss=False)
    busy, span = bt.busy_ms() / steps, bt.span_ms() / steps
    return {"step_kernel_busy_ms": round(busy, 3), "instrumented_ms_per_step": round(span, 3),
            "idle_ms_per_step": round(span - busy, 3), "launches_per_step": len(bt.iv) // steps}


def step_record(timer, tr, x, m):
    """The per-leg step diagnostics: per-step spread of the timed region + the busy pass."""
    return {"step_ms": step_spread(timer), **busy_pass(tr, x, m)}


CONV_FAMILIES = (("conv3x3_fwd", "fwd", "conv3x3_fwd_kernel"),
                 ("conv3x3_dgrad", "dgrad", "conv3x3_fwd_kernel.dgrad"),
                 ("conv3x3_wgrad", "wgrad", "conv3x3_wgrad_bf16_kernel"))


def conv_roofline(args, timer, steps, step_flops, elapsed, dtype):
    """roofline of the dominant kernel family, the conv3x3 implicit-GEMM MFMA kernels (forward, data
    gradient, weight gradient: ~99 % of the step's FLOPs).  achieved = the family's algorithmic FLOPs
    / the wall time during which any of its launches ran (union of the HIP-event intervals on both
    streams: the weight gradients run on a side stream concurrently with the data gradients, so the
    summed spans would count shared time twice).  components: each kernel's own rate over its summed
    spans as it runs in the step (overlapped), and -- from the committed PMC pass, where the counter
    collection serialises the streams -- its standalone launch time and MFMA-busy fraction."""
    ks = timer.summary()
    peak = PEAK_TFLOPS[dtype]
    fams = [f for f, _, _ in CONV_FAMILIES if f in ks]
    flops = sum(ks[f]["flops"] for f in fams)
    launches = sum(ks[f]["launches"] for f in fams)
    union = timer.union_ms(fams)
    achieved = flops / (union * 1e-3) / 1e12 if union else None
    roof = {"kernel": "conv3x3 implicit-GEMM MFMA family: conv3x3_fwd_kernel (forward + data-gradient launches) "
                      "+ conv3x3_wgrad kernel", "bound": "mfma",
            "achieved": round(achieved, 2) if achieved else None, "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4) if achieved else None, "traffic": None,
            "launches_per_step": launches // max(1, steps),
            "family_wall_ms_per_step": round(union / steps, 3),
            "family_flops_per_step": flops / steps,
            "algorithmic_bytes_per_launch": round(sum(ks[f]["bytes"] for f in fams) / max(1, launches)),
            "step_frac": round(step_flops / (elapsed / steps) / 1e12 / peak, 4),
            "components": {}}
    traffic, src, have_all = 0.0, None, True
    for fam, nm, kname in CONV_FAMILIES:
        if fam not in ks:
            continue
        k = ks[fam]
        per = k["flops"] / max(1, k["launches"])
        comp = {"launches_per_step": k["launches"] // max(1, steps), "ms_per_step_spans": round(k["ms"] / steps, 3),
                "frac_overlapped_spans": round(k["flops"] / (k["ms"] * 1e-3) / 1e12 / peak, 4)}
        mf = pmc_mfma(args, kname) if dtype == args.dtype else None
        if mf is not None:
            comp["serialised_us_per_launch"] = round(mf["us_per_launch"], 1)
            comp["frac_serialised"] = round(per / (mf["us_per_launch"] * 1e-6) / 1e12 / peak, 4)
            comp["mfma_busy_frac"] = round(mf["mfma_busy_frac"], 4)
            comp["clock_ghz"] = round(mf["clock_ghz"], 3)
            comp["pmc_source"] = mf["source"]
        pm = pmc_traffic(args, kname) if dtype == args.dtype else None
        if pm is not None:
            comp["traffic_per_launch"] = round(pm[0])
            traffic += pm[0] * k["launches"]
            src = pm[1]
        else:
            have_all = False
        roof["components"][nm] = comp
    if have_all and src:
        roof["traffic"] = round(traffic / max(1, launches))
        roof["traffic_source"] = src
    if "conv3x3_fwd.encoder" in ks:  # BASELINE north_star's target is stated on the 3x3 encoder convs
        en = ks["conv3x3_fwd.encoder"]
        en_tf = en["flops"] / (en["ms"] * 1e-3) / 1e12
        roof["encoder_fwd"] = {"achieved": round(en_tf, 2), "frac": round(en_tf / peak, 4),
                               "ms_per_step": round(en["ms"] / steps, 3),
                               "launches_per_step": en["launches"] // max(1, steps),
                               "covers": "forward launches of enc1.3 and enc2-4 .0/.3 (enc1.0, Cin=1, runs on the "
                                         "HBM-bound conv_small kernel)"}
    if "conv3x3.encoder_train" in ks:  # the same convs' forward + data + weight gradients, over their union wall
        et = ks["conv3x3.encoder_train"]
        wall = timer.union_ms(["conv3x3.encoder_train"])
        et_tf = et["flops"] / (wall * 1e-3) / 1e12 if wall else None
        roof["encoder_train"] = {"achieved": round(et_tf, 2) if et_tf else None,
                                 "frac": round(et_tf / peak, 4) if et_tf else None,
                                 "wall_ms_per_step": round(wall / steps, 3),
                                 "spans_ms_per_step": round(et["ms"] / steps, 3),
                                 "launches_per_step": et["launches"] // max(1, steps),
                                 "covers": "every conv3x3 MFMA launch of the encoder blocks (enc1.3, enc2-4 .0/.3): "
                                           "forward, data gradient and weight gradient (side stream included); "
                                           "FLOPs over the union of their HIP-event intervals"}
    return roof


def step_flops_of(args, base, size, batch, dual=None):
    from oracle.eunet_ref import flops_per_pixel
    from oracle.dual_ref import dual_flops_per_pixel
    dual = args.dual if dual is None else dual
    fpp = dual_flops_per_pixel(base, 1, 2) if dual else flops_per_pixel(base, 1, 2)
    return fpp * size * size * batch


def dp_world1_leg(args, tr, x, m, dev, ms_plain):
    """The configs[3] per-rank workload through the data-parallel path on RCCL at world size 1:
    DataParallel (flat gradient buffer in backward order, bucketed async all-reduces issued from the
    backward, flat BN-buffer broadcast) on the nccl backend, same trainer and inputs; prices the
    bucketing and RCCL launches against the plain step."""
    import socket
    from eunet.dp import DataParallel
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        tr.dp = DataParallel(tr.model)
        el, t = timed_steps(tr, x, m, args.steps, args.warmup, 1, dev)
        nb = len(tr.dp.buckets)
        tr.dp = None
    finally:
        dist.destroy_process_group()
    ms = 1e3 * el / args.steps
    return {"dp_world1_ms_per_step": round(ms, 3), "overhead_pct": round(100.0 * (ms - ms_plain) / ms_plain, 2),
            "buckets": nb, "backend": "nccl (RCCL)", "step_ms": step_spread(t),
            "note": "same per-rank workload through eunet.dp.DataParallel at world size 1 (bucketed all-reduce "
                    "from inside the HIP backward, BN-buffer broadcast); BASELINE configs[3] per rank"}


def fp32_configs1_leg(args, dev):
    """BASELINE configs[1] (base 64, 1x512^2, batch 8, fp32: the 1e-3 parity path) timed in the same
    invocation: value, ms/step and its conv roofline against the fp32 MFMA peak."""
    from eunet import synth
    size, batch = 512, 8
    tr = build_trainer(args, dev, dtype="fp32", base=64)
    x, m = synth.batch(batch, size, size, start_index=0, num_classes=2, in_channels=1, device=dev)
    el, timer = timed_steps(tr, x, m, args.steps, args.warmup, 1, dev)
    diag = step_record(timer, tr, x, m)
    sf = step_flops_of(args, 64, size, batch)
    a32 = argparse.Namespace(**vars(args))
    a32.size, a32.batch, a32.dtype, a32.base = size, batch, "fp32", 64
    roof = conv_roofline(a32, timer, args.steps, sf, el, "fp32")
    out = {"value": round(batch * args.steps / el, 3), "unit": "img/s", "ms_per_step": round(1e3 * el / args.steps, 3),
           "workload": "base_ch=64, 1x512x512 1-ch->2-cls, batch 8, fp32 (BASELINE configs[1])",
           "model_tflops": round(sf / (el / args.steps) / 1e12, 2), "roofline": roof, "steps_diag": diag}
    del tr
    torch.cuda.empty_cache()
    return out


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start N ranks under torch.distributed.run (one process per
    GPU, rendezvous on 127.0.0.1) as a child process and return its exit code.  Runs before anything has
    touched the GPU (torch.cuda.device_count() does not initialise it on this image)."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def dual_configs4_leg(args, dev):
    """BASELINE configs[4] per GPU (dual-branch base 96 + deep supervision, 1x2048^2, batch 2, bf16;
    models.py:253-333, train_eval.py:199-234) timed in the same invocation: value, ms/step, the conv
    roofline against the bf16 MFMA peak and the step diagnostics."""
    from eunet import synth
    size, batch, base = 2048, 2, 96
    tr = build_trainer(args, dev, dtype="bf16", base=base, dual=True)
    x, m = synth.batch(batch, size, size, start_index=0, num_classes=2, in_channels=1, device=dev)
    el, timer = timed_steps(tr, x, m, args.steps, args.warmup, 1, dev)
    diag = step_record(timer, tr, x, m)
    sf = step_flops_of(args, base, size, batch, dual=True)
    a4 = argparse.Namespace(**vars(args))
    a4.size, a4.batch, a4.dtype, a4.base, a4.dual = size, batch, "bf16", base, True
    roof = conv_roofline(a4, timer, args.steps, sf, el, "bf16")
    roof.pop("encoder_fwd", None)
    roof.pop("encoder_train", None)
    out = {"value": round(batch * args.steps / el, 3), "unit": "img/s", "ms_per_step": round(1e3 * el / args.steps, 3),
           "workload": "dual-branch + deep supervision, base_ch=96, 1x2048x2048 1-ch->2-cls, batch 2/GPU, bf16 "
                       "(BASELINE configs[4] per GPU)",
           "model_tflops": round(sf / (el / args.steps) / 1e12, 2), "roofline": roof, "steps_diag": diag}
    del tr, x, m
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # nccl == RCCL over xGMI; EUNET_DIST_BACKEND=gloo only to rehearse N ranks on one GPU
    backend = os.environ.get("EUNET_DIST_BACKEND", "nccl")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    ngpu = torch.cuda.device_count()
    if ngpu < world and backend != "gloo":
        sys.exit(f"bench.py: {world} ranks need {world} GPUs, {ngpu} visible")
    # one process per GPU: bind the device before the process group, so RCCL's communicator is created on it
    local = local % max(1, ngpu)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group(backend, init_method="env://", device_id=dev)
        else:
            dist.init_process_group(backend, init_method="env://")
        if dist.get_world_size() != args.gpus:
            sys.exit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    from eunet import synth
    from eunet.engine import UNetEngine
    UNetEngine.overlap_wgrad = not args.no_overlap

    tr = build_trainer(args, dev)
    if world > 1:
        from eunet.dp import DataParallel
        tr.dp = DataParallel(tr.model)
    x, m = synth.batch(args.batch, args.size, args.size, start_index=rank * args.batch, num_classes=2,
                       in_channels=1, device=dev)
    elapsed, timer = timed_steps(tr, x, m, args.steps, args.warmup, world, dev)
    per_rank = None
    if world > 1:  # every rank's own step time and exposed communication (train_eval.py:337-343 per rank)
        mine = {"rank": rank, "ms_per_step": round(1e3 * timer.local_s / args.steps, 3), **(timer.dp or {})}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    diag = step_record(timer, tr, x, m)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    imgs = world * args.batch * args.steps
    step_flops = step_flops_of(args, args.base, args.size, args.batch)
    roof = conv_roofline(args, timer, args.steps, step_flops, elapsed, args.dtype)
    ms_plain = 1e3 * elapsed / args.steps
    dpw1 = None
    if world == 1 and not args.no_dp_world1 and not args.dual:
        dpw1 = dp_world1_leg(args, tr, x, m, dev, ms_plain)
    del tr
    torch.cuda.empty_cache()
    fp32 = None
    if world == 1 and not args.no_fp32_leg and not args.dual and \
            (args.base, args.size, args.batch, args.dtype) == (64, 1024, 4, "bf16"):
        fp32 = fp32_configs1_leg(args, dev)
    dual4 = None
    if world == 1 and not args.no_dual_leg and not args.dual and \
            (args.base, args.size, args.batch, args.dtype) == (64, 1024, 4, "bf16"):
        dual4 = dual_configs4_leg(args, dev)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    dice = logits_err = None
    if args.dice_size > 0 and not args.dual:
        pmodel = train_parity_model(args, dev)
        logits_err = logits_rel_err_vs_cpu(pmodel, args, dev)
        dice = dice_vs_cpu_ref(pmodel, args, dev)
    line = {
        "metric": METRIC,
        "value": round(imgs / elapsed, 3),
        "unit": "img/s",
        "n_gpus": world,
        "world": {"size": dist.get_world_size() if world > 1 else 1,
                  "backend": backend + (" (RCCL)" if backend == "nccl" else "") if world > 1 else None,
                  "per_rank": per_rank},
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_plain, 3),
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
        "steps_diag": diag,
        "dp_world1": dpw1,
        "fp32_configs1": fp32,
        "dual_configs4": dual4,
        "cpu_baseline": cpu,
        "logits_rel_err_vs_cpu": logits_err,
        "dice_vs_cpu_ref": dice,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
