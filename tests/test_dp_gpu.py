"""Data-parallel path with the HIP engine: world size 2 on one GPU (gloo carries the
collectives; on a multi-GPU node bench.py uses nccl = RCCL with one GPU per rank).

Each rank trains its own shard through DataParallel (bucketed all-reduce launched
from inside the HIP backward) and, separately, computes its local gradients
without DP; the DP gradients must equal the mean of the ranks' local gradients and
be identical on both ranks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "enhanced-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import eunet_ref as R
        from eunet import synth
        from eunet.dp import DataParallel
        from eunet.losses import combined_loss
        from eunet.models import EnhancedUNet
        sd = {k: v.float() if v.is_floating_point() else v for k, v in R.formula_weights(16, 1, 2).items()}
        x, m = synth.batch(2, 64, 64, start_index=100 + 2 * rank, num_classes=2, in_channels=1, device="cuda")

        def fresh():
            mod = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
            mod.load_state_dict(sd)
            return mod.cuda().train()

        ref = fresh()
        combined_loss(ref.forward_lowres(x), m).backward()
        local = torch.cat([p.grad.reshape(-1) for _, p in ref.named_parameters()]).cpu()
        model = fresh()
        dp = DataParallel(model, bucket_mb=0.05)
        dp.before_forward()
        combined_loss(model.forward_lowres(x), m).backward()
        torch.cuda.synchronize()
        got = torch.cat([p.grad.reshape(-1) for _, p in model.named_parameters()]).cpu()
        locs = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(locs, local)
        gots = [torch.zeros_like(got) for _ in range(world)]
        dist.all_gather(gots, got)
        want = sum(locs) / world
        err = float((got - want).abs().max() / want.abs().max())
        same = all(torch.equal(g, gots[0]) for g in gots)
        q.put((rank, err, same, len(dp.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp_world2_on_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=500) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, same, nb in res:
        assert nb > 3
        assert same, "ranks must hold identical averaged gradients"
        assert err < 1e-6, err


def _nccl_worker(port, q):
    """world size 1 on the RCCL backend: the communicator is created, every gradient bucket is
    all-reduced through RCCL from inside the HIP backward (BucketSink), BN buffers are broadcast
    as one flat tensor; with one rank the averaged gradients must equal the plain run's bit for
    bit, and the replicated training step must match as well."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "enhanced-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from oracle import eunet_ref as R
        from eunet import synth
        from eunet.dp import DataParallel
        from eunet.losses import combined_loss
        from eunet.models import EnhancedUNet
        from eunet.train_eval import Trainer
        sd = {k: v.float() if v.is_floating_point() else v for k, v in R.formula_weights(16, 1, 2).items()}
        x, m = synth.batch(2, 64, 64, start_index=200, num_classes=2, in_channels=1, device="cuda")

        def fresh():
            mod = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16, dtype="bf16")
            mod.load_state_dict(sd)
            return mod.cuda().train()

        ref = fresh()
        combined_loss(ref.forward_lowres(x), m).backward()
        model = fresh()
        dp = DataParallel(model, bucket_mb=0.05)
        buffers_are_views = all(b.untyped_storage().data_ptr() == dp.flat_buffers.untyped_storage().data_ptr()
                                for n, b in model.named_buffers() if b.dtype.is_floating_point)
        dp.before_forward()
        combined_loss(model.forward_lowres(x), m).backward()
        torch.cuda.synchronize()
        grads_equal = all(torch.equal(p.grad, q.grad) for p, q in zip(model.parameters(), ref.parameters()))
        # three Trainer steps with DP vs without: identical parameters and BN buffers
        ta, tb = Trainer(fresh(), "cuda", "enhanced_unet"), Trainer(fresh(), "cuda", "enhanced_unet")
        ta.dp = DataParallel(ta.model, bucket_mb=0.05)
        la = [ta.step(x, m) for _ in range(3)]
        lb = [tb.step(x, m) for _ in range(3)]
        same_step = la == lb and all(torch.equal(p, q) for p, q in zip(ta.model.state_dict().values(),
                                                                         tb.model.state_dict().values()))
        q.put(dict(backend=dist.get_backend(), rccl=str(torch.cuda.nccl.version()), buckets=len(dp.buckets),
                   views=buffers_are_views, grads_equal=grads_equal, same_step=same_step))
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put(dict(error=repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp_nccl_world1_rccl_buckets():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=500)
    p.join(timeout=120)
    print("RCCL world-1 DP:", res)
    assert "error" not in res, res
    assert p.exitcode == 0
    assert res["backend"] == "nccl" and res["buckets"] > 3
    assert res["views"], "BN buffers must be views of the flat broadcast buffer"
    assert res["grads_equal"], "RCCL-averaged gradients (world 1) must equal the plain backward"
    assert res["same_step"], "Trainer steps with DataParallel(world 1) must equal the plain steps"


def _nccl_cfg3_worker(port, q):
    """BASELINE configs[3]'s per-rank workload (base 64, 1x1024^2, batch 4, bf16) through the RCCL
    data-parallel path at world size 1: default 8 MiB buckets, weight gradients on the side stream
    (the bench schedule), bucket all-reduces issued from the side stream inside the backward.  The
    gradients and two Trainer steps must equal the plain (non-DP) run bit for bit."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "enhanced-unet_amd")]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        from eunet import synth
        from eunet.dp import DataParallel
        from eunet.engine import UNetEngine
        from eunet.losses import combined_loss
        from eunet.models import EnhancedUNet
        from eunet.train_eval import Trainer
        assert UNetEngine.overlap_wgrad, "the bench schedule runs the weight gradients on the side stream"
        x, m = synth.batch(4, 1024, 1024, start_index=0, num_classes=2, in_channels=1, device="cuda")

        def fresh():
            torch.manual_seed(0)
            return EnhancedUNet(num_classes=2, in_channels=1, base_ch=64, dtype="bf16").cuda().train()

        ref = fresh()
        combined_loss(ref.forward_lowres(x), m).backward()
        model = fresh()
        dp = DataParallel(model)  # default 8 MiB buckets
        dp.before_forward()
        combined_loss(model.forward_lowres(x), m).backward()
        torch.cuda.synchronize()
        grads_equal = all(torch.equal(p.grad, r.grad) for p, r in zip(model.parameters(), ref.parameters()))
        ta, tb = Trainer(fresh(), "cuda", "enhanced_unet"), Trainer(fresh(), "cuda", "enhanced_unet")
        ta.dp = DataParallel(ta.model)
        la = [ta.step(x, m) for _ in range(2)]
        lb = [tb.step(x, m) for _ in range(2)]
        same_step = la == lb and all(torch.equal(a, b) for a, b in zip(ta.model.state_dict().values(),
                                                                        tb.model.state_dict().values()))
        q.put(dict(buckets=len(dp.buckets), mb=round(dp.flat.numel() * 4 / 2 ** 20, 2), grads_equal=grads_equal,
                   same_step=same_step, losses=la))
    except Exception as e:
        q.put(dict(error=repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp_nccl_world1_configs3_workload_bit_identical():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_cfg3_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=500)
    p.join(timeout=120)
    print("RCCL world-1 DP at configs[3] per-rank workload:", res)
    assert "error" not in res, res
    assert p.exitcode == 0
    assert res["buckets"] == 4 and res["mb"] > 29, res  # 31 MB of gradients in 8 MiB buckets
    assert res["grads_equal"], "DP gradients (world 1, RCCL) must equal the plain backward bit for bit"
    assert res["same_step"], "two Trainer steps with DataParallel must equal the plain steps bit for bit"


def _flat_state(model, which):
    ts = [p.detach() for p in model.parameters()] if which == "params" else \
        [b.detach() for b in model.buffers() if b.dtype.is_floating_point]
    return torch.cat([t.reshape(-1).float().cpu() for t in ts])


def _trainer_worker(rank, world, port, q, cfg):
    """World-2 Trainer steps through DataParallel with the HIP engine, gloo carrying the collectives
    (both ranks share the one GPU): bf16, default 8 MiB buckets, weight gradients on the side stream.
    Per step: every rank's parameters equal bit for bit; the BN running statistics differ before the
    broadcast (each replica normalised its own shard) and equal bit for bit after it.  cfg 'fp32'
    additionally returns the step's averaged, clipped gradients and each rank's branch-pinned oracle
    gradients of its shard (fp64 and fp32) for the mean-of-shards check in the parent."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "enhanced-unet_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import dual_ref as D
        from oracle import eunet_ref as R
        from eunet import synth
        from eunet.dp import DataParallel
        from eunet.engine import UNetEngine
        from eunet.models import EnhancedUNet
        from eunet.train_eval import Trainer
        assert UNetEngine.overlap_wgrad
        dual = cfg == "dual"
        base, H, dt = {"single": (64, 256, "bf16"), "dual": (16, 64, "bf16"), "fp32": (16, 64, "fp32")}[cfg]
        W = (D.dual_formula_weights if dual else R.formula_weights)(base, 1, 2)
        mod = EnhancedUNet(num_classes=2, in_channels=1, base_ch=base, dtype=dt, dual_branch=dual)
        mod.load_state_dict({k: (v.float() if v.is_floating_point() else v) for k, v in W.items()})
        mod = mod.cuda().train()
        if dual:
            gen = torch.Generator().manual_seed(9 + rank)
            mod._engine.drop_keep = ((torch.rand(2, 256, generator=gen) > 0.2).float(),
                                     (torch.rand(2, 128, generator=gen) > 0.15).float())
        tr = Trainer(mod, "cuda", "enhanced_unet")
        for g in tr.optimizer.param_groups:
            g["lr"] = 1e-3
        tr.dp = DataParallel(mod)  # default buckets
        out = dict(rank=rank, buckets=len(tr.dp.buckets), steps=[])
        if cfg == "fp32":
            import _pins
            _pins.keep(mod)
        for step in range(3):
            x, m = synth.batch(2, H, H, start_index=300 + 10 * step + 2 * rank, num_classes=2, in_channels=1,
                               device="cuda")
            loss = tr.step(x, m)
            torch.cuda.synchronize()
            params = _flat_state(mod, "params")
            pre = _flat_state(mod, "buffers")
            tr.dp.before_forward()  # the broadcast the next step starts with
            torch.cuda.synchronize()
            post = _flat_state(mod, "buffers")
            gs = [torch.zeros_like(t) for t in (params, pre, post) for _ in range(world)]
            for i, t in enumerate((params, pre, post)):
                dist.all_gather(gs[i * world:(i + 1) * world], t)
            P, B0, B1 = gs[:world], gs[world:2 * world], gs[2 * world:]
            rec = dict(loss=loss, params_equal=all(torch.equal(P[0], t) for t in P[1:]),
                       pre_differ=not all(torch.equal(B0[0], t) for t in B0[1:]),
                       post_equal=all(torch.equal(B1[0], t) for t in B1[1:]))
            if cfg == "fp32" and step == 0:
                pins = _pins.model_pins(mod)
                # numpy arrays travel through the queue by value (torch CPU tensors would be shared through
                # files that vanish with this process)
                rec["grads"] = {k: p.grad.detach().double().cpu().numpy() for k, p in mod.named_parameters()}
                for odt, key in ((torch.float64, "oracle64"), (torch.float32, "oracle32")):
                    S = R.formula_weights(base, 1, 2, dtype=odt)
                    for k in S:
                        if S[k].is_floating_point() and "running" not in k:
                            S[k].requires_grad_(True)
                    orec = {} if odt == torch.float64 else None
                    R.batch_loss(R.forward(S, x.cpu().to(odt), True, pins=pins, record=orec), m.cpu()).backward()
                    if orec is not None:  # every disputed branch within rounding of its kink / tie
                        rec["pin_audit"] = _pins.audit(pins, orec, "fp32", label=f"world-{world} rank {rank}")
                    rec[key] = {k: S[k].grad.double().numpy() for k in rec["grads"]}
            out["steps"].append(rec)
        q.put(out)
    except Exception as e:  # report instead of hanging the parent on q.get
        import traceback
        q.put(dict(rank=rank, error=traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _run_world2(cfg, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, world, port, q, cfg)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in procs:
            r = q.get(timeout=500)
            res.append(r)
            # a rank that failed leaves its peer blocked in a collective: stop both now
            assert "error" not in r, r["error"]
    finally:
        for p in procs:
            p.join(timeout=60 if all("error" not in r for r in res) else 1)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    for p in procs:
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r["rank"])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cfg", ["single", "dual"])
def test_dp_world2_trainer_steps_keep_replicas_identical(cfg):
    """Three clipped AdamW Trainer steps at world size 2 (train_eval.py:337-343 per rank + the
    gradient all-reduce): single-branch base 64 at 256^2 and the dual model (its own bucket order:
    fusion head -> gate -> unetpp -> deeplab) at base 16; bf16, default buckets, side-stream weight
    gradients.  After every step both ranks hold bit-identical parameters; the BN running statistics
    differ between the replicas until rank 0's are broadcast, and are bit-identical after it."""
    res = _run_world2(cfg)
    for r in res:
        print(cfg, "rank", r["rank"], "buckets", r["buckets"], [(s["loss"], s["params_equal"], s["pre_differ"],
                                                                   s["post_equal"]) for s in r["steps"]])
        assert len(r["steps"]) == 3
        for s in r["steps"]:
            assert s["params_equal"] and s["post_equal"] and s["pre_differ"], s
    assert res[0]["steps"][-1]["loss"] != res[1]["steps"][-1]["loss"]  # the shards really differ


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_dp_world2_step_is_mean_of_shards_oracle(world):
    """fp32 step at world size 2 and 4 (base 16, 64^2, B 2 per rank; all ranks share the one GPU, gloo
    carries the collectives): the all-reduced, clipped gradients every rank applies equal the oracle's
    mean over the shards of each shard's branch-pinned gradient (its own BatchNorm statistics, as
    per-replica BN under DDP), clipped to total norm 1.0 (train_eval.py:341), within max(1e-3, 3x the
    fp32 oracle's error) relative L2 per tensor."""
    res = _run_world2("fp32", world)
    st = [r["steps"][0] for r in res]
    s0 = st[0]
    for s in st:
        assert s["params_equal"] and s["post_equal"]

    for s in st:
        for key in ("grads", "oracle64", "oracle32"):
            s[key] = {k: torch.from_numpy(v) for k, v in s[key].items()}

    def mean_clipped(key):
        g = {k: sum(s[key][k] for s in st) / world for k in s0[key]}
        norm = float(torch.sqrt(sum((v ** 2).sum() for v in g.values())))
        c = min(1.0, 1.0 / (norm + 1e-6))
        return {k: v * c for k, v in g.items()}

    ref, ref32 = mean_clipped("oracle64"), mean_clipped("oracle32")
    scale = max(float(v.abs().max()) for v in ref.values())
    rows = []
    for k, g in s0["grads"].items():
        assert all(torch.equal(g, s["grads"][k]) for s in st[1:]), k
        if k.endswith((".0.bias", ".3.bias")) and not k.startswith("enhance.3"):
            assert float((g - ref[k]).abs().max()) < 1e-4 * scale, k
            continue
        err = float((g - ref[k]).norm() / ref[k].norm().clamp_min(1e-30))
        tol = max(1e-3, 3 * float((ref32[k] - ref[k]).norm() / ref[k].norm().clamp_min(1e-30)))
        rows.append((err / tol, k, err, tol))
    for r in sorted(rows, reverse=True)[:4]:
        print(f"world-{world} mean-of-shards grad (ratio, name, err, tol):", r)
    assert all(r[0] < 1.0 for r in rows), sorted(rows, reverse=True)[:3]
