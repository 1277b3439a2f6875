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
