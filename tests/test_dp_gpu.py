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
