"""Data-parallel path on CPU: world sizes 2 and 4 over gloo (SURVEY.md §8e DP oracle).

Each rank computes its shard's gradients with the oracle (the HIP engine needs
a GPU) and feeds them to eunet.dp's BucketSink exactly as the engine does
(slot -> write -> ready(names) in backward order).  Checks: replicas start
identical (rank-0 broadcast), buckets are all-reduced as they complete, and
the result equals the mean of the per-shard gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grads(state, rank):
    from eunet import synth
    from oracle import eunet_ref as R
    S = {k: v.detach().clone().double() if v.is_floating_point() else v.clone() for k, v in state.items()}
    for k in S:
        if S[k].is_floating_point() and "running" not in k:
            S[k].requires_grad_(True)
    x, m = synth.batch(2, 32, 32, start_index=100 + 2 * rank, num_classes=2, in_channels=1)
    R.batch_loss(R.forward(S, x.double(), training=True), m).backward()
    return {k: S[k].grad for k in S if S[k].is_floating_point() and S[k].grad is not None}


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "enhanced-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from eunet.dp import DataParallel
        from eunet.models import EnhancedUNet
        torch.manual_seed(1234 + rank)  # deliberately different replicas before the broadcast
        model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
        with torch.no_grad():
            model.enhance[1].running_mean.fill_(float(rank))
        dp = DataParallel(model, bucket_mb=0.02)
        state = model.state_dict()
        ck = torch.tensor([sum(float(v.double().sum()) for v in state.values() if v.is_floating_point())],
                          dtype=torch.float64)
        cks = [torch.zeros_like(ck) for _ in range(world)]
        dist.all_gather(cks, ck)
        same = all(abs(float(c) - float(cks[0])) < 1e-9 for c in cks)
        mine = _shard_grads(state, rank)
        expected = {k: sum(_shard_grads(state, r)[k] for r in range(world)) / world for k in mine}
        sink = model.grad_sink_factory()
        launched_early = 0
        for name in dp.order:
            slot = sink.slot(name, mine[name].shape)
            slot.copy_(mine[name].float())
            sink.ready([name])
            launched_early = max(launched_early, len(sink.works))
        grads = sink.finish()
        err = max(float((grads[k].double() - expected[k]).abs().max() / expected[k].abs().max().clamp_min(1e-12))
                  for k in expected if not k.endswith((".0.bias", ".3.bias")))
        rm = float(model.enhance[1].running_mean.abs().max())
        dp.before_forward()  # buffers still alias the flat broadcast buffer: fine
        model.double()  # module._apply replaces every buffer: the broadcast would no longer reach them
        try:
            dp.before_forward()
            stale_raised = False
        except RuntimeError:
            stale_raised = True
        q.put((rank, same, len(dp.buckets), launched_early, err, rm, stale_raised))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_dp_world2_gloo_bucketed_allreduce(world):
    """(world 4 rehearses the ring over more ranks than the GPU tests can place on one card with RCCL)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same, nb, early, err, rm, stale_raised in res:
        assert stale_raised, "a buffer replaced after DataParallel was built must be reported"
        assert same, "replicas must be identical after the rank-0 broadcast"
        assert nb > 3, "expected several buckets"
        assert early >= nb - 1, "buckets must be launched as they complete, not at finish()"
        assert err < 1e-5, err
        assert rm == 0.0, "BN running stats broadcast from rank 0"


def test_backward_order_covers_parameters():
    from eunet.dp import backward_order
    from eunet.models import EnhancedUNet
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
    order = backward_order(m)
    assert order[0].startswith("enhance.") and order[-1].startswith("model.enc1.")
    assert sorted(order) == sorted(n for n, _ in m.named_parameters())
