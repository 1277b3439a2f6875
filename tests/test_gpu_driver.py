"""train_model driver and checkpoint interchange (train_eval.py:1036-1162, 1186-1202) on the GPU."""
import os

import numpy as np
import pytest
import torch

from oracle import eunet_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _SelfLabelledVal:
    """Validation loader whose ground truth is the model's own current prediction: the epoch-3
    validation then scores sem_mean_iou = 1.0 > best_miou = 0, so train_model must write the
    checkpoint (deterministic, whatever the short training learned)."""

    def __init__(self, model, x):
        self.model, self.x = model, x

    def __iter__(self):
        from eunet.evaluator import Evaluator
        ev = Evaluator(self.model, DEV, "enhanced_unet")
        gt = [torch.from_numpy(ev.predict_semantic_mask(img)) for img in self.x]
        self.model.train()
        yield {"images": self.x, "batch_items": [{"semantic_mask": g} for g in gt]}


def test_train_model_checkpoint_roundtrip(tmp_path):
    from eunet import synth
    from eunet.models import EnhancedUNet
    from eunet.train_eval import CHECKPOINT_KEYS, load_checkpoint, train_model
    tl = synth.loader(2, 2, 64, 64, start_index=0, num_classes=3, in_channels=3)
    model = EnhancedUNet(num_classes=3, in_channels=3, base_ch=16).to(DEV)
    vx, _ = synth.batch(1, 64, 64, start_index=50, num_classes=3, in_channels=3)
    path = train_model("enhanced_unet", device=DEV, num_epochs=4, train_loader=tl, val_loader=_SelfLabelledVal(model, vx),
                       save_dir=str(tmp_path), model=model, verbose=False)
    assert os.path.basename(path) == "best_model.pth"
    assert os.path.exists(path), "epoch-3 validation (mIoU 1.0 > 0) must save the checkpoint"
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert set(CHECKPOINT_KEYS) <= set(ck)
    assert ck["epoch"] == 3 and ck["best_miou"] == 1.0
    lrs = ck["history"]["learning_rate"]  # history as saved at the epoch-3 checkpoint
    np.testing.assert_allclose(lrs, R.lr_trajectory(4)[:len(lrs)], rtol=1e-12)
    fresh = EnhancedUNet(num_classes=3, in_channels=3, base_ch=16).to(DEV)
    load_checkpoint(fresh, path)
    for (k, a), (_, b) in zip(ck["model_state_dict"].items(), fresh.state_dict().items()):
        assert torch.equal(a, b.cpu()), k


def test_reference_format_checkpoint_loads(golden_dir, tmp_path):
    """A checkpoint in the reference's dict format (model_state_dict with its 109 keys) loads
    and reproduces the reference's eval-mode output."""
    from eunet.models import EnhancedUNet
    from eunet.train_eval import load_checkpoint
    g = np.load(os.path.join(golden_dir, "fwd_c3k3.npz"), allow_pickle=False)
    sd = {k: (v.float() if v.is_floating_point() else v) for k, v in R.formula_weights(64, 3, 3).items()}
    for k in g.files:
        if k.startswith("bn:"):
            sd[k[3:]] = torch.from_numpy(g[k]).float()
    path = tmp_path / "best_model.pth"
    # the reference writes numpy scalars (np.mean results, train_eval.py:1017) into the dict
    torch.save({"epoch": 3, "model_state_dict": sd, "best_miou": np.float64(0.5), "best_loss": 1.0,
                "history": {"val_miou": [np.float64(0.5)]}}, path)
    m = EnhancedUNet(num_classes=3)
    ck = load_checkpoint(m, str(path))
    assert ck["best_miou"] == 0.5
    m = m.to(DEV).eval()
    with torch.no_grad():
        out = m(torch.from_numpy(g["x"]).to(DEV)).double().cpu()
    ref = torch.from_numpy(g["out_eval"]).double()
    assert float((out - ref).abs().max() / ref.abs().max()) < 1e-3


def test_deferred_steps_bound_the_host_run_ahead():
    """Trainer.step(sync_loss=False) keeps at most max_inflight steps queued (the weight gradients'
    record_stream-ed operands are reusable only once the GPU has passed their step: unbounded run-ahead
    grew the reserved memory until the allocator's OOM retry stalled the GPU for seconds), and the
    bounded deferred steps give the same parameters as synchronous ones, bit for bit."""
    import torch
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    torch.manual_seed(0)
    x = torch.rand(2, 1, 64, 64, device="cuda")
    m = torch.randint(0, 2, (2, 64, 64), device="cuda")
    out = []
    for deferred in (True, False):
        torch.manual_seed(1)
        model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16).to("cuda")
        tr = Trainer(model, "cuda", "enhanced_unet", total_epochs=50)
        tr.epoch_lr_step(0)
        for _ in range(6):
            tr.step(x, m, sync_loss=not deferred)
            assert len(tr._inflight) <= tr.max_inflight
        torch.cuda.synchronize()
        out.append({k: v.detach().clone() for k, v in model.state_dict().items()})
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k


def test_stream_wait_orders_the_side_stream():
    """eunet_stream_wait (the engine's side-stream forks / joins, device-scope event release): work enqueued on
    `to` after the wait sees everything enqueued on `from` before it, across a long producer (the consumer
    would otherwise read the tensor mid-write), for many forks in a row (the event ring wraps)."""
    from eunet import ops
    main, side = torch.cuda.current_stream(), torch.cuda.Stream()
    n = 1 << 24
    a = torch.zeros(n, device=DEV)
    for i in range(80):  # > the ring of 64 events per device
        big = torch.full((n,), float(i + 1), device=DEV)
        for _ in range(3):
            big = big * 1.0 + 0.0  # a few dependent kernels: the producer runs for a while
        a.copy_(big)
        ops.stream_wait(main, side)
        with torch.cuda.stream(side):
            b = a.clone()
        ops.stream_wait(side, main)
        a.record_stream(side)
        b.record_stream(main)
        assert float(b[0]) == float(i + 1) and float(b[-1]) == float(i + 1)
    # the engine's knob: the same step with torch's wait_stream is bit-identical
    from eunet.engine import UNetEngine
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    x = torch.rand(2, 1, 64, 64, device=DEV)
    m = torch.randint(0, 2, (2, 64, 64), device=DEV)
    out = []
    for dev_fence in (True, False):
        old = UNetEngine.device_fence_forks
        UNetEngine.device_fence_forks = dev_fence
        try:
            torch.manual_seed(1)
            model = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16, dtype="bf16").to(DEV)
            tr = Trainer(model, DEV, "enhanced_unet", total_epochs=50)
            tr.epoch_lr_step(0)
            for _ in range(2):
                tr.step(x, m)
            torch.cuda.synchronize()
            out.append({k: v.detach().clone() for k, v in model.state_dict().items()})
        finally:
            UNetEngine.device_fence_forks = old
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k
