"""Drop-in training loop of reference train_eval.py for the Enhanced-UNet path.

Trainer keeps the reference constructor, hyper-parameters and attributes
(train_eval.py:63-132): AdamW(lr 4e-3, wd 1e-4, betas (0.9, 0.999)), warmup
LinearLR(0.001 -> 1, max(1, min(5, E//6)) epochs) + CosineAnnealingWarmRestarts
(T_0 = max(10, E//3), T_mult 2, eta_min 1e-7), loss weights 2.5/2.5/1.0.
train_epoch(dataloader) -> mean loss, same batch dict as dataset.collate_fn
(dataset.py:355-361): {'images': [B,C,H,W] float in [0,1],
'batch_items': [{'semantic_mask': [H,W] int}, ...]}.

Differences that are implementation, not semantics:
  * the per-sample loss loop (train_eval.py:262-335) runs as one batched HIP
    kernel (per-sample sums are kept per sample);
  * the 2H->H bilinear resize of the logits (train_eval.py:306-310) is fused
    into the network tail as the exact 2x2 mean it is;
  * clip_grad_norm_ + AdamW run as one native step (eunet.optim.ClipAdamW) on torch's AdamW state;
    Trainer.native_clip_adamw = False restores torch's clip + fused AdamW.
"""
from __future__ import annotations

import collections
import gc
import math
import warnings
from typing import Dict

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import losses as L
from . import ops
from .losses import CrossEntropyLoss, FocalLoss, check_targets, combined_loss, consistency_loss  # noqa: F401
from .models import EnhancedUNet


class Trainer:
    def __init__(self, model, device, model_name, total_epochs: int = 50):
        self.model = model
        self.device = device
        self.model_name = model_name
        self.total_epochs = max(1, total_epochs)
        if model_name != "enhanced_unet":
            raise ValueError("this build implements the enhanced_unet training path only")
        # train_eval.py:74-80: the focal and CE modules with the reference's class weights
        class_weights = torch.tensor([1.0, 20.0, 10.0]).to(device)
        alpha = [1.0, 8.0, 5.0]
        self.focal_loss = FocalLoss(alpha=alpha, gamma=5.0, ignore_index=None, class_weights=class_weights)
        self.ce_loss = CrossEntropyLoss(weight=class_weights)
        self.dice_loss_weight = 2.5
        self.focal_loss_weight = 2.5
        self.tversky_loss_weight = 1.0
        self.aux_branch_weights = {"unetpp": 0.6, "deeplab": 0.5}
        self.consistency_weight = 0.4
        base_lr = 4e-3
        params = [p for p in model.parameters()]
        try:
            self.optimizer = torch.optim.AdamW(params, lr=base_lr, weight_decay=1e-4, betas=(0.9, 0.999),
                                               fused=True)
        except (RuntimeError, TypeError):
            self.optimizer = torch.optim.AdamW(params, lr=base_lr, weight_decay=1e-4, betas=(0.9, 0.999),
                                               foreach=True)
        self.warmup_epochs = max(1, min(5, self.total_epochs // 6))
        self.scheduler = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(
            self.optimizer, T_0=max(10, self.total_epochs // 3), T_mult=2, eta_min=1e-7)
        self.warmup_scheduler = torch.optim.lr_scheduler.LinearLR(
            self.optimizer, start_factor=0.001, end_factor=1.0, total_iters=self.warmup_epochs)
        self.dp = None  # eunet.dp.DataParallel when training on several GPUs
        # clip_grad_norm_ + AdamW as one native step (eunet.optim.ClipAdamW, csrc/optim.hip) when the
        # optimizer allows it (CUDA fp32 parameters, one group); False: torch's clip + fused AdamW
        self.native_clip_adamw = True
        self._clip_adamw = None
        # step_graph: replay deferred-loss steps from captured HIP graphs (StepGraph) once
        # graph_warmup eager steps have run; one graph per batch shape (a ragged last batch keeps
        # its own), at most graph_cache of them, re-captured when the engine schedule, the loss
        # parameters or the parameter storage change (not the learning rate: AdamW runs eagerly)
        self.step_graph = False
        self.graph_warmup = 2
        self.graph_cache = 4
        self._graphs = {}  # key -> StepGraph, least recently used first
        self._graph = None  # the graph of the last replayed step
        self._graph_warm = {}  # engine knobs + dtype (key[5]) -> eager warm-up steps run with them
        self.graph_captures = 0
        # max_inflight: deferred-loss steps (sync_loss=False) the host may run ahead of the GPU.  The weight
        # gradients' operands are record_stream-ed on the side stream, so the caching allocator can reuse
        # them only once the GPU has passed that step: a host that ran 20+ steps ahead reserved a step's
        # activations per queued step until hipMalloc failed, and the allocator's retry (device sync,
        # free every cached block, allocate again) idled the GPU for 1.5-6 s (bench r5: allocator
        # num_alloc_retries 2 inside the timed region).  Two steps in flight keep the GPU fed (a step's
        # host issue takes ~6 ms, its GPU time >= 22 ms) with a bounded footprint.
        self.max_inflight = 2
        self._inflight = collections.deque()

    # ---- reference loss API (single sample, logits [K,H,W], target [H,W]) ----
    def loss_params(self):
        """The combined loss as _compute_combined_loss forms it from this Trainer's attributes
        (train_eval.py:183-197): self.focal_loss's alpha / gamma / class_weights / ignore_index,
        Dice / Tversky class weights, the three term weights, num_classes = 3."""
        f = self.focal_loss
        return L.make_params(ce_weight=f.class_weights, alpha=f.alpha, gamma=f.gamma, ignore_index=f.ignore_index,
                             w_focal=self.focal_loss_weight, w_dice=self.dice_loss_weight,
                             w_tversky=self.tversky_loss_weight, class_div=3.0)

    def _compute_combined_loss(self, logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return combined_loss(logits.unsqueeze(0), target.long().to(logits.device).unsqueeze(0),
                             params=self.loss_params())

    def dice_loss(self, pred, target, num_classes=3):
        return L.dice_loss(pred, target, num_classes)

    def tversky_loss(self, pred, target, num_classes=3, alpha=0.7):
        return L.tversky_loss(pred, target, num_classes, alpha)

    def aux_loss(self, fused, aux_outputs, masks):
        """Batched train_eval.py:326-337 with _apply_auxiliary_supervision (:199-234):
        (1/B) sum_i [CL(fused_i) + sum_b w_b (CL(branch_b,i) + consistency_weight MSE(p_b,i, p_f,i))]."""
        prm = self.loss_params()
        loss = combined_loss(fused, masks, params=prm)
        if not aux_outputs or not self.aux_branch_weights:
            return loss
        for name, w in self.aux_branch_weights.items():
            loss = loss + w * combined_loss(aux_outputs[name], masks, params=prm)
        if self.consistency_weight > 0:
            (n0, w0), (n1, w1) = list(self.aux_branch_weights.items())
            loss = loss + consistency_loss(fused, aux_outputs[n0], aux_outputs[n1], self.consistency_weight * w0,
                                           self.consistency_weight * w1)
        return loss

    # ---- the hot loop ----------------------------------------------------------
    @staticmethod
    def _masks(batch, device, h_pad, w_pad):
        ms = []
        for item in batch["batch_items"]:
            m = item["semantic_mask"]
            if m.dim() != 2:
                m = m.squeeze()
                if m.dim() != 2:
                    raise ValueError(f"gt_mask should be 2D after squeeze, got {tuple(m.shape)}")
            ms.append(m)
        m = torch.stack(ms).to(device, non_blocking=True).long()
        if h_pad or w_pad:
            m = F.pad(m, (0, w_pad, 0, h_pad), mode="constant", value=0)
        return m

    def step(self, images: torch.Tensor, masks: torch.Tensor, sync_loss: bool = True):
        """One optimisation step on device-resident images [B,C,H,W] / masks [B,H,W].

        With self.step_graph set, a deferred-loss step (sync_loss=False, no DataParallel) replays a
        captured HIP graph of this same step (StepGraph): same kernels, same bits, one launch.

        A target outside [0, K) leaves the model as the reference leaves it when its loss raises
        (train_eval.py:325 -> FocalLoss:39, before backward and optimizer.step()): with sync_loss the
        step raises before its update; deferred, the update guard (ops.set_update_guard, pointed at the
        loss's device-side count of such targets) keeps this step and every later one from touching
        the parameters, the optimizer state and the BN running statistics until check_targets()
        raises at the next host synchronisation."""
        if images.is_cuda:
            ops.set_update_guard(images.device, L.bad_target_accumulator(images.device))
        if self.step_graph and not sync_loss and self.dp is None and images.is_cuda:
            out = self._graphed_step(images, masks)
        else:
            out = self._step(images, masks, sync_loss)
        if not sync_loss and images.is_cuda:
            self._bound_inflight()
        return out

    def _bound_inflight(self):
        """Block the host until at most max_inflight deferred steps are queued on the GPU."""
        ev = torch.cuda.Event()
        ev.record()
        self._inflight.append(ev)
        while len(self._inflight) > max(1, self.max_inflight):
            self._inflight.popleft().synchronize()

    def _graphed_step(self, images, masks):
        key = StepGraph.key(self, images, masks)
        g = self._graphs.pop(key, None)
        if g is None:
            warm = self._graph_warm.get(key[5], 0)
            if warm < self.graph_warmup:
                # eager warm-up steps (real steps): lazy allocations, AdamW state, the loss tables'
                # host copies, every kernel's first launch happen outside the capture -- again after a
                # dtype / schedule change (its buffers and kernels are new)
                self._graph_warm[key[5]] = warm + 1
                return self._step(images, masks, False)
            self._trim_graphs(max(1, self.graph_cache) - 1)  # free pools before capturing anew
            g = StepGraph(self, images, masks, key)
            self.graph_captures += 1
        self._graphs[key] = g  # most recently used last
        self._graph = g
        self._trim_graphs(max(1, self.graph_cache))
        return g.replay(images, masks)

    def _trim_graphs(self, n):
        """Drop least recently used graphs (and their memory pools) until n remain."""
        while len(self._graphs) > n:
            old = self._graphs.pop(next(iter(self._graphs)))
            if old is self._graph:
                self._graph = None
            del old

    def _native_opt(self) -> bool:
        from . import optim
        if not self.native_clip_adamw or not optim.supported(self.optimizer):
            return False
        if self._clip_adamw is None or self._clip_adamw.optimizer is not self.optimizer:
            self._clip_adamw = optim.ClipAdamW(self.optimizer)
        return True

    def _optimizer_step(self):
        """train_eval.py:341-343's clip_grad_norm_(max_norm=1.0) + optimizer.step(): the clip runs
        here (fused with AdamW) on the native path, in _forward_backward otherwise."""
        if self._native_opt():
            self._clip_adamw.step(1.0)
        else:
            self.optimizer.step()

    def _step(self, images, masks, sync_loss):
        loss = self._forward_backward(images, masks, sync_loss)
        self._optimizer_step()
        if not sync_loss:
            return loss.detach()
        return loss.item()

    def _forward_backward(self, images, masks, sync_loss):
        """zero_grad, forward, loss, backward, DP all-reduce and -- unless the native optimizer step
        runs it fused with AdamW -- clip_grad_norm_ (train_eval.py:244-345 up to the optimizer step); a
        StepGraph captures exactly this."""
        self.model.train()
        _, _, h, w = images.shape
        h_pad, w_pad = (32 - h % 32) % 32, (32 - w % 32) % 32
        if h_pad or w_pad:  # train_eval.py:248-253
            images = F.pad(images, (0, w_pad, 0, h_pad), mode="reflect")
            masks = F.pad(masks, (0, w_pad, 0, h_pad), mode="constant", value=0)
        self.optimizer.zero_grad(set_to_none=True)
        if self.dp is not None:
            self.dp.before_forward()
        if isinstance(self.model, EnhancedUNet) and self.model.dual_branch:
            # SMP-path model: fused + branch outputs at mask size (train_eval.py:255-257, 326-335)
            fused = self.model(images)
            loss = self.aux_loss(fused, self.model.get_aux_outputs(), masks)
        else:
            if isinstance(self.model, EnhancedUNet):
                logits = self.model.forward_lowres(images)
            else:
                out = self.model(images)
                logits = F.interpolate(out, size=masks.shape[-2:], mode="bilinear", align_corners=False)
            loss = combined_loss(logits, masks, params=self.loss_params())
        if sync_loss:
            # out-of-range targets raise here, before backward and the update, where the reference's
            # F.cross_entropy raises (one extra host sync; the deferred path below has none)
            check_targets()
        loss.backward()
        if self.dp is not None:
            self.dp.after_backward()
        if not self._native_opt():
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=1.0, foreach=True)
        return loss

    def train_epoch(self, dataloader):
        """Mean loss over the epoch (train_eval.py:236-353).  A target outside [0, K) raises ValueError
        with the model in the state the reference's raise at that batch leaves it (train_eval.py:325 ->
        FocalLoss:39, before that batch's backward and optimizer.step()): the earlier batches' updates
        applied, that batch's and later ones' not (parameters, AdamW state, BN running statistics --
        that batch's forward did update them, as there).  On the native optimizer path the steps are
        deferred (one host sync per epoch): the update guard (Trainer.step) holds the state from the
        offending loss on, the remaining batches run without effect and the error is raised at the
        epoch's sync.  With torch's optimizer every step synchronises and raises before its update."""
        self.model.train()
        deferred = str(self.device).startswith("cuda") and self._native_opt()
        total = None  # device-side running sum: one host sync per epoch, not per step
        n = 0
        for batch in dataloader:
            images = batch["images"].to(self.device, non_blocking=True)
            masks = self._masks(batch, self.device, 0, 0)
            if deferred:
                loss = self.step(images, masks, sync_loss=False).double()
            else:
                loss = self.step(images, masks, sync_loss=True)
            total = loss if total is None else total + loss
            n += 1
        check_targets()
        return float(total) / n if n else 0.0

    def epoch_lr_step(self, epoch: int) -> float:
        """train_model's per-epoch stepping (train_eval.py:1104-1111).  The reference steps the
        scheduler at the start of the epoch, before any optimizer.step(); torch warns about
        that order, the LR trajectory is the reference's (pinned by lr_traj.npz)."""
        with warnings.catch_warnings():
            warnings.filterwarnings("ignore", message="Detected call of `lr_scheduler.step\\(\\)` before")
            if epoch < self.warmup_epochs:
                self.warmup_scheduler.step()
            else:
                self.scheduler.step()
        return self.optimizer.param_groups[0]["lr"]


ENGINE_KNOBS = ("overlap_wgrad", "materialize_za", "fuse_bn_reduce", "wg3_late", "fuse_bn_apply", "fuse_bn_apply_a",
                "dgrad_first", "wg3_early_last", "fork_once", "dec1_recompute", "pool_recompute", "device_fence_forks",
                "narrow_mfma")


def _engine_knobs(eng):
    """Every schedule knob a captured step depends on: the engine's, and for the dual-branch engine its
    two trunk engines' too (their knobs are UNetEngine class attributes unless set per instance)."""
    engines = [eng] + [getattr(eng, n) for n in ("ea", "eb") if hasattr(eng, n)]
    return tuple(tuple(_hashable(getattr(e, k, None)) for k in ENGINE_KNOBS) for e in engines)


def _hashable(v):
    """A per-block knob (a set of block names) as a sorted tuple, for the graph key."""
    return tuple(sorted(v)) if isinstance(v, (set, frozenset, list)) else v


class StepGraph:
    """A Trainer step's forward, fused loss and backward (+ clip_grad_norm_ on the torch optimizer
    path) captured as a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm) and replayed per batch,
    followed by the eager optimizer step (the native clip + AdamW, or torch's fused AdamW): a few host
    calls instead of several hundred launches, so a small tile (the reference's
    640x480 batch of 2) is no longer bound by Python + ctypes issue and the data loader's host work
    fits beside it.

    A replay runs the eager step's kernels in the eager order with the same arguments: the engine
    launches on torch's current stream (the capture stream) and forks / joins its weight-gradient
    side stream with events; the loss adds its out-of-range target count into a persistent device
    accumulator in place (losses.bad_target_accumulator); the gradient norm and the BN running
    statistics never leave the device.  The gradients live in the graph's memory pool: a replay
    points the parameters' .grad at them before AdamW runs.  AdamW stays outside the graph because
    its learning rate is a host double that changes every epoch (a device-tensor LR would be rounded
    to fp32, and re-capturing per epoch costs more than the launches it saves).  What the graph
    bakes in from the host is in key(): shapes, the loss parameters, the engine schedule and the
    parameter storage (load_state_dict replacing it -> re-capture)."""

    def __init__(self, trainer, images, masks, key):
        from . import losses as _L
        self.key = key
        dev = images.device
        self.images = torch.empty_like(images)
        self.masks = torch.empty_like(masks)
        _L.bad_target_accumulator(dev)
        self.optimizer = trainer.optimizer
        self.optimizer_step = trainer._optimizer_step
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: a DataLoader producer thread may launch and allocate on its own stream
        # while this thread captures (the default global mode would invalidate the capture).
        # The cyclic garbage collector is off during the capture (torch.cuda.graph collects right before
        # it): a collection inside it would run the finalizers of earlier steps' objects -- a
        # torch.cuda.Event's hipEventDestroy among them -- in the middle of the capture, where HIP refuses
        # them ("operation not permitted when stream is capturing", seen from the autograd thread)
        gc_was_on = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self.loss = trainer._forward_backward(self.images, self.masks, False).detach()
        finally:
            if gc_was_on:
                gc.enable()
        self.params = [p for g in self.optimizer.param_groups for p in g["params"]]
        self.grads = [p.grad for p in self.params]

    def replay(self, images, masks):
        from . import losses as _L
        self.images.copy_(images, non_blocking=True)
        self.masks.copy_(masks, non_blocking=True)
        self.graph.replay()
        _L.mark_pending()
        for p, g in zip(self.params, self.grads):
            if p.grad is not g:
                p.grad = g
        self.optimizer_step()
        return self.loss.clone()

    @staticmethod
    def key(trainer, images, masks):
        eng = getattr(trainer.model, "_engine", None)
        if getattr(eng, "drop_keep", None) is not None:
            raise RuntimeError("Trainer.step_graph: fixed dropout keep masks (a test hook) are host inputs")
        # the compute dtype is baked into the captured kernels and buffers: EnhancedUNet.set_dtype
        # (which only changes the engine's dtype) must re-capture
        knobs = _engine_knobs(eng) + (str(getattr(eng, "dtype", None)), str(getattr(trainer.model, "compute_dtype", None)))
        ps = [p for g in trainer.optimizer.param_groups for p in g["params"]]
        store = (id(trainer.optimizer), ps[0].data_ptr(), ps[-1].data_ptr(), len(ps))
        lossp = (bytes(trainer.loss_params()), tuple(trainer.aux_branch_weights.items()), trainer.consistency_weight,
                 trainer._native_opt())  # where the clip runs (in the graph or in the native step)
        return (tuple(images.shape), images.dtype, images.device, tuple(masks.shape), masks.dtype, knobs, store,
                lossp)


from .evaluator import Evaluator  # noqa: E402,F401  (train_eval.Evaluator, train_eval.py:356-904)


# ---- train_model driver + checkpoint interchange (train_eval.py:1036-1162, 1186-1202) -------
CHECKPOINT_KEYS = ("epoch", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict", "best_miou",
                   "best_loss", "history")


def train_model(model_name: str, data_dir: str = None, device: str = "cuda", num_epochs: int = 50,
                skip_training: bool = False, *, train_loader=None, val_loader=None, save_dir: str = None,
                model=None, verbose: bool = True, step_graph: bool = None, loader_workers: int = None,
                **model_kwargs):
    """train_eval.train_model: per-epoch LR stepping (warmup LinearLR, then cosine restarts) before
    each train_epoch, semantic validation every 3 epochs, best-mIoU checkpoint in the reference's
    dict format ('checkpoints/<model>/best_model.pth'), early stop after patience 10 (epoch > 25).

    Without train_loader / val_loader it builds the reference's loaders (train_eval.py:1054-1075):
    eunet.data.CellDataset(data_dir, 'train' / 'val', max_size=640), batch 2 on cuda (1 otherwise),
    the train split shuffled, val batch 1; on cuda the training loader prefetches 2 batches and,
    with loader_workers > 0 (opt-in; default 0 = the reference's num_workers=0), decodes in that many
    'spawn' worker processes -- the calling script then needs an `if __name__ == "__main__":` guard.
    The Python `random` augmentation decisions follow the reference's draw order; the Gaussian noise
    values do so only with host_noise (eunet.data.CellDataset).
    Any iterable of collate_fn batch dicts ({'images', 'batch_items': [{'semantic_mask'}]}) may be
    passed instead, e.g. eunet.synth.loader.  step_graph (default: on for the single-branch model on
    cuda) replays the training steps from captured HIP graphs (Trainer.step_graph, bit-identical)."""
    import os
    from .models import get_model
    save_dir = save_dir or os.path.join("checkpoints", model_name)
    os.makedirs(save_dir, exist_ok=True)
    checkpoint_path = os.path.join(save_dir, "best_model.pth")
    if os.path.exists(checkpoint_path) and skip_training:
        return checkpoint_path
    own_loader = train_loader is None
    if train_loader is None:
        from .data import CellDataset, DataLoader, collate_fn
        if data_dir is None:
            raise ValueError("train_model needs data_dir (a LabelMe directory) or explicit loaders")
        on_gpu = str(device).startswith("cuda")
        batch_size = 2 if on_gpu else 1  # train_eval.py:1058-1059
        workers = 0 if loader_workers is None else loader_workers
        train_loader = DataLoader(CellDataset(data_dir, split="train", max_size=640, device=device),
                                  batch_size=batch_size, shuffle=True, collate_fn=collate_fn, workers=workers,
                                  prefetch=2 if on_gpu else 0)
        if val_loader is None:
            val_loader = DataLoader(CellDataset(data_dir, split="val", max_size=640, device=device), batch_size=1,
                                    shuffle=False, collate_fn=collate_fn)
    if model is None:
        model = get_model(model_name, num_classes=3, device=device, **model_kwargs).to(device)
    history = {"train_loss": [], "val_loss": [], "val_miou": [], "val_live_iou": [], "val_dead_iou": [],
               "val_dice": [], "learning_rate": [], "epoch_axis": []}
    train_epochs = num_epochs
    trainer = Trainer(model, device, model_name, total_epochs=train_epochs)
    if step_graph is None:
        step_graph = str(device).startswith("cuda") and not getattr(model, "dual_branch", False)
    trainer.step_graph = bool(step_graph)
    patience = 10 if model_name == "enhanced_unet" else 8
    try:
        _train_epochs(trainer, model, model_name, device, train_loader, val_loader, history, checkpoint_path,
                      train_epochs, patience, verbose)
    finally:
        close = getattr(train_loader, "close", None) if own_loader else None
        if callable(close):  # worker processes end with the training, not at garbage collection
            close()
    return checkpoint_path


def _train_epochs(trainer, model, model_name, device, train_loader, val_loader, history, checkpoint_path,
                  train_epochs, patience, verbose):
    best_loss, best_miou = float("inf"), 0.0
    patience_counter = 0
    for epoch in range(train_epochs):
        current_lr = trainer.epoch_lr_step(epoch)
        loss = trainer.train_epoch(train_loader)
        history["train_loss"].append(loss)
        history["learning_rate"].append(current_lr)
        if verbose:
            print(f"Epoch {epoch + 1}/{train_epochs}  lr {current_lr:.6f}  loss {loss:.4f}")
        if (epoch + 1) % 3 == 0:
            res = Evaluator(model, device, model_name).evaluate_semantic(val_loader or train_loader)
            val_iou = res.get("sem_mean_iou", 0.0)
            history["val_miou"].append(val_iou)
            history["val_live_iou"].append(res.get("sem_live_iou", 0.0))
            history["val_dead_iou"].append(res.get("sem_dead_iou", 0.0))
            history["val_dice"].append([res.get("sem_live_dice", 0.0), res.get("sem_dead_dice", 0.0)])
            history["val_loss"].append(loss)
            history["epoch_axis"].append(epoch + 1)
            if val_iou > best_miou:
                best_miou, best_loss, patience_counter = val_iou, loss, 0
                torch.save({"epoch": epoch + 1, "model_state_dict": model.state_dict(),
                            "optimizer_state_dict": trainer.optimizer.state_dict(),
                            "scheduler_state_dict": trainer.scheduler.state_dict(), "best_miou": best_miou,
                            "best_loss": best_loss, "history": history}, checkpoint_path)
            else:
                patience_counter += 1
        if patience_counter >= patience and epoch > 25:
            break


def _numpy_safe_globals():
    """The numpy scalar reconstructors a reference checkpoint holds: best_miou and the history
    values are np.float64 (Evaluator.evaluate returns np.mean results, train_eval.py:1017).
    Allow-listed for the weights-only unpickler by name, under numpy 1.x and 2.x module paths;
    nothing else is admitted."""
    import numpy as np
    try:
        from numpy._core import multiarray as ma
    except ImportError:  # numpy < 2
        from numpy.core import multiarray as ma
    out = [ma.scalar, (ma.scalar, "numpy.core.multiarray.scalar"), (ma.scalar, "numpy._core.multiarray.scalar"),
           np.dtype]
    for nm in ("Float64DType", "Float32DType", "Float16DType", "Int64DType", "Int32DType", "BoolDType"):
        dt = getattr(getattr(np, "dtypes", None), nm, None)
        if dt is not None:
            out.append(dt)
    return out


def load_checkpoint(model, checkpoint_path: str, map_location=None):
    """evaluate_model's checkpoint load (train_eval.py:1186-1202) with the weights-only loader:
    tensors, plain containers and numpy scalars (_numpy_safe_globals) only, so reference
    checkpoints (np.float64 best_miou / history) load while nothing executable is admitted.
    Also accepts a bare state_dict."""
    with torch.serialization.safe_globals(_numpy_safe_globals()):
        ckpt = torch.load(checkpoint_path, map_location=map_location or "cpu", weights_only=True)
    sd = ckpt["model_state_dict"] if isinstance(ckpt, dict) and "model_state_dict" in ckpt else ckpt
    model.load_state_dict(sd)
    return ckpt
