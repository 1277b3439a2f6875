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
  * clip_grad_norm_ / AdamW stay PyTorch (foreach/fused kernels).
"""
from __future__ import annotations

import math
import warnings
from typing import Dict

import torch
import torch.nn as nn
import torch.nn.functional as F

from .losses import combined_loss, consistency_loss
from .models import EnhancedUNet


class FocalLoss(nn.Module):
    """API mirror of train_eval.FocalLoss (train_eval.py:28-60) for the Enhanced-UNet
    configuration (alpha [1,8,5], gamma 5, CE weights [1,20,10]); computed by the
    fused loss kernel.  inputs [N,K,H,W], targets [N,H,W] -> mean focal term."""

    def forward(self, inputs, targets):
        _, parts = combined_loss(inputs, targets, return_parts=True)
        return parts[:, 0].mean()


class Trainer:
    def __init__(self, model, device, model_name, total_epochs: int = 50):
        self.model = model
        self.device = device
        self.model_name = model_name
        self.total_epochs = max(1, total_epochs)
        if model_name != "enhanced_unet":
            raise ValueError("this build implements the enhanced_unet training path only")
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

    # ---- reference loss API (single sample, logits [K,H,W], target [H,W]) ----
    def _compute_combined_loss(self, logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return combined_loss(logits.unsqueeze(0), target.long().to(logits.device).unsqueeze(0))

    def dice_loss(self, pred, target, num_classes=3):
        return combined_loss(pred, target, return_parts=True)[1][:, 1].mean()

    def tversky_loss(self, pred, target, num_classes=3, alpha=0.7):
        return combined_loss(pred, target, return_parts=True)[1][:, 2].mean()

    def aux_loss(self, fused, aux_outputs, masks):
        """Batched train_eval.py:326-337 with _apply_auxiliary_supervision (:199-234):
        (1/B) sum_i [CL(fused_i) + sum_b w_b (CL(branch_b,i) + consistency_weight MSE(p_b,i, p_f,i))]."""
        loss = combined_loss(fused, masks)
        if not aux_outputs or not self.aux_branch_weights:
            return loss
        for name, w in self.aux_branch_weights.items():
            loss = loss + w * combined_loss(aux_outputs[name], masks)
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
        """One optimisation step on device-resident images [B,C,H,W] / masks [B,H,W]."""
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
            loss = combined_loss(logits, masks)
        loss.backward()
        if self.dp is not None:
            self.dp.after_backward()
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=1.0, foreach=True)
        self.optimizer.step()
        return loss.item() if sync_loss else loss.detach()

    def train_epoch(self, dataloader):
        self.model.train()
        total = None  # device-side running sum: one host sync per epoch, not per step
        n = 0
        for batch in dataloader:
            images = batch["images"].to(self.device, non_blocking=True)
            masks = self._masks(batch, self.device, 0, 0)
            loss = self.step(images, masks, sync_loss=False).double()
            total = loss if total is None else total + loss
            n += 1
        return float(total.item()) / n if n else 0.0

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


from .evaluator import Evaluator  # noqa: E402,F401  (train_eval.Evaluator, train_eval.py:356-904)


# ---- train_model driver + checkpoint interchange (train_eval.py:1036-1162, 1186-1202) -------
CHECKPOINT_KEYS = ("epoch", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict", "best_miou",
                   "best_loss", "history")


def train_model(model_name: str, data_dir: str = None, device: str = "cuda", num_epochs: int = 50,
                skip_training: bool = False, *, train_loader=None, val_loader=None, save_dir: str = None,
                model=None, verbose: bool = True, **model_kwargs):
    """train_eval.train_model: per-epoch LR stepping (warmup LinearLR, then cosine restarts) before
    each train_epoch, semantic validation every 3 epochs, best-mIoU checkpoint in the reference's
    dict format ('checkpoints/<model>/best_model.pth'), early stop after patience 10 (epoch > 25).

    The reference builds its loaders from CellDataset (cv2 / PIL LabelMe pipeline, dataset.py),
    which this build does not provide: pass train_loader / val_loader yielding the collate_fn batch
    dict ({'images', 'batch_items': [{'semantic_mask'}]}), e.g. eunet.synth.loader."""
    import os
    from .models import get_model
    save_dir = save_dir or os.path.join("checkpoints", model_name)
    os.makedirs(save_dir, exist_ok=True)
    checkpoint_path = os.path.join(save_dir, "best_model.pth")
    if os.path.exists(checkpoint_path) and skip_training:
        return checkpoint_path
    if train_loader is None:
        raise NotImplementedError("CellDataset (dataset.py, cv2/PIL LabelMe loader) is not part of this build: "
                                  "pass train_loader/val_loader")
    if model is None:
        model = get_model(model_name, num_classes=3, device=device, **model_kwargs).to(device)
    history = {"train_loss": [], "val_loss": [], "val_miou": [], "val_live_iou": [], "val_dead_iou": [],
               "val_dice": [], "learning_rate": [], "epoch_axis": []}
    train_epochs = num_epochs
    trainer = Trainer(model, device, model_name, total_epochs=train_epochs)
    best_loss, best_miou = float("inf"), 0.0
    patience = 10 if model_name == "enhanced_unet" else 8
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
    return checkpoint_path


def load_checkpoint(model, checkpoint_path: str, map_location=None):
    """evaluate_model's checkpoint load (train_eval.py:1186-1202), safe loader: the file holds
    only tensors and plain containers, so weights_only=True reads reference checkpoints too.
    Also accepts a bare state_dict."""
    ckpt = torch.load(checkpoint_path, map_location=map_location or "cpu", weights_only=True)
    sd = ckpt["model_state_dict"] if isinstance(ckpt, dict) and "model_state_dict" in ckpt else ckpt
    model.load_state_dict(sd)
    return ckpt
