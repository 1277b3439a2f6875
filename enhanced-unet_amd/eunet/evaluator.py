"""Drop-in inference path of reference train_eval.Evaluator (semantic part).

    Evaluator(model, device, model_name)                       # train_eval.py:356-363
    ._run_model_single(image [C,h,w]) -> probs [K,h,w]          # train_eval.py:397-417
    ._run_tta_inference(image) -> probs (5-view TTA mean)       # train_eval.py:419-453
    ._convert_probs_to_mask(probs) -> int64 mask [h,w] (numpy)  # train_eval.py:455-568
    .predict_semantic_mask(image) -> int64 mask [h,w] (numpy)   # train_eval.py:570-606
    .evaluate_semantic(dataloader) -> mean semantic metrics     # train_eval.py:852-904 (semantic rows)

Every per-pixel step runs in HIP (evalpath.hip): the flips and 0.75/1.25
rescales (PyTorch bilinear index math), softmax + crop, the TTA mean, the
thresholded mask conversion (two passes; the pixel-ratio refinement reads the
pass-1 counts on the device).  The network is the fused forward_lowres (the
2H->H bilinear resize of train_eval.py:413 is the exact 2x2 mean it computes).

_prepare_image_tensor (train_eval.py:365-395) runs in HIP too (imgproc.hip):
CHW float -> uint8 (x255 when max <= 1), RGB -> Lab, CLAHE(2.0, 8x8) on L,
Lab -> RGB, filter2D sharpening x0.15, /255.  cv2 is absent, so those kernels
follow OpenCV's documented algorithms (parity unpinned, oracle/imgproc_ref.py).
preprocess=None skips the step, a callable replaces it.

Not built: instance splitting / COCO metrics (cv2, skimage,
pycocotools).
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Optional, Union

import numpy as np
import torch
import torch.nn.functional as F

from . import ops
from .metrics import calculate_semantic_metrics

TTA_SCALES = (0.75, 1.25)


def reference_preprocess(image: torch.Tensor) -> torch.Tensor:
    """train_eval.py:365-395 on the device: [3,h,w] float -> CLAHE(2.0) + sharpen(0.15) -> [3,h,w] / 255."""
    if image.dim() != 3 or image.shape[0] != 3:
        raise ValueError("the reference preprocessing converts RGB -> Lab: image must be [3, h, w]")
    u8 = ops.chw_to_u8(image)
    return ops.to_tensor(ops.sharpen_u8(ops.clahe_rgb_u8(u8, 2.0), 0.15))


class Evaluator:
    def __init__(self, model, device, model_name, preprocess: Union[str, Callable, None] = "reference"):
        self.model = model
        self.device = device
        self.model_name = model_name
        self.enable_tta = model_name == "enhanced_unet"
        self.preprocess = preprocess

    # ---- train_eval.py:365-395 -------------------------------------------------
    def _prepare_image_tensor(self, image: torch.Tensor) -> torch.Tensor:
        image = image.to(self.device).float()
        if self.preprocess is None:
            return image
        if callable(self.preprocess):
            return self.preprocess(image)
        if self.preprocess != "reference":
            raise ValueError(f"preprocess must be 'reference', None or a callable, not {self.preprocess!r}")
        return reference_preprocess(image)

    def _logits(self, image_padded: torch.Tensor) -> torch.Tensor:
        m = self.model
        if hasattr(m, "forward_lowres"):
            return m.forward_lowres(image_padded)
        out = m(image_padded)
        return F.interpolate(out, size=image_padded.shape[-2:], mode="bilinear", align_corners=False)

    # ---- train_eval.py:397-417 -------------------------------------------------
    def _run_model_single(self, image: torch.Tensor, flip_h: bool = False, flip_w: bool = False) -> torch.Tensor:
        """image [C,h,w] on the device -> softmax probs [K,h,w]; flip_* mirror the
        probabilities back (the TTA flips of train_eval.py:427-437)."""
        h, w = image.shape[1:]
        h_pad, w_pad = (32 - h % 32) % 32, (32 - w % 32) % 32
        x = image.unsqueeze(0)
        if h_pad or w_pad:
            x = F.pad(x, (0, w_pad, 0, h_pad), mode="reflect")
        logits = self._logits(x)[0]
        return ops.softmax_crop(logits, h, w, flip_h=flip_h, flip_w=flip_w)

    # ---- train_eval.py:419-453 -------------------------------------------------
    def _run_tta_inference(self, image: torch.Tensor) -> torch.Tensor:
        image = image.contiguous().float()
        acc = self._run_model_single(image)
        if not self.enable_tta:
            return acc
        h, w = image.shape[1:]
        views = 1 + 2 + len(TTA_SCALES)
        done = 1
        for fh, fw in ((False, True), (True, False)):  # horizontal (dims=[2]) then vertical (dims=[1])
            flipped = ops.resize_bilinear(image, h, w, 1.0, 1.0, flip_h=fh, flip_w=fw)
            p = self._run_model_single(flipped, flip_h=fh, flip_w=fw)
            done += 1
            ops.accumulate(acc, p, 2 if done == views else 1, views)
        for s in TTA_SCALES:
            hs, ws = int(math.floor(h * s)), int(math.floor(w * s))
            scaled = ops.resize_bilinear(image, hs, ws, 1.0 / s, 1.0 / s)
            ps = self._run_model_single(scaled)
            p = ops.resize_bilinear(ps, h, w)
            done += 1
            ops.accumulate(acc, p, 2 if done == views else 1, views)
        return acc

    # ---- train_eval.py:455-568 -------------------------------------------------
    def _convert_probs_to_mask(self, probs: torch.Tensor, h_pad: int = 0, w_pad: int = 0,
                               h_orig: int = None, w_orig: int = None) -> np.ndarray:
        probs = probs.to(self.device)
        mask = ops.probs_to_mask(probs)
        if h_pad > 0 or w_pad > 0:
            mask = mask[:h_orig, :w_orig]
        return mask.cpu().numpy()

    def predict_semantic_mask(self, image: torch.Tensor) -> np.ndarray:
        self.model.eval()
        with torch.no_grad():
            x = self._prepare_image_tensor(image)
            if self.model_name == "enhanced_unet":
                return self._convert_probs_to_mask(self._run_tta_inference(x))
            return self._convert_probs_to_mask(self._run_model_single(x))

    def evaluate_semantic(self, dataloader) -> Dict[str, float]:
        """Mean of calculate_semantic_metrics over the images (the semantic rows of evaluate())."""
        acc: Dict[str, list] = {}
        for batch in dataloader:
            for i, item in enumerate(batch["batch_items"]):
                pred = self.predict_semantic_mask(batch["images"][i])
                for k, v in calculate_semantic_metrics(pred, item["semantic_mask"]).items():
                    acc.setdefault(k, []).append(v)
        return {k: float(np.mean(v)) for k, v in acc.items()}
