"""Drop-in model surface of reference models.py for the Enhanced-UNet path.

Same names, signatures and state_dict schema as the reference (SMP-absent
build, which is what the reference selects when segmentation_models_pytorch
is not importable, models.py:71-76, 304-314):

    get_model(model_name, num_classes=3, device='cuda', train_mode=False,
              data_dir=None, max_size=640)                    # models.py:590-624
    EnhancedUNet(num_classes=3).forward(x) -> [B,K,2H,2W]     # models.py:246-343
    EnhancedUNet.get_aux_outputs() -> None                    # models.py:341-343
    state_dict keys: model.enc1.0.weight ... enhance.3.bias   # 109 keys (c3, K3)

Build-side keyword-only generalisations (BASELINE configs): in_channels,
base_ch, dtype ('fp32' | 'bf16' compute/storage of activations; parameters,
BN statistics and the loss stay fp32).

The nn layers below are parameter containers only (their initialisation and
state_dict naming match the reference); forward never runs them -- it runs the
HIP engine (engine.py).  There is no CPU path: forward on a CPU tensor raises.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .dual import DualEngine, DualFunction, dual_backward_order
from .engine import UNetEngine, UNetFunction

_DTYPES = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}


def _double_conv(cin: int, cout: int) -> nn.Sequential:
    # indices 0..5 = Conv, BN, ReLU, Conv, BN, ReLU (models.py:217-225 key layout)
    return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
                         nn.Conv2d(cout, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class _UNetParams(nn.Module):
    """Parameter tree of BasicUNet (models.py:199-215)."""

    def __init__(self, in_channels: int, base_ch: int, num_classes: int):
        super().__init__()
        b = base_ch
        self.enc1 = _double_conv(in_channels, b)
        self.enc2 = _double_conv(b, 2 * b)
        self.enc3 = _double_conv(2 * b, 4 * b)
        self.enc4 = _double_conv(4 * b, 8 * b)
        self.dec4 = _double_conv(8 * b + 4 * b, 4 * b)
        self.dec3 = _double_conv(4 * b + 2 * b, 2 * b)
        self.dec2 = _double_conv(2 * b + b, b)
        self.dec1 = nn.Conv2d(b, num_classes, 1)


class UNet(nn.Module):
    """Reference UNet wrapper (models.py:175-243), SMP-absent: holds BasicUNet as .model."""

    def __init__(self, num_classes: int = 3, *, in_channels: int = 3, base_ch: int = 64):
        super().__init__()
        self.num_classes = num_classes
        self.model = _UNetParams(in_channels, base_ch, num_classes)


class EnhancedUNet(nn.Module):
    """Enhanced U-Net (reference fallback definition) on the MI355X engine."""

    def __init__(self, num_classes: int = 3, *, in_channels: int = 3, base_ch: int = 64, dtype: str = "fp32",
                 dual_branch: bool = False):
        super().__init__()
        if not 1 <= num_classes <= 3:
            raise ValueError("num_classes must be 1..3 (the reference loss tables have 3 classes)")
        if in_channels > 4:
            raise ValueError("in_channels must be <= 4")
        if base_ch % 16:
            raise ValueError("base_ch must be a multiple of 16")
        self.num_classes = num_classes
        self.in_channels = in_channels
        self.base_ch = base_ch
        self.compute_dtype = _DTYPES[dtype]
        self.dual_branch = dual_branch
        self._aux_outputs = None
        self.grad_sink_factory = None  # set by eunet.dp for bucketed all-reduce overlap
        if dual_branch:  # the reference's SMP path (models.py:253-302), build-defined branches
            k2 = 2 * num_classes
            self.unetpp = _UNetParams(in_channels, base_ch, num_classes)
            self.deeplab = _UNetParams(in_channels, base_ch, num_classes)
            self.attention_gate = nn.Sequential(
                nn.Conv2d(k2, k2 // 2, 3, padding=1, bias=False), nn.BatchNorm2d(k2 // 2), nn.GELU(),
                nn.Conv2d(k2 // 2, k2, 1, bias=False), nn.BatchNorm2d(k2), nn.Sigmoid())
            self.fusion_head = nn.Sequential(
                nn.Conv2d(k2, 256, 3, padding=1, bias=False), nn.BatchNorm2d(256), nn.ReLU(inplace=True),
                nn.Dropout2d(0.2),
                nn.Conv2d(256, 128, 3, padding=1, bias=False), nn.BatchNorm2d(128), nn.ReLU(inplace=True),
                nn.Dropout2d(0.15),
                nn.Conv2d(128, 64, 3, padding=1, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                nn.Conv2d(64, num_classes, 1))
            self.fusion_residual = nn.Conv2d(k2, num_classes, 1)
            self._engine = DualEngine(self)
        else:  # SMP-absent fallback (models.py:304-314)
            self.model = UNet(num_classes, in_channels=in_channels, base_ch=base_ch).model
            self.enhance = nn.Sequential(nn.Conv2d(num_classes, 64, 3, padding=1), nn.BatchNorm2d(64),
                                         nn.ReLU(inplace=True), nn.Conv2d(64, num_classes, 1))
            self._engine = UNetEngine(self)

    def set_dtype(self, dtype: str):
        self.compute_dtype = _DTYPES[dtype]
        self._engine.dtype = self.compute_dtype
        return self

    def backward_param_order(self):
        """Parameter names in gradient-production order (eunet.dp buckets)."""
        return dual_backward_order(self) if self.dual_branch else None

    def _run_dual(self, x: torch.Tensor) -> torch.Tensor:
        """models.py:317-333: fused logits [B,K,H,W]; _aux_outputs = branch logits."""
        if self.training and torch.is_grad_enabled():
            out, aux_a, aux_b = DualFunction.apply(x, self._engine, self.grad_sink_factory,
                                                   *[p for _, p in self.named_parameters()])
        else:
            with torch.no_grad():
                out, aux_a, aux_b, _ = self._engine.forward(x, training=self.training)
        self._aux_outputs = {"unetpp": aux_a, "deeplab": aux_b}
        return out

    def _run(self, x: torch.Tensor, want: str) -> torch.Tensor:
        if self.dual_branch:
            return self._run_dual(x)
        self._aux_outputs = None
        if self.training:
            if torch.is_grad_enabled():
                return UNetFunction.apply(x, want, self._engine, self.grad_sink_factory,
                                          *[p for _, p in self.named_parameters()])
            with torch.no_grad():
                return self._engine.forward(x, training=True, want=want)[0]
        with torch.no_grad():
            return self._engine.forward(x, training=False, want=want)[0]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x [B,C,H,W] -> logits [B,K,2H,2W] (models.py:316-339, fallback branch)."""
        return self._run(x, "out2h")

    def forward_lowres(self, x: torch.Tensor) -> torch.Tensor:
        """Fused forward + the training loop's 2H->H bilinear resize (train_eval.py:306-310,
        an exact 2x2 mean): logits [B,K,H,W] without materialising the 2H output."""
        return self._run(x, "logits")

    def get_aux_outputs(self):
        return getattr(self, "_aux_outputs", None)


def get_model(model_name: str, num_classes: int = 3, device: str = "cuda", train_mode: bool = False,
              data_dir: str = None, max_size: int = 640, **kwargs):
    """models.py:590-624.  Only the Enhanced-UNet hot path is built here; the other
    reference nets are out of scope and raise like unknown names."""
    if model_name == "enhanced_unet":
        return EnhancedUNet(num_classes=num_classes, **kwargs)
    if model_name == "unet":
        raise ValueError("unet (SMP resnet50 / BasicUNet) is out of scope of this build; use 'enhanced_unet'")
    raise ValueError(f"Unknown model: {model_name}")
