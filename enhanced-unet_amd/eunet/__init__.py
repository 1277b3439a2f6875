"""eunet -- MI355X-native Enhanced-UNet training hot path.

Drop-in modules mirroring the reference (whh1747012859/Enhanced-UNet):
    eunet.models      <-> models.py      (get_model, EnhancedUNet, UNet)
    eunet.train_eval  <-> train_eval.py  (Trainer, FocalLoss)
Kernels: libeunet_hip.so (HIP, gfx950) through the C-ABI in include/eunet.h.
"""
from ._lib import EunetError, load as load_library, version  # noqa: F401

__all__ = ["EunetError", "load_library", "version"]
