"""CPU restatement of the reference dual-branch Enhanced-UNet (TEST INFRASTRUCTURE).

Used only by tests/ (and never by the product path) as the checker.

Restated (citations into /root/reference):
  * EnhancedUNet SMP path   models.py:253-302 (attention gate, fusion head, residual),
                            models.py:316-333 (forward, _aux_outputs)
  * aux supervision         train_eval.py:199-234 (branch losses x {unetpp 0.6, deeplab 0.5},
                            consistency 0.4 * MSE(softmax(branch), softmax(fused)), :86-87)
  * per-sample loop         train_eval.py:262-337 (fused loss + aux loss per sample, / B)

The two SMP backbones (UnetPlusPlus / efficientnet-b5, DeepLabV3Plus /
efficientnet-b4) are third-party (segmentation_models_pytorch >= 0.3.0,
requirements.txt:10), un-vendored and need pretrained ImageNet weights: they
cannot run here.  The build defines both branches as BasicUNet trunks
(models.py:199-238) that end at input resolution -- dec1 applied to d2 without
the final upsample, i.e. what an SMP decoder's segmentation head returns --
and everything the reference itself owns (gate, fusion head, residual, aux
outputs, deep supervision, consistency) is restated exactly.
tests/golden/dual_c3k3.npz pins it: the reference module built with a stand-in
`segmentation_models_pytorch` whose two classes return such trunks
(tests/golden/gen_golden.py gen_dual).  Parity of the real SMP backbones: unpinned.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F

from . import eunet_ref as R

BRANCHES = ("unetpp", "deeplab")
AUX_WEIGHTS = {"unetpp": 0.6, "deeplab": 0.5}   # train_eval.py:86
CONSISTENCY = 0.4                                # train_eval.py:87
DROP_P = (0.2, 0.15)                             # models.py:287, 291
FUSION = (256, 128, 64)                          # models.py:285-293


def dual_state_spec(base: int = 64, in_ch: int = 3, K: int = 3):
    spec = []
    trunk = [(k[len("model."):], s, f) for k, s, f in R.state_spec(base, in_ch, K) if k.startswith("model.")]
    for br in BRANCHES:
        spec += [(f"{br}.{k}", s, f) for k, s, f in trunk]

    def bn(prefix, c):
        spec.extend([(f"{prefix}.weight", (c,), None), (f"{prefix}.bias", (c,), None),
                     (f"{prefix}.running_mean", (c,), None), (f"{prefix}.running_var", (c,), None),
                     (f"{prefix}.num_batches_tracked", (), None)])

    c2 = 2 * K
    spec.append(("attention_gate.0.weight", (c2 // 2, c2, 3, 3), c2 * 9))
    bn("attention_gate.1", c2 // 2)
    spec.append(("attention_gate.3.weight", (c2, c2 // 2, 1, 1), c2 // 2))
    bn("attention_gate.4", c2)
    cin = c2
    for i, co in zip((0, 4, 8), FUSION):
        spec.append((f"fusion_head.{i}.weight", (co, cin, 3, 3), cin * 9))
        bn(f"fusion_head.{i + 1}", co)
        cin = co
    spec.append(("fusion_head.11.weight", (K, FUSION[-1], 1, 1), FUSION[-1]))
    spec.append(("fusion_head.11.bias", (K,), FUSION[-1]))
    spec.append(("fusion_residual.weight", (K, c2, 1, 1), c2))
    spec.append(("fusion_residual.bias", (K,), c2))
    return spec


def dual_formula_weights(base=64, in_ch=3, K=3, dtype=torch.float64) -> Dict[str, torch.Tensor]:
    import numpy as np
    from .weights import formula_state_dict
    out = {}
    for k, v in formula_state_dict(dual_state_spec(base, in_ch, K)).items():
        out[k] = torch.tensor(0, dtype=torch.long) if k.endswith("num_batches_tracked") else \
            torch.from_numpy(np.asarray(v)).to(dtype)
    return out


def branch_forward(S, prefix: str, x, training: bool, pins=None, record=None):
    """BasicUNet trunk (models.py:227-237) ending at input resolution: dec1(d2).  pins: the trunk's
    branch configuration (eunet_ref.trunk); record: optional dict of its ReLU inputs."""
    d2, _ = R.trunk(S, x, training, pins, prefix=prefix + ".", record=record)
    return F.conv2d(d2, S[prefix + ".dec1.weight"], S[prefix + ".dec1.bias"])


def _drop(h, mask, p, training):
    if not training:
        return h
    if mask is None:
        return F.dropout2d(h, p, True)
    return h * mask.to(h.dtype)[:, :, None, None] / (1.0 - p)


def dual_forward(S, x, training: bool = True, drop_masks=None, pins=None, record=None):
    """x [B,C,H,W] -> (fused [B,K,H,W], {'unetpp': .., 'deeplab': ..}); models.py:316-333.
    drop_masks: optional ([B,256], [B,128]) 0/1 keep masks for the two Dropout2d.
    pins: optional branch configuration {'unetpp': trunk pins, 'deeplab': trunk pins,
    'fusion_head.1' / '.5' / '.9': ReLU masks} (eunet_ref._relu).
    record: optional dict receiving the ReLU inputs in the same layout as pins (tests/_pins.py audit)."""
    pins = pins or {}
    rec = (lambda k, h: record.__setitem__(k, h.detach())) if record is not None else (lambda k, h: None)
    if record is not None:
        record["unetpp"], record["deeplab"] = {}, {}
    out_main = branch_forward(S, "unetpp", x, training, pins.get("unetpp"),
                              record["unetpp"] if record is not None else None)
    out_aux = branch_forward(S, "deeplab", x, training, pins.get("deeplab"),
                             record["deeplab"] if record is not None else None)
    ff = torch.cat([out_main, out_aux], 1)
    a = F.conv2d(ff, S["attention_gate.0.weight"], padding=1)
    a = F.gelu(R._bn(S, "attention_gate.1", a, training))
    a = F.conv2d(a, S["attention_gate.3.weight"])
    att = torch.sigmoid(R._bn(S, "attention_gate.4", a, training))
    ff = ff * att
    dm = drop_masks or (None, None)
    h = R._bn(S, "fusion_head.1", F.conv2d(ff, S["fusion_head.0.weight"], padding=1), training)
    rec("fusion_head.1", h)
    h = _drop(R._relu(h, pins.get("fusion_head.1")), dm[0], DROP_P[0], training)
    h = R._bn(S, "fusion_head.5", F.conv2d(h, S["fusion_head.4.weight"], padding=1), training)
    rec("fusion_head.5", h)
    h = _drop(R._relu(h, pins.get("fusion_head.5")), dm[1], DROP_P[1], training)
    h = R._bn(S, "fusion_head.9", F.conv2d(h, S["fusion_head.8.weight"], padding=1), training)
    rec("fusion_head.9", h)
    h = R._relu(h, pins.get("fusion_head.9"))
    fused = F.conv2d(h, S["fusion_head.11.weight"], S["fusion_head.11.bias"])
    fused = fused + F.conv2d(ff, S["fusion_residual.weight"], S["fusion_residual.bias"])
    return fused, {"unetpp": out_main, "deeplab": out_aux}


def aux_supervision(aux, i: int, target, fused_logits):
    """train_eval.py:199-234 for sample i (branch logits already at mask size)."""
    total = torch.zeros((), dtype=fused_logits.dtype)
    fused_probs = F.softmax(fused_logits.unsqueeze(0), dim=1)
    for name, w in AUX_WEIGHTS.items():
        bl = aux[name][i]
        total = total + w * R.combined_loss(bl, target)
        bp = F.softmax(bl.unsqueeze(0), dim=1)
        total = total + w * CONSISTENCY * F.mse_loss(bp, fused_probs)
    return total


def dual_batch_loss(fused, aux, target):
    B = fused.shape[0]
    loss = 0.0
    for i in range(B):
        loss = loss + R.combined_loss(fused[i], target[i])
        loss = loss + aux_supervision(aux, i, target[i], fused[i])
    return loss / B


class DualOracleTrainer(R.OracleTrainer):
    def __init__(self, S, total_epochs: int = 50, lr: float = 4e-3, drop_masks=None):
        super().__init__(S, total_epochs, lr)
        self.drop_masks = drop_masks

    def step(self, images, masks, clip: bool = True):
        self.optimizer.zero_grad()
        fused, aux = dual_forward(self.S, images, training=True, drop_masks=self.drop_masks)
        loss = dual_batch_loss(fused, aux, masks)
        loss.backward()
        if clip:
            torch.nn.utils.clip_grad_norm_(self.params, max_norm=1.0)
        self.optimizer.step()
        return float(loss.item())


def dual_flops_per_pixel(base: int, in_ch: int, K: int) -> float:
    """Train FLOP per input pixel: two trunks without the 2H tail + gate + fusion head."""
    b, c = base, in_ch
    trunk_mac = 9 * c * b + 9 * b * b + 0.25 * 9 * (b * 2 * b + 4 * b * b) \
        + (1 / 16) * 9 * (2 * b * 4 * b + 16 * b * b) + (1 / 64) * 9 * (4 * b * 8 * b + 64 * b * b) \
        + (1 / 16) * 9 * (12 * b * 4 * b + 16 * b * b) + 0.25 * 9 * (6 * b * 2 * b + 4 * b * b) \
        + 9 * (3 * b * b + b * b) + b * K
    gate = 9 * 2 * K * K + K * 2 * K
    head = 9 * (2 * K * 256 + 256 * 128 + 128 * 64) + 64 * K + 2 * K * K
    return 6.0 * (2 * trunk_mac + gate + head)
