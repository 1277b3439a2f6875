"""CPU-side checks: the C-ABI library loads and exports every declared symbol, the
host layer mirrors the reference API, and the product fails loudly without a GPU."""
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "eunet.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\*|int)\s+(eunet_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    from eunet import _lib
    lib = _lib.load()
    declared = _declared_symbols()
    assert len(declared) >= 30
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib.exported_symbols())
    assert "gfx950" in _lib.version()


def test_state_dict_schema_matches_reference():
    from eunet.models import EnhancedUNet, get_model
    from oracle.eunet_ref import state_spec
    m = get_model("enhanced_unet", num_classes=3)
    keys = list(m.state_dict().keys())
    assert keys == [k for k, _, _ in state_spec(64, 3, 3)]
    assert len(keys) == 109
    assert sum(p.numel() for p in m.parameters()) == 7790790
    m2 = EnhancedUNet(num_classes=2, in_channels=1, base_ch=64)
    assert sum(p.numel() for p in m2.parameters()) == 7788932
    with pytest.raises(ValueError):
        get_model("segnet")


def test_product_path_fails_loudly_on_cpu():
    from eunet import EunetError
    from eunet.models import EnhancedUNet
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
    with pytest.raises(EunetError):
        m(torch.rand(1, 1, 32, 32))


def test_trainer_hyperparameters_and_schedule():
    from eunet.models import EnhancedUNet
    from eunet.train_eval import Trainer
    from oracle.eunet_ref import lr_trajectory
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
    tr = Trainer(m, "cpu", "enhanced_unet", total_epochs=50)
    g = tr.optimizer.param_groups[0]
    assert g["weight_decay"] == 1e-4 and g["betas"] == (0.9, 0.999)
    assert tr.warmup_epochs == 5
    lrs = [tr.epoch_lr_step(e) for e in range(50)]
    assert max(abs(a - b) for a, b in zip(lrs, lr_trajectory(50))) < 1e-12


def test_synthetic_tiles_deterministic():
    from eunet import synth
    x1, m1 = synth.batch(2, 64, 64, start_index=3)
    x2, m2 = synth.batch(2, 64, 64, start_index=3)
    assert torch.equal(x1, x2) and torch.equal(m1, m2)
    assert x1.min() >= 0 and x1.max() <= 1 and m1.max() <= 1
    assert (m1 == 1).float().mean() > 0.01


def test_header_declares_reference_citations():
    src = open(os.path.join(ROOT, "include", "eunet.h")).read()
    for cite in ("models.py:219", "models.py:214", "train_eval.py:28-60", "models.py:308-313"):
        assert cite in src, cite


def test_dual_branch_schema_matches_reference():
    """SMP-path EnhancedUNet parameter tree (models.py:253-302): keys and order of the
    reference module with stand-in branches (oracle/dual_ref.dual_state_spec)."""
    from eunet.dp import backward_order
    from eunet.models import EnhancedUNet
    from oracle.dual_ref import dual_state_spec
    m = EnhancedUNet(num_classes=3, dual_branch=True)
    assert list(m.state_dict().keys()) == [k for k, _, _ in dual_state_spec(64, 3, 3)]
    assert sorted(backward_order(m)) == sorted(n for n, _ in m.named_parameters())
    assert m.get_aux_outputs() is None


def test_checkpoint_format_roundtrip_cpu(tmp_path):
    """load_checkpoint reads the reference's best_model.pth dict (and bare state_dicts) with the
    safe loader."""
    from eunet.models import EnhancedUNet
    from eunet.train_eval import load_checkpoint
    a = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
    b = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
    p = tmp_path / "ck.pth"
    torch.save({"epoch": 1, "model_state_dict": a.state_dict(), "best_miou": 0.1, "best_loss": 2.0,
                "history": {"train_loss": [2.0]}}, p)
    load_checkpoint(b, str(p))
    assert all(torch.equal(x, y) for x, y in zip(a.state_dict().values(), b.state_dict().values()))
    torch.save(a.state_dict(), tmp_path / "sd.pth")
    load_checkpoint(b, str(tmp_path / "sd.pth"))
