"""CPU-side checks: the C-ABI library loads and exports every declared symbol, the
host layer mirrors the reference API, and the product fails loudly without a GPU."""
import os
import re

import numpy as np
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


@pytest.mark.parametrize("n,hw,cout,cin,dtype", [
    (4, 256, 256, 768, "bf16"), (4, 512, 128, 384, "bf16"), (4, 1024, 64, 192, "bf16"),
    (4, 128, 512, 512, "bf16"), (4, 1024, 64, 64, "bf16"), (8, 128, 256, 768, "fp32"), (1, 16, 64, 64, "bf16")])
def test_wgrad_split_count_fills_launch_waves(n, hw, cout, cin, dtype):
    """Host-only: the weight-gradient split count (eunet_conv3x3_wgrad_splits) leaves no nearly
    empty last wave of 512 blocks (the decoder concat layers had 528 / 516 / 513 blocks), covers
    every tile, and keeps the fp32 partials <= 256 MiB."""
    import ctypes
    from eunet import _lib
    lib = _lib.load()
    dtc = _lib.EUNET_BF16 if dtype == "bf16" else _lib.EUNET_F32
    dy = _lib.Act(0x1000, n, hw, hw, cout, cout, 0, dtc)  # descriptor only: nothing is dereferenced
    s = ctypes.c_int()
    assert lib.eunet_conv3x3_wgrad_splits(ctypes.byref(dy), cin, dtc, ctypes.byref(s)) == 0
    ns = s.value
    bf = dtype == "bf16"
    th, tw, kc = (8, 16, 64) if bf else (4, 32, 32)  # bf16: the double-buffered 8 x 16 tiles (round 6)
    ntiles = n * -(-hw // th) * -(-hw // tw)
    blocks = -(-cout // 64) * -(-cin // kc)
    assert 1 <= ns <= ntiles
    per = -(-ntiles // ns)
    assert -(-ntiles // per) == ns  # every split non-empty
    assert cout * 9 * cin * 4 * ns <= 256 << 20
    total = ns * blocks
    if total >= 512:  # the last wave is at least 90 % full
        waves = -(-total // 512)
        assert total / (waves * 512) >= 0.9, (ns, blocks, total)


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
    weights-only loader.  The reference stores best_miou and history values as np.float64
    (Evaluator.evaluate returns np.mean results, train_eval.py:1017)."""
    import numpy as np
    from eunet.models import EnhancedUNet
    from eunet.train_eval import load_checkpoint
    a = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
    b = EnhancedUNet(num_classes=2, in_channels=1, base_ch=16)
    p = tmp_path / "ck.pth"
    torch.save({"epoch": 1, "model_state_dict": a.state_dict(), "best_miou": np.float64(0.5),
                "best_loss": np.float64(2.0),
                "history": {"train_loss": [2.0], "val_miou": [np.float64(0.5)],
                            "val_dice": [[np.float64(0.1), np.float64(0.2)]]}}, p)
    ck = load_checkpoint(b, str(p))
    assert ck["best_miou"] == 0.5 and ck["history"]["val_dice"][0][1] == 0.2
    assert all(torch.equal(x, y) for x, y in zip(a.state_dict().values(), b.state_dict().values()))
    torch.save(a.state_dict(), tmp_path / "sd.pth")
    load_checkpoint(b, str(tmp_path / "sd.pth"))


def test_reference_loss_api_surface():
    """train_eval.FocalLoss(alpha, gamma, ignore_index, class_weights) constructs like the
    reference's (train_eval.py:28-35); Trainer carries focal_loss / ce_loss (:79-80) and the
    loss methods with the reference signatures (:134, :159, :183)."""
    import inspect
    from eunet.models import EnhancedUNet
    from eunet.train_eval import CrossEntropyLoss, FocalLoss, Trainer
    fl = FocalLoss(alpha=[1.0, 8.0, 5.0], gamma=5.0, ignore_index=None, class_weights=torch.tensor([1.0, 20.0, 10.0]))
    assert fl.gamma == 5.0 and fl.alpha == [1.0, 8.0, 5.0] and fl.ignore_index is None
    assert FocalLoss().gamma == 2.0 and FocalLoss().alpha is None
    tr = Trainer(EnhancedUNet(num_classes=3, base_ch=16), "cpu", "enhanced_unet")
    assert isinstance(tr.focal_loss, FocalLoss) and isinstance(tr.ce_loss, CrossEntropyLoss)
    assert tr.focal_loss.gamma == 5.0 and tr.focal_loss.class_weights.tolist() == [1.0, 20.0, 10.0]
    assert list(inspect.signature(tr.dice_loss).parameters) == ["pred", "target", "num_classes"]
    assert list(inspect.signature(tr.tversky_loss).parameters) == ["pred", "target", "num_classes", "alpha"]
    p = tr.loss_params()
    assert list(p.ce_weight) == [1.0, 20.0, 10.0] and list(p.alpha) == [1.0, 8.0, 5.0] and p.gamma == 5.0
    assert (p.w_focal, p.w_dice, p.w_tversky, p.class_div) == (2.5, 2.5, 1.0, 3.0)
    tr.focal_loss.gamma = 3.0  # _compute_combined_loss reads the module's attributes each call
    assert tr.loss_params().gamma == 3.0
    # class_weights' host copy is cached per tensor version (no device sync per step), so an in-place
    # change or a new tensor is still seen
    tr.focal_loss.class_weights.mul_(2.0)
    assert list(tr.loss_params().ce_weight) == [2.0, 40.0, 20.0]
    tr.focal_loss.class_weights = torch.tensor([3.0, 1.0, 1.0])
    assert list(tr.loss_params().ce_weight) == [3.0, 1.0, 1.0]
    with pytest.raises(ValueError):
        FocalLoss(alpha=[1.0, 2.0, 3.0, 4.0]).params()


def test_train_model_builds_reference_loaders(tmp_path):
    """train_model without loaders builds CellDataset train / val loaders from data_dir
    (train_eval.py:1054-1075); zero epochs keeps it on the CPU."""
    import json
    from eunet import data as D
    from eunet.train_eval import train_model
    for i in range(10):
        (tmp_path / f"im{i}.jpg").write_bytes(b"")
        (tmp_path / f"im{i}.json").write_text(json.dumps({"shapes": []}))
    built = []
    orig = D.CellDataset.__init__

    def spy(self, *a, **k):
        orig(self, *a, **k)
        built.append((self.split, self.max_size, len(self)))

    D.CellDataset.__init__ = spy
    try:
        train_model("enhanced_unet", data_dir=str(tmp_path), device="cpu", num_epochs=0,
                    save_dir=str(tmp_path / "ck"), verbose=False, base_ch=16)
    finally:
        D.CellDataset.__init__ = orig
    assert built == [("train", 640, 7), ("val", 640, 1)]


def test_loader_shuffle_matches_torch_random_sampler():
    """eunet.data.DataLoader draws from torch's global generator as torch's DataLoader +
    RandomSampler do (the reference's loaders, train_eval.py:1071-1075): the same permutation
    under the same torch seed, the global stream left at the same position, and Python's
    `random` stream -- the one the augmentations draw from -- untouched."""
    import random

    import torch.utils.data as tud

    from eunet.data import DataLoader

    class _Items:
        def __len__(self):
            return 23

        def __getitem__(self, i):
            return i

    def ident(b):
        return b

    for shuffle in (True, False):
        random.seed(5)
        state = random.getstate()
        torch.manual_seed(77)
        ours = [i for b in DataLoader(_Items(), batch_size=4, shuffle=shuffle, collate_fn=ident) for i in b]
        ours_next = torch.rand(1).item()
        assert random.getstate() == state
        torch.manual_seed(77)
        ref = [i for b in tud.DataLoader(_Items(), batch_size=4, shuffle=shuffle, collate_fn=ident) for i in b]
        assert ours == ref and sorted(ours) == list(range(23))
        assert ours_next == torch.rand(1).item()


def test_network_ops_registered_with_the_dispatcher():
    """The network's device ops are torch.ops.eunet.* (SURVEY.md §8b): one schema per C-ABI entry point, the
    written arguments alias-annotated, CPU tensors rejected (no CPU fallback) through the dispatcher too."""
    from eunet import EunetError, ops
    expect = {"conv3x3_fwd", "conv3x3_dgrad", "conv3x3_dgrad_bnbwd", "conv3x3_dgrad_fused", "conv3x3_wgrad",
              "wgrad_reduce", "conv_small_fwd", "conv_small_wgrad", "bn_finalize", "bnrelu_pool", "bnrelu_upsample",
              "bnrelu_conv1x1", "head_fwd", "head_bwd", "bn_bwd_apply", "bn_bwd_coef", "bn_bwd_apply_coef",
              "pool_bwd_add_bnr", "upsample_bwd_bnr", "conv1x1_bwd_bnr", "bn_bwd_apply_1x1", "bn_bwd_apply_pool",
              "colsum", "conv3x3_pack"}
    assert expect <= set(ops.DISPATCHED)
    sch = str(torch.ops.eunet.conv3x3_fwd.default._schema)
    assert sch.startswith("eunet::conv3x3_fwd(Tensor x, int x_coff, int x_c, Tensor wp, Tensor(a!) y,"), sch
    assert "Tensor(b!)? stats" in sch
    assert str(torch.ops.eunet.conv3x3_pack.default._schema).endswith("-> Tensor")
    with pytest.raises(EunetError):
        torch.ops.eunet.bn_bwd_coef(*[torch.zeros(4)] * 6, 16, torch.zeros(16))


def test_opt_table_layout_and_supported():
    """eunet_opt_table (host code of the native clip + AdamW step): one 7-column row per parameter
    (pointers, numel, first block of 2048 elements), the launch's block count; optim.supported
    accepts only a one-group AdamW of fp32 CUDA tensors (CPU parameters keep torch's step)."""
    import ctypes
    from eunet import _lib, optim
    ns = [1, 2048, 2049, 70001]
    rows = [(0x1000 * (k + 1), 0x2000 * (k + 1), 0x3000 * (k + 1), 0x4000 * (k + 1), 0x5000 * (k + 1), n)
            for k, n in enumerate(ns)]
    descs = (_lib.OptTensor * len(rows))(*[_lib.OptTensor(*r) for r in rows])
    table = (ctypes.c_int64 * (7 * len(rows)))()
    nb = ctypes.c_int()
    _lib.call("eunet_opt_table", ctypes.cast(descs, ctypes.c_void_p), len(rows), ctypes.cast(table, ctypes.c_void_p),
              ctypes.byref(nb))
    b0 = 0
    for k, r in enumerate(rows):
        assert list(table[7 * k:7 * k + 6]) == list(r)
        assert table[7 * k + 6] == b0
        b0 += -(-r[5] // 2048)
    assert nb.value == b0 == 1 + 1 + 2 + 35
    p = torch.nn.Parameter(torch.zeros(3))
    assert not optim.supported(torch.optim.AdamW([p]))  # CPU parameter
    assert not optim.supported(torch.optim.SGD([p], lr=0.1))


def test_upsample_index_closed_forms_equal_the_float_rule():
    """The head kernels' integer x2 source indices (common.h up2_src_i) and closed-form adjoint weights
    (up2_adj_w4) restated and checked against up2_src / up2_adj_w's float rule (PyTorch's
    area_pixel_compute_source_index at scale 1/2, align_corners=False; models.py:236's upsample) for every
    high-res position of every size up to 70, fp32 arithmetic as on the device."""
    f32 = np.float32

    def src_float(o, n):
        s = f32(0.5) * (f32(o) + f32(0.5)) - f32(0.5)
        s = max(s, f32(0.0))
        i0 = int(s)
        return i0, i0 + (1 if i0 < n - 1 else 0), f32(s - f32(i0))

    def src_int(o, n):
        m, odd = o >> 1, (o & 1) == 1
        i0 = m if odd else max(m - 1, 0)
        return i0, min(i0 + 1, n - 1), f32(0.25 if odd else (0.0 if o == 0 else 0.75))

    def adj_w(o, n, i):
        i0, i1, l1 = src_float(o, n)
        return (f32(1.0) - l1 if i0 == i else f32(0.0)) + (l1 if i1 == i else f32(0.0))

    def adj_w4(i, n):
        w = [0.25, 0.75, 0.75, 0.25]
        if i == 0:
            w[0], w[1] = 0.0, 1.0
        if i == n - 1:
            w[2], w[3] = 1.0, 0.0
        return [f32(v) for v in w]

    for n in range(1, 71):
        for o in range(2 * n):
            assert src_int(o, n) == src_float(o, n), (n, o)
        for i in range(n):
            w4 = adj_w4(i, n)
            for d in range(4):
                o = 2 * i - 1 + d
                ref = adj_w(o, n, i) if 0 <= o < 2 * n else f32(0.0)
                assert w4[d] == ref, (n, i, d)
