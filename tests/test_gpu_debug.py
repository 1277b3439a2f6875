"""The bounds-checked debug build (libeunet_hip_debug.so, -DEUNET_DEBUG), run once:
in a child process whose EUNET_LIB points at it, a deliberately failing device check is reported
(unit and line), and then full training steps of the single- and dual-branch models (bf16 and
fp32, ragged tile edges, multi-split weight gradients, the fused BN-backward staging) trip none of
the device-side checks on staging offsets, tile / split indices and output addresses."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, torch
sys.path[:0] = [ROOT, ROOT + "/enhanced-unet_amd"]
from eunet import _lib, synth
from eunet.losses import combined_loss
from eunet.models import EnhancedUNet
from eunet.train_eval import Trainer
lib = _lib.load()
assert lib.eunet_debug_enabled() == 1, "not the debug build"
_lib.call("eunet_debug_selftest", None)
line, cnt = _lib.debug_status(reset=True)
assert cnt > 0 and line // 100000 == 1, (line, cnt)
print("selftest reported", line, cnt)
assert _lib.debug_status() == (0, 0)
for dtype, base, size, dual in (("bf16", 16, 72, False), ("fp32", 16, 40, False), ("bf16", 64, 128, False),
                                ("bf16", 16, 64, True), ("fp32", 16, 48, True)):
    torch.manual_seed(0)
    m = EnhancedUNet(num_classes=2, in_channels=1, base_ch=base, dtype=dtype, dual_branch=dual).cuda()
    tr = Trainer(m, "cuda", "enhanced_unet")
    x, msk = synth.batch(2, size, size + 16, start_index=3, num_classes=2, in_channels=1, device="cuda")
    tr.step(x, msk)
    tr.step(x, msk)
    st = _lib.debug_status()
    print(dtype, base, size, dual, "debug status", st)
    assert st == (0, 0), (dtype, base, size, dual, st)
print("DEBUG_OK")
'''


@pytest.mark.timeout(600)
def test_debug_build_checks_pass_on_training_steps():
    lib = os.path.join(ROOT, "enhanced-unet_amd", "eunet", "libeunet_hip_debug.so")
    assert os.path.exists(lib), "build it: make -C enhanced-unet_amd debug"
    env = dict(os.environ, EUNET_LIB=lib)
    r = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], env=env, capture_output=True,
                       text=True, timeout=500)
    print(r.stdout[-3000:], r.stderr[-3000:])
    assert r.returncode == 0 and "DEBUG_OK" in r.stdout
